"""Packet-level known-answer tests of the reference, restated as data.

Wire bytes: tests/golden/kats_packets.json, extracted from the reference's own
test sources by tests/golden/make_kats_packets.py (key "file:function:var").
Expected results: transcribed by hand from the Rust assertions next to each
array, written in the reference's serde JSON form (the shape
`serde_json::to_string` gives the Rust value, pinned for every shape used here
by the golden pcap fixtures).  Each case cites the test it restates.

A case is a list of template maps ("peers"); each map is a sequence of steps
    (kind, wire, expect)
  kind    "ipfix" = IpfixPacket::parse, "nf9" = NetFlowV9Packet::parse,
          "nf9set" = netflow Set::parse of a lone set (wrapped into a v9
          message for the codec-level device run); "ipfixset" = IPFIX
          Set::parse of a lone set, "tplrec" = TemplateRecord::parse,
          "fspec" = FieldSpecifier::parse, "datarec" = DataRecord::parse with
          the map's one preloaded template (each wrapped into an IPFIX
          message, kat_runner.ipfix_wrap)
  wire    fixture key, or raw bytes
  expect  ("ok", packet_json)    parsed completely, equal to the Rust value
          ("ok?", None)          the test only unwraps Ok (values unpinned)
          ("err", error_json)    the Rust error value, exactly
          ("err?", None)         the test asserts only is_err()
          ("same", step_index)   equal to the result of an earlier step
Optional per-map "preload": templates a test inserts straight into the
TemplatesMap (DecodingTemplate::new) instead of parsing a template set;
"counts": processed_count asserted after the last step.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "kats_packets.json")) as _f:
    WIRES = {k: bytes.fromhex(v["hex"]) for k, v in json.load(_f).items()}


def wire(key):
    return WIRES[key]


# --- serde JSON builders -----------------------------------------------------
def S(el, length):
    """FieldSpecifier {element_id, length}; el: IANA name, or a dict for
    vendor / unknown IEs."""
    return {"element_id": el, "length": length}


def vie(vendor, name):
    return {vendor: name}


def vunk_ie(vendor, id_):
    return {vendor: {"Unknown": {"id": id_}}}


def unk_ie(pen, id_):
    return {"Unknown": {"pen": pen, "id": id_}}


def T(tid, *specs):
    return {"id": tid, "field_specifiers": list(specs)}


def OT(tid, scope, fields):
    return {"id": tid, "scope_field_specifiers": list(scope), "field_specifiers": list(fields)}


def F(name, value):
    return {name: value}


def V(vendor, name, value):
    return {vendor: {name: value}}


def VU(vendor, id_, value):
    return {vendor: {"Unknown": {"id": id_, "value": list(value)}}}


def U(pen, id_, value):
    return {"Unknown": {"pen": pen, "id": id_, "value": list(value)}}


def tcp(fin, syn, rst, psh, ack, urg, ece, cwr):
    """TCPHeaderFlags::new argument order (crates/iana/src/tcp.rs:76-85)."""
    return {"FIN": fin, "SYN": syn, "RST": rst, "PSH": psh, "ACK": ack, "URG": urg, "ECE": ece, "CWR": cwr}


NO_FLAGS = tcp(False, False, False, False, False, False, False, False)


def R(fields, scope=()):
    def conv(xs):
        return [x if isinstance(x, dict) else {x[0]: x[1]} for x in xs]
    return {"scope_fields": conv(scope), "fields": conv(fields)}


def D(tid, *records):
    return {"Data": {"id": tid, "records": list(records)}}


def TS(*recs):
    return {"Template": list(recs)}


def OTS(*recs):
    return {"OptionsTemplate": list(recs)}


def ipfix(export_time, seq, domain, *sets):
    return {"version": 10, "export_time": export_time, "sequence_number": seq,
            "observation_domain_id": domain, "sets": list(sets)}


def nf9(sys_up, unix_time, seq, source_id, *sets):
    return {"version": 9, "sys_up_time": sys_up, "unix_time": unix_time, "sequence_number": seq,
            "source_id": source_id, "sets": list(sets)}


# --- shared templates ---------------------------------------------------------
# ipfix.rs:81-103 (template 307, also test_data_packet :212-236 and the bench's
# IPFIX_PKT_TEMPLATE_RAW)
T307 = [S("sourceIPv4Address", 4), S("destinationIPv4Address", 4), S("ipClassOfService", 1),
        S("protocolIdentifier", 1), S("sourceTransportPort", 2), S("destinationTransportPort", 2),
        S("icmpTypeCodeIPv4", 2), S("ingressInterface", 4), S("bgpSourceAsNumber", 4),
        S("bgpDestinationAsNumber", 4), S("bgpNextHopIPv4Address", 4), S("egressInterface", 4),
        S("octetDeltaCount", 4), S("packetDeltaCount", 4), S("flowStartSysUpTime", 4), S("flowEndSysUpTime", 4),
        S("ipNextHopIPv4Address", 4), S("sourceIPv4PrefixLength", 1), S("destinationIPv4PrefixLength", 1),
        S("tcpControlBits", 1), S("ipVersion", 1), S("flowStartMilliseconds", 8), S("flowEndMilliseconds", 8)]
T307_PKT = ipfix("2016-11-29T20:08:57Z", 3812, 0, TS(T(307, *T307)))

# ipfix.rs:921-945 / netflow.rs:653-677 (IANA sub-registry template 400)
T400_SUBREGS = [S("sourceIPv4Address", 4), S("destinationIPv4Address", 4), S("sourceTransportPort", 2),
                S("destinationTransportPort", 2), S("flowId", 8), S("protocolIdentifier", 1),
                S("octetDeltaCount", 4), S("packetDeltaCount", 4), S("mplsTopLabelType", 1),
                S("forwardingStatus", 4), S("classificationEngineId", 1), S("flowEndReason", 1),
                S("natOriginatingAddressRealm", 1), S("firewallEvent", 1), S("biflowDirection", 1),
                S("observationPointType", 1), S("anonymizationTechnique", 2), S("natType", 1),
                S("valueDistributionMethod", 1), S("flowSelectorAlgorithm", 2), S("dataLinkFrameType", 2),
                S("mibCaptureTimeSemantics", 1), S("natQuotaExceededEvent", 1), S("natThresholdEvent", 1),
                S("srhIPv6ActiveSegmentType", 1)]
# ipfix.rs:959-999 / netflow.rs:692-732
R400_SUBREGS = R([
    ("sourceIPv4Address", "10.100.0.1"), ("destinationIPv4Address", "10.100.0.151"),
    ("sourceTransportPort", 10004), ("destinationTransportPort", 1), ("flowId", 10101010),
    ("protocolIdentifier", "ICMP"), ("octetDeltaCount", 1200), ("packetDeltaCount", 1),
    ("mplsTopLabelType", "Unknown"), ("forwardingStatus", {"Dropped": "Badheaderchecksum"}),
    ("classificationEngineId", "ETHERTYPE"), ("flowEndReason", "lackofresources"),
    ("natOriginatingAddressRealm", {"Unassigned": 15}), ("firewallEvent", "FlowDeleted"),
    ("biflowDirection", "perimeter"), ("observationPointType", "Physicalport"),
    ("anonymizationTechnique", "StructuredPermutation"), ("natType", "NAT66translated"),
    ("valueDistributionMethod", "SimpleUniformDistribution"),
    ("flowSelectorAlgorithm", "UniformprobabilisticSampling"), ("dataLinkFrameType", {"Unassigned": 10}),
    ("mibCaptureTimeSemantics", "average"), ("natQuotaExceededEvent", "Maximumactivehostsorsubscribers"),
    ("natThresholdEvent", "Addresspoolhighthresholdevent"),
    ("srhIPv6ActiveSegmentType", "BGPSegmentRoutingPrefixSID")])

# netflow.rs:49-61 / 89-101 (template 1024)
T1024_NF = [S("sourceIPv4Address", 4), S("destinationIPv4Address", 4), S("flowEndSysUpTime", 4),
            S("flowStartSysUpTime", 4), S("octetDeltaCount", 4), S("packetDeltaCount", 4),
            S("ingressInterface", 4), S("egressInterface", 4), S("sourceTransportPort", 2),
            S("destinationTransportPort", 2), S("protocolIdentifier", 1), S("tcpControlBits", 1),
            S("ipVersion", 1)]

# netflow.rs:227-259 (template 313)
T313_NF = [S("mplsTopLabelStackSection", 3), S("mplsLabelStackSection2", 3), S("mplsLabelStackSection3", 3),
           S("mplsLabelStackSection4", 3), S("mplsLabelStackSection5", 3), S("mplsLabelStackSection6", 3),
           S("ingressInterface", 4), S("egressInterface", 4), S("octetDeltaCount", 4), S("packetDeltaCount", 4),
           S("flowEndSysUpTime", 4), S("flowStartSysUpTime", 4), S("mplsTopLabelIPv4Address", 4),
           S("sourceIPv6Address", 16), S("destinationIPv6Address", 16), S("flowLabelIPv6", 4),
           S("ipv6ExtensionHeaders", 4), S("sourceIPv4Address", 4), S("destinationIPv4Address", 4),
           S("sourceTransportPort", 2), S("destinationTransportPort", 2), S("mplsTopLabelPrefixLength", 1),
           S("mplsTopLabelType", 1), S("forwardingStatus", 1), S("flowDirection", 1), S("ipClassOfService", 1),
           S("protocolIdentifier", 1), S("tcpControlBits", 1), S("samplerId", 2), S("ingressVRFID", 4),
           S("egressVRFID", 4)]


def _r313(start_up, sport):
    # netflow.rs:276-310 / 316-350
    return R([("mplsTopLabelStackSection", [0x05, 0xde, 0x01])] +
             [("mplsLabelStackSection%d" % i, [0, 0, 0]) for i in range(2, 7)] +
             [("ingressInterface", 207), ("egressInterface", 161), ("octetDeltaCount", 128),
              ("packetDeltaCount", 2), ("flowEndSysUpTime", 0x0c09ceb5), ("flowStartSysUpTime", start_up),
              ("mplsTopLabelIPv4Address", "0.0.0.0"), ("sourceIPv6Address", "::"),
              ("destinationIPv6Address", "::"), ("flowLabelIPv6", 0), ("ipv6ExtensionHeaders", 0),
              ("sourceIPv4Address", "213.3.196.34"), ("destinationIPv4Address", "138.187.111.116"),
              ("sourceTransportPort", sport), ("destinationTransportPort", 53),
              ("mplsTopLabelPrefixLength", 0), ("mplsTopLabelType", "Unknown"),
              ("forwardingStatus", {"Forwarded": "Unknown"}), ("flowDirection", "ingress"),
              ("ipClassOfService", 0), ("protocolIdentifier", "TCP"),
              ("tcpControlBits", tcp(False, True, False, False, False, False, False, False)),
              ("samplerId", 1), ("ingressVRFID", 1610612736), ("egressVRFID", 1610612741)])


def _r1024(src, dst, end, start, octets, sport, dport):
    # netflow.rs:118-192
    return R([("sourceIPv4Address", src), ("destinationIPv4Address", dst), ("flowEndSysUpTime", end),
              ("flowStartSysUpTime", start), ("octetDeltaCount", octets), ("packetDeltaCount", 1),
              ("ingressInterface", 0), ("egressInterface", 0), ("sourceTransportPort", sport),
              ("destinationTransportPort", dport), ("protocolIdentifier", "UDP"), ("tcpControlBits", NO_FLAGS),
              ("ipVersion", 4)])


def _r2599(src, dst, octets, up, ingress, egress, dport, hw, flags, flow_label, sampler, ivrf, selector,
           dmac, smac, vlan, prio):
    # ipfix.rs:1237-1296 / 1300-1356
    return R([("sourceIPv6Address", src), ("destinationIPv6Address", dst), ("ipNextHopIPv6Address", "::1"),
              ("packetDeltaCount", 1), ("octetDeltaCount", octets), ("flowStartSysUpTime", up),
              ("flowEndSysUpTime", up), ("systemInitTimeMilliseconds", "2025-08-26T07:02:40Z"),
              ("bgpNextHopIPv6Address", "::"), ("ingressInterface", ingress), ("egressInterface", egress),
              ("bgpSourceAsNumber", 0), ("bgpDestinationAsNumber", 0), ("sourceTransportPort", 179),
              ("destinationTransportPort", dport), ("vlanId", 0), ("postVlanId", 0),
              VU("Huawei", 232, hw), ("tcpControlBits", flags), ("protocolIdentifier", "TCP"),
              ("ipClassOfService", 192), ("sourceIPv6PrefixLength", 128), ("destinationIPv6PrefixLength", 128),
              ("flowDirection", "ingress"), ("forwardingStatus", {"Unknown": {"Unassigned": 0}}),
              ("flowLabelIPv6", flow_label), ("flowEndReason", "idletimeout"), ("paddingOctets", [0, 0, 0]),
              ("samplerId", sampler), ("ingressVRFID", ivrf), ("egressVRFID", 0), ("selectorId", selector),
              ("ipv6ExtensionHeadersFull", [0] * 32), ("destinationMacAddress", dmac),
              ("sourceMacAddress", smac), ("dot1qVlanId", vlan), ("dot1qCustomerVlanId", 0),
              ("dot1qPriority", prio), ("dot1qCustomerPriority", 0), ("paddingOctets", [0, 0]),
              ("srhTagIPv6", 0), ("srhFlagsIPv6", 0), ("srhSegmentsIPv6Left", 0),
              ("srhActiveSegmentIPv6", "::"), ("srhIPv6ActiveSegmentType", "Unknown"),
              ("paddingOctets", [0, 0]), ("srhSegmentIPv6ListSection", [])])


_APP = [(0x50, "2426945984", "4285581510"), (0x51, "877825990", "1742571168"), (0x52, "3318228306", "3693899980"),
        (0x53, "3345427587", "3062462844"), (0x54, "247430229", "1508192498"), (0x55, "496746293", "3398434384"),
        (0x56, "2764408791", "2466434107"), (0x57, "2600679433", "1670804265"), (0x58, "2533647043", "888036656"),
        (0x59, "1342289478", "3856588635")]  # ipfix.rs:1616-1685

W = "ipfix.rs:"
M = "mod.rs:"
N = "netflow.rs:"
B = "serde_benchmark.rs:<top>:"

CASES = {
    # ipfix.rs:29-134 test_ipfix_header (one map across the three parses)
    "ipfix_header": [{"steps": [
        ("ipfix", W + "test_ipfix_header:good_wire", ("ok", T307_PKT)),
        ("ipfix", W + "test_ipfix_header:bad_version_wire",
         ("err", {"UnsupportedVersion": {"offset": 0, "version": 0}})),
        ("ipfix", W + "test_ipfix_header:bad_length_wire", ("err", {"InvalidLength": {"offset": 2, "length": 0}})),
    ]}],
    # ipfix.rs:136-193
    "ipfix_template_packet": [{"steps": [("ipfix", W + "test_template_packet:good_wire", ("ok", T307_PKT))]}],
    # ipfix.rs:195-292 (template 307 inserted into the map; processed_count 1 after)
    "ipfix_data_packet": [{"preload": {307: ([], T307)}, "counts": {307: 1}, "steps": [
        ("ipfix", W + "test_data_packet:good_wire", ("ok", ipfix("2016-11-29T20:08:57Z", 3812, 0, D(307, R([
            ("sourceIPv4Address", "70.1.115.1"), ("destinationIPv4Address", "50.0.71.1"), ("ipClassOfService", 0),
            ("protocolIdentifier", "anyhostinternalprotocol"), ("sourceTransportPort", 0),
            ("destinationTransportPort", 0), ("icmpTypeCodeIPv4", 0), ("ingressInterface", 827),
            ("bgpSourceAsNumber", 2), ("bgpDestinationAsNumber", 3), ("bgpNextHopIPv4Address", "204.42.110.101"),
            ("egressInterface", 854), ("octetDeltaCount", 1312), ("packetDeltaCount", 9),
            ("flowStartSysUpTime", 0xb3f906ee), ("flowEndSysUpTime", 0xb3fbaf3c),
            ("ipNextHopIPv4Address", "204.42.110.189"), ("sourceIPv4PrefixLength", 24),
            ("destinationIPv4PrefixLength", 24), ("tcpControlBits", NO_FLAGS), ("ipVersion", 4),
            ("flowStartMilliseconds", "2016-11-29T20:05:31.519Z"),
            ("flowEndMilliseconds", "2016-11-29T20:08:25.677Z")])))))]}],
    # ipfix.rs:294-329
    "ipfix_options_template_packet": [{"steps": [
        ("ipfix", W + "test_options_template_packet:good_wire", ("ok", ipfix(
            "2016-11-29T20:08:55Z", 3791, 0, OTS(OT(308, [S("ipClassOfService", 1)],
                                                    [S("flowActiveTimeout", 2), S("flowIdleTimeout", 2)]))))),
    ]}],
    # ipfix.rs:331-466 (both parses only unwrap Ok)
    "ipfix_complex_sequence": [{"steps": [
        ("ipfix", W + "test_complex_sequence:pkt1_wire", ("ok?", None)),
        ("ipfix", W + "test_complex_sequence:pkt2_wire", ("ok?", None)),
    ]}],
    # ipfix.rs:468-517 (options template with 2 bytes of set padding)
    "ipfix_example": [{"steps": [
        ("ipfix", W + "test_example:good_wire", ("ok", ipfix("2023-01-28T15:56:28Z", 3571, 524288, OTS(OT(
            512, [S("exportingProcessId", 4)],
            [S("exportedMessageTotalCount", 8), S("exportedFlowRecordTotalCount", 8),
             S("systemInitTimeMilliseconds", 8), S("exporterIPv4Address", 4), S("exporterIPv6Address", 16),
             S("samplingInterval", 4), S("flowActiveTimeout", 2), S("flowIdleTimeout", 2),
             S("exportProtocolVersion", 1), S("exportTransportProtocol", 1)]))))),
    ]}],
    # ipfix.rs:519-595
    "ipfix_with_variable_string_length": [{"steps": [
        ("ipfix", W + "test_with_variable_string_length:good_template_wire", ("ok", ipfix(
            "2023-12-22T15:18:53Z", 118278, 33312, OTS(OT(
                257, [S("selectorId", 4)],
                [S("samplingPacketInterval", 4), S("selectorAlgorithm", 2), S("samplingSize", 4),
                 S("samplingPopulation", 4), S("samplerName", 90), S("selectorName", 65535)]))))),
        ("ipfix", W + "test_with_variable_string_length:good_data_wire", ("ok", ipfix(
            "2023-12-22T15:18:53Z", 118278, 33312, D(257, R(
                [("samplingPacketInterval", 1), ("selectorAlgorithm", "RandomnoutofNSampling"),
                 ("samplingSize", 1), ("samplingPopulation", 1), ("samplerName", "NETFLOW-SAMPLER-MAP"),
                 ("selectorName", "NETFLOW-SAMPLER-MAP")], scope=[("selectorId", 1)]))))),
    ]}],
    # ipfix.rs:597-688
    "ipfix_with_nokia_pen_fields": [{"steps": [
        ("ipfix", W + "test_with_nokia_pen_fields:good_template_wire", ("ok", ipfix(
            "2024-06-20T14:00:00Z", 0, 0, TS(T(
                400, S("sourceIPv4Address", 4), S("destinationIPv4Address", 4), S("sourceTransportPort", 2),
                S("destinationTransportPort", 2), S("postNATSourceIPv4Address", 4),
                S("postNAPTSourceTransportPort", 2), S("flowId", 8), S("protocolIdentifier", 1),
                S("engineType", 1), S(vie("Nokia", "aluInsideServiceId"), 2),
                S(vie("Nokia", "aluOutsideServiceId"), 2), S(vie("Nokia", "aluNatSubString"), 65535),
                S("octetDeltaCount", 4), S("packetDeltaCount", 4)))))),
        ("ipfix", W + "test_with_nokia_pen_fields:good_data_wire", ("ok", ipfix(
            "2024-06-20T14:00:00Z", 0, 0, D(400, R([
                ("sourceIPv4Address", "10.100.0.1"), ("destinationIPv4Address", "10.100.0.151"),
                ("sourceTransportPort", 10004), ("destinationTransportPort", 1),
                ("postNATSourceIPv4Address", "8.8.8.8"), ("postNAPTSourceTransportPort", 8881),
                ("flowId", 10101010), ("protocolIdentifier", "ICMP"), ("engineType", 0),
                V("Nokia", "aluInsideServiceId", 1), V("Nokia", "aluOutsideServiceId", 15),
                V("Nokia", "aluNatSubString", "LSN-Host@10.10.10.101"), ("octetDeltaCount", 1200),
                ("packetDeltaCount", 1)]))))),
    ]}],
    # ipfix.rs:690-804
    "ipfix_with_vmware_pen_fields": [{"steps": [
        ("ipfix", W + "test_with_vmware_pen_fields:good_template_wire", ("ok", ipfix(
            "2024-07-08T10:00:00Z", 0, 0, TS(T(
                400, S("sourceIPv4Address", 4), S("destinationIPv4Address", 4), S("sourceTransportPort", 2),
                S("destinationTransportPort", 2), S("flowId", 8), S("protocolIdentifier", 1),
                S("octetDeltaCount", 4), S("packetDeltaCount", 4), S(vie("VMWare", "ingressInterfaceAttr"), 2),
                S(vie("VMWare", "egressInterfaceAttr"), 2), S(vie("VMWare", "vxlanExportRole"), 1),
                S(vie("VMWare", "tenantSourceIPv4"), 4), S(vie("VMWare", "tenantDestIPv4"), 4),
                S(vie("VMWare", "tenantSourcePort"), 2), S(vie("VMWare", "tenantDestPort"), 2),
                S(vie("VMWare", "tenantProtocol"), 1), S(vie("VMWare", "flowDirection"), 1),
                S(vie("VMWare", "virtualObsID"), 65535)))))),
        ("ipfix", W + "test_with_vmware_pen_fields:good_data_wire", ("ok", ipfix(
            "2024-06-20T14:00:00Z", 0, 0, D(400, R([
                ("sourceIPv4Address", "10.100.0.1"), ("destinationIPv4Address", "10.100.0.151"),
                ("sourceTransportPort", 10004), ("destinationTransportPort", 1), ("flowId", 10101010),
                ("protocolIdentifier", "ICMP"), ("octetDeltaCount", 1200), ("packetDeltaCount", 1),
                V("VMWare", "ingressInterfaceAttr", 10), V("VMWare", "egressInterfaceAttr", 12),
                V("VMWare", "vxlanExportRole", 0), V("VMWare", "tenantSourceIPv4", "192.168.140.6"),
                V("VMWare", "tenantDestIPv4", "192.168.140.68"), V("VMWare", "tenantSourcePort", 20023),
                V("VMWare", "tenantDestPort", 443), V("VMWare", "tenantProtocol", "TCP"),
                V("VMWare", "flowDirection", "ingress"),
                V("VMWare", "virtualObsID", "aaaaaaaa-bbbb-cccc-dddd-eeeeeeeeeeee")]))))),
    ]}],
    # ipfix.rs:806-890
    "ipfix_with_vendor_unknown_fields": [{"steps": [
        ("ipfix", W + "test_with_vendor_unknown_fields:good_template_wire", ("ok", ipfix(
            "2024-07-08T10:00:00Z", 0, 0, TS(T(
                400, S("sourceIPv4Address", 4), S("protocolIdentifier", 1), S("packetDeltaCount", 4),
                S(vie("VMWare", "ingressInterfaceAttr"), 2), S(vunk_ie("VMWare", 2552), 2),
                S(vunk_ie("VMWare", 2553), 65535), S(vie("VMWare", "vxlanExportRole"), 1)))))),
        ("ipfix", W + "test_with_vendor_unknown_fields:good_data_wire", ("ok", ipfix(
            "2024-06-20T14:00:00Z", 0, 0, D(400, R([
                ("sourceIPv4Address", "10.100.0.1"), ("protocolIdentifier", "ICMP"), ("packetDeltaCount", 1),
                V("VMWare", "ingressInterfaceAttr", 10), VU("VMWare", 2552, [0x11, 0xee]),
                VU("VMWare", 2553, [0x02, 0xee, 0xff]), V("VMWare", "vxlanExportRole", 0)]))))),
    ]}],
    # ipfix.rs:892-1021
    "ipfix_with_iana_subregs": [{"steps": [
        ("ipfix", W + "test_with_iana_subregs:good_template_wire", ("ok", ipfix(
            "2024-07-08T10:00:00Z", 0, 0, TS(T(400, *T400_SUBREGS))))),
        ("ipfix", W + "test_with_iana_subregs:good_data_wire", ("ok", ipfix(
            "2024-06-20T14:00:00Z", 0, 0, D(400, R400_SUBREGS)))),
    ]}],
    # ipfix.rs:1023-1035 (asserts only is_err; no divide by zero)
    "ipfix_zero_length_fields": [{"steps": [
        ("ipfix", W + "test_zero_length_fields:good_template_wire", ("err?", None))]}],
    # ipfix.rs:1037-1117
    "ipfix_with_unknown_pen": [{"steps": [
        ("ipfix", W + "test_with_unknown_pen:good_template_wire", ("ok", ipfix(
            "2024-07-08T10:00:00Z", 0, 0, TS(T(
                400, S("sourceIPv4Address", 4), S("destinationIPv4Address", 4), S(unk_ie(213, 567), 4),
                S("natThresholdEvent", 1), S(unk_ie(213, 769), 8), S("srhIPv6ActiveSegmentType", 1)))))),
        ("ipfix", W + "test_with_unknown_pen:good_data_wire", ("ok", ipfix(
            "2024-06-20T14:00:00Z", 0, 0, D(400, R([
                ("sourceIPv4Address", "10.100.0.1"), ("destinationIPv4Address", "10.100.0.151"),
                U(213, 567, [1, 2, 3, 4]), ("natThresholdEvent", "Addresspoolhighthresholdevent"),
                U(213, 769, [1, 2, 3, 4, 5, 6, 7, 8]),
                ("srhIPv6ActiveSegmentType", "BGPSegmentRoutingPrefixSID")]))))),
    ]}],
    # ipfix.rs:1119-1379
    "ipfix_with_vendor_unknown_field_complex": [{"steps": [
        ("ipfix", W + "test_with_vendor_unknown_field_complex:good_template_wire", ("ok", ipfix(
            "2025-08-26T08:48:44Z", 2230, 2149482753, TS(T(
                2599, S("sourceIPv6Address", 16), S("destinationIPv6Address", 16), S("ipNextHopIPv6Address", 16),
                S("packetDeltaCount", 4), S("octetDeltaCount", 4), S("flowStartSysUpTime", 4),
                S("flowEndSysUpTime", 4), S("systemInitTimeMilliseconds", 8), S("bgpNextHopIPv6Address", 16),
                S("ingressInterface", 4), S("egressInterface", 4), S("bgpSourceAsNumber", 2),
                S("bgpDestinationAsNumber", 2), S("sourceTransportPort", 2), S("destinationTransportPort", 2),
                S("vlanId", 2), S("postVlanId", 2), S(vunk_ie("Huawei", 232), 2), S("tcpControlBits", 1),
                S("protocolIdentifier", 1), S("ipClassOfService", 1), S("sourceIPv6PrefixLength", 1),
                S("destinationIPv6PrefixLength", 1), S("flowDirection", 1), S("forwardingStatus", 1),
                S("flowLabelIPv6", 3), S("flowEndReason", 1), S("paddingOctets", 3), S("samplerId", 4),
                S("ingressVRFID", 4), S("egressVRFID", 4), S("selectorId", 8), S("ipv6ExtensionHeadersFull", 4),
                S("destinationMacAddress", 6), S("sourceMacAddress", 6), S("dot1qVlanId", 2),
                S("dot1qCustomerVlanId", 2), S("dot1qPriority", 1), S("dot1qCustomerPriority", 1),
                S("paddingOctets", 2), S("srhTagIPv6", 2), S("srhFlagsIPv6", 1), S("srhSegmentsIPv6Left", 1),
                S("srhActiveSegmentIPv6", 16), S("srhIPv6ActiveSegmentType", 1), S("paddingOctets", 2),
                S("srhSegmentIPv6ListSection", 65535)))))),
        ("ipfix", W + "test_with_vendor_unknown_field_complex:good_data_wire", ("ok", ipfix(
            "2025-08-26T08:49:03Z", 2231, 2149482753, D(
                2599,
                _r2599("2001:db8:44::1", "2001:db8:48::1", 98, 6360000, 25, 152, 64299, [0, 0],
                       tcp(False, False, False, False, True, False, False, False), 0, 25, 0, 6,
                       [36, 70, 228, 168, 77, 29], [96, 38, 170, 125, 154, 196], 0, 0),
                _r2599("fd00::2", "fd00::1", 117, 6366000, 154, 154, 61351, [0, 1],
                       tcp(False, False, False, True, True, False, False, False), 325809, 154, 1, 4,
                       [36, 70, 228, 168, 77, 13], [48, 251, 184, 230, 103, 172], 23, 6))))),
    ]}],
    # ipfix.rs:1381-1539: the same data under a fixed-length and a
    # variable-length (65535) applicationId template, in two maps
    "ipfix_octet_array_variable_len": [
        {"steps": [
            ("ipfix", W + "test_octet_array_variable_len:template_fixed_size_wire", ("ok", ipfix(
                "2024-12-27T20:46:44Z", 1, 12345, TS(T(256, S("sourceIPv4Address", 4),
                                                       S("destinationIPv4Address", 4), S("applicationId", 4)))))),
            ("ipfix", W + "test_octet_array_variable_len:data_fixed_wire", ("ok", ipfix(
                "2024-12-27T20:46:45Z", 2, 12345, D(256, R([
                    ("sourceIPv4Address", "192.168.1.100"), ("destinationIPv4Address", "10.0.0.1"),
                    ("applicationId", [0x03, 0x00, 0x00, 0x09])]))))),
        ]},
        {"steps": [
            ("ipfix", W + "test_octet_array_variable_len:template_variable_size_wire", ("ok", ipfix(
                "2024-12-27T20:46:44Z", 1, 12345, TS(T(256, S("sourceIPv4Address", 4),
                                                       S("destinationIPv4Address", 4),
                                                       S("applicationId", 65535)))))),
            ("ipfix", W + "test_octet_array_variable_len:template_variable_size_wire", ("same", 0)),
            ("ipfix", W + "test_octet_array_variable_len:data_variable_wire", ("ok", ipfix(
                "2024-12-27T20:46:45Z", 2, 12345, D(256, R([
                    ("sourceIPv4Address", "192.168.1.100"), ("destinationIPv4Address", "10.0.0.1"),
                    ("applicationId", [0x03, 0x00, 0x00, 0x09])]))))),
        ]},
    ],
    # ipfix.rs:1541-1701: the template parse, and the data packet that
    # test_write_with_one_input(&data, ...) serializes to data_wire (its inverse)
    "ipfix_flow_set_len_bug": [{"steps": [
        ("ipfix", W + "test_flow_set_len_bug:template_wire", ("ok", ipfix(
            "2025-12-22T11:24:08Z", 1, 0, OTS(OT(500, [S("applicationId", 4)],
                                                 [S("applicationName", 65535),
                                                  S("applicationCategoryName", 65535)]))))),
        ("ipfix", W + "test_flow_set_len_bug:data_wire", ("ok", ipfix(
            "2025-12-22T11:24:08Z", 10, 0, D(500, *[
                R([("applicationName", "name for id: " + a), ("applicationCategoryName", "category for id: " + c)],
                  scope=[("applicationId", [0x0d, 0x00, 0x00, b])]) for b, a, c in _APP])))),
    ]}],
    # ipfix.rs:1877-1929 (template 500 inserted into the map)
    "ipfix_padding_min_length_issue_360": [{
        "preload": {500: ([S(vie("VMWare", "sessionFlags"), 1), S(vie("VMWare", "vifId"), 65535)],
                          [S("applicationName", 65535), S("applicationCategoryName", 65535)])},
        "steps": [
            ("ipfix", W + "test_padding_min_length_issue_360:data_wire", ("ok", ipfix(
                "2025-12-22T11:24:08Z", 10, 0, D(500, R(
                    [("applicationName", "name for id: 2426945984"),
                     ("applicationCategoryName", "category for id: 4285581510")],
                    scope=[V("VMWare", "sessionFlags", 0xee), V("VMWare", "vifId", "some-id")]))))),
        ]}],
    # serde_benchmark.rs:12-161, 163-166: every parse unwraps Ok; the data-only
    # packet reuses the templates the mixed packet defines (:225-230)
    "bench_template_only": [{"steps": [("ipfix", B + "IPFIX_PKT_TEMPLATE_RAW", ("ok", T307_PKT))]}],
    "bench_options_template_only": [{"steps": [("ipfix", B + "IPFIX_PKT_OPTIONS_TEMPLATE_RAW", ("ok?", None))]}],
    "bench_mixed_then_data_only": [{"steps": [
        ("ipfix", B + "IPFIX_PKT_MIXED", ("ok?", None)),
        ("ipfix", B + "IPFIX_PKT_DATA_PKT_ONLY", ("ok?", None)),
        ("ipfix", B + "IPFIX_PKT_DATA_PKT_ONLY", ("same", 1)),
    ]}],

    # mod.rs:35-65 test_template_record: TemplateRecord::parse of a lone record (wrapped into a template set
    # of an IPFIX message for the codec-level device run); template id 0 is InvalidTemplateId at the record
    # start (ipfix.rs:384-413)
    "mod_template_record": [{"steps": [
        ("tplrec", M + "test_template_record:good_wire",
         ("ok", T(2049, S("sourceIPv6Address", 16), S("destinationIPv6Address", 16)))),
        ("tplrec", M + "test_template_record:bad_template_id_wire",
         ("err", {"InvalidTemplateId": {"offset": 0, "template_id": 0}})),
    ]}],
    # mod.rs:67-74 test_field: FieldSpecifier::parse (deserializer/mod.rs:53-66), wrapped into a one-field
    # template record 256
    "mod_field": [{"steps": [("fspec", M + "test_field:good_ipv4_src_wire", ("ok", S("sourceIPv4Address", 4)))]}],
    # mod.rs:346-374 test_data_record_value: DataRecord::parse with the DecodingTemplate [sourceMacAddress 6,
    # destinationMacAddress 6] (inserted as template 256; the record wrapped into a data set of it)
    "mod_data_record_value": [{"preload": {256: ([], [S("sourceMacAddress", 6), S("destinationMacAddress", 6)])},
                               "steps": [
        ("datarec", M + "test_data_record_value:value_wire", ("ok", R([
            ("sourceMacAddress", [0x12, 0xc6, 0x21, 0x12, 0x69, 0x32]),
            ("destinationMacAddress", [0x12, 0xc6, 0x21, 0x12, 0x69, 0x32])]))),
    ]}],
    # mod.rs:376-420 test_set_template: Set::parse of a lone template set (template 307), wrapped into an
    # IPFIX message
    "mod_set_template": [{"steps": [("ipfixset", M + "test_set_template:good_wire", ("ok", TS(T(307, *T307))))]}],

    # netflow.rs:30-69
    "nf9_template_record": [{"steps": [
        ("nf9", N + "test_netflow9_template_record:good_wire", ("ok", nf9(
            398475, "2017-07-25T12:49:01Z", 0, 0, TS(T(1024, *T1024_NF))))),
    ]}],
    # netflow.rs:71-202 (template 1024 inserted into the map)
    "nf9_data_record": [{"preload": {1024: ([], T1024_NF)}, "counts": {1024: 4}, "steps": [
        ("nf9", N + "test_netflow9_data_record:good_wire", ("ok", nf9(
            458441, "2017-07-25T12:50:01Z", 1, 0, D(
                1024,
                _r1024("192.168.1.100", "216.58.211.99", 107173, 106988, 66, 52357, 443),
                _r1024("216.58.211.99", "192.168.1.100", 107173, 106988, 1378, 443, 52357),
                _r1024("192.168.1.100", "216.58.211.110", 117589, 117589, 66, 63111, 443),
                _r1024("192.168.1.100", "216.58.211.110", 145525, 145525, 51, 63273, 443))))),
    ]}],
    # netflow.rs:204-364 (template 313 inserted; processed_count 2 after)
    "nf9_data_packet": [{"preload": {313: ([], T313_NF)}, "counts": {313: 2}, "steps": [
        ("nf9", N + "test_data_packet:good_wire", ("ok", nf9(
            201984782, "2023-01-28T15:56:09Z", 14925203, 2081,
            D(313, _r313(0x0c09cac2, 38718), _r313(0x0c09cac3, 38722))))),
    ]}],
    # netflow.rs:366-386, 388-407 (Set::parse of a lone options template set)
    "nf9_mix_option_template_set": [{"steps": [
        ("nf9set", N + "test_mix_option_template_set:good_wire", ("ok", OTS(OT(
            277, [S("System", 4)], [S("ingressInterface", 2), S("interfaceName", 16),
                                    S("interfaceDescription", 32)])))),
    ]}],
    "nf9_mix_option_template_set2": [{"steps": [
        ("nf9set", N + "test_mix_option_template_set2:good_wire", ("ok", OTS(OT(
            334, [S("System", 4)], [S("ingressVRFID", 4), S("VRFname", 32)])))),
    ]}],
    # netflow.rs:409-620: padded / unpadded give equal packets; bad padding
    # errors carry exact offsets; the bad pair shares one map
    "nf9_padding": [
        {"steps": [("nf9", N + "test_padding:good_no_padding_wire", ("ok?", None))]},
        {"steps": [("nf9", N + "test_padding:good_with_padding_wire", ("ok?", None))]},
        {"steps": [
            ("nf9", N + "test_padding:bad_padding_options_wire",
             ("err", {"SetError": {"InvalidPaddingValue": {"offset": 51, "value": 17}}})),
            ("nf9", N + "test_padding:bad_padding_data_wire",
             ("err", {"SetError": {"InvalidPaddingValue": {"offset": 107, "value": 1}}})),
        ]},
    ],
    # netflow.rs:622-754
    "nf9_with_iana_subregs": [{"steps": [
        ("nf9", N + "test_with_iana_subregs:good_template_wire", ("ok", nf9(
            120, "2024-07-08T13:00:00Z", 0, 0, TS(T(400, *T400_SUBREGS))))),
        ("nf9", N + "test_with_iana_subregs:good_data_wire", ("ok", nf9(
            120, "2024-07-08T13:00:00Z", 1, 0, D(400, R400_SUBREGS)))),
    ]}],
    # netflow.rs:756-770, 772-802 (assert only is_err: no divide by zero, no
    # count underflow)
    "nf9_zero_length_fields": [{"steps": [("nf9", N + "test_zero_length_fields:good_template_wire", ("err?", None))]}],
    "nf9_records_len_larger_than_count": [{"steps": [
        ("nf9", N + "test_records_len_larger_than_count:good_template_wire", ("err?", None))]}],
}

# Equal-packet assertions across maps (netflow.rs:595-605): the padded and the
# unpadded v9 packet parse to the same value.
SAME_ACROSS = [("nf9_padding", (0, 0), (1, 0))]


# --- SliceReader KATs (crates/parse-utils/src/reader.rs:298-561) ---------------
# (test, fixture data key, [(op, args, expected)]) where op is one of
#   u8 / u16 / u32 / i32 / i64 / u64 (fixed reads), padded(N, len),
#   uint32(len) / uint64(len) (reduced size), int32(len) / int64(len),
#   take(n) (-> (offset, bytes)), offset / remaining
# and expected is a value or ("eof", offset, needed, available) /
# ("pad", offset, requested, ret_len).
R_ = "reader.rs:"
READER_KATS = [
    ("reads_advance_and_track_offset", [("u8", (), 0x00), ("u16", (), 0x0102), ("offset", (), 3),
                                        ("remaining", (), 2)]),
    ("eof_reports_offset_needed_available", [("u8", (), 0xAA), ("u32", (), ("eof", 1, 4, 1))]),
    ("peek_does_not_advance", [("peek16", (), 0x1234), ("offset", (), 0)]),
    ("take_slice_carries_absolute_offset", [("u16", (), 0x0001), ("take", (3,), (2, bytes([2, 3, 4])))]),
    ("len_equal_to_n_reads_full_no_padding", [("padded", (4, 4), bytes([0xDE, 0xAD, 0xBE, 0xEF])),
                                              ("offset", (), 4), ("remaining", (), 0)]),
    ("short_len_left_aligns_and_zero_pads_tail", [("padded", (4, 2), bytes([0xAA, 0xBB, 0, 0])),
                                                  ("offset", (), 2), ("rest", (), bytes([0xCC]))]),
    ("zero_len_yields_all_zeros_without_advancing", [("padded", (4, 0), bytes(4)), ("offset", (), 0),
                                                     ("remaining", (), 2)]),
    ("len_within_n_but_buffer_too_short_is_eof", [("padded", (4, 3), ("eof", 0, 3, 1)), ("offset", (), 0)]),
    ("capacity_error_reports_current_offset", [("u16", (), 0), ("padded", (2, 5), ("pad", 2, 5, 2)),
                                               ("offset", (), 2)]),
    ("uint_be_full_width_matches_fixed_read", [("uint64", (8,), 0x0123456789ABCDEF)]),
    ("uint_be_zero_len_reads_nothing", [("uint64", (0,), 0), ("offset", (), 0)]),
    ("uint_be_short_buffer_is_eof", [("uint64", (4,), ("eof", 0, 4, 2))]),
    ("int_be_sign_extends_shortened_negative", [("int64", (1,), -2)]),
    ("int_be_keeps_positive_values_unsigned", [("int64", (1,), 127)]),
    ("int_be_full_width_matches_fixed_read", [("int64", (8,), -2), ("int64", (8,), ("eof", 8, 8, 0))]),
    ("int_be_zero_len_is_not_negative", [("int64", (0,), 0), ("offset", (), 0)]),
    ("uint32_be_full_width_matches_fixed_read", [("uint32", (4,), 0x01234567)]),
    ("uint32_be_zero_len_reads_nothing", [("uint32", (0,), 0), ("offset", (), 0)]),
    ("uint32_be_short_buffer_is_eof", [("uint32", (4,), ("eof", 0, 4, 1))]),
    ("int32_be_sign_extends_shortened_negative", [("int32", (1,), -2)]),
    ("int32_be_keeps_positive_values_unsigned", [("int32", (1,), 127)]),
    ("int32_be_full_width_matches_fixed_read", [("int32", (4,), -2), ("int32", (4,), ("eof", 4, 4, 0))]),
    ("int32_be_zero_len_is_not_negative", [("int32", (0,), 0), ("offset", (), 0)]),
]
# reader.rs:400-412, 481-493: 0x0000ABCD carried in 2, 3 and 4 octets (no data
# variable: the wires are inline in the loop)
READER_SHORTENED = [bytes([0xAB, 0xCD]), bytes([0x00, 0xAB, 0xCD]), bytes([0x00, 0x00, 0xAB, 0xCD])]
# reader.rs:430-439, 511-520: len beyond the width is rejected before consuming
READER_TOO_WIDE = [("uint64", 9, ("pad", 0, 9, 8)), ("uint32", 5, ("pad", 0, 5, 4))]


# --- FlowInfoCodec::decode KAT (crates/flow-pkt/src/codec.rs:226-249) ---------------------------
# test_decode_partial_messages: one codec, two decode calls on their own buffers.  value1 is an
# IPFIX header announcing 116 bytes followed by 2 of them (18 bytes), value2 a single byte (shorter
# than the 16-byte header gate, codec.rs:197-201): both Ok(None) -- NGZ_DG_NEED_MORE at the C ABI --
# and neither consumes a byte (the gates return before the buffer is touched, codec.rs:197-207).
C_ = "codec.rs:test_decode_partial_messages:"
CODEC_PARTIAL = [(C_ + "value1", None), (C_ + "value2", None)]  # (wire, expected decode result)

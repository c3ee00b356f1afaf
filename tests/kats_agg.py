"""Known-answer vectors of the reference's aggregation unit tests, restated as data
(crates/collector/src/flow/aggregation/aggregator/tests.rs).  Used to pin
oracle/ngz_agg_oracle.py (tests/test_oracle_agg.py) and, as wire bytes, the device
aggregation (tests/test_gpu_agg.py).

IE ids: sourceIPv4Address 8, destinationIPv4Address 12, protocolIdentifier 4,
octetDeltaCount 1, packetDeltaCount 2, minimumTTL 52, maximumTTL 53,
sourceTransportPort 7, destinationTransportPort 11, tcpControlBits 6,
fragmentFlags 197.  TCPHeaderFlags::new(fin, syn, rst, psh, ack, urg, ece, cwr)
is the u8 with FIN = 0x01 ... CWR = 0x80 (iana/src/tcp.rs).
"""
import struct

OP_KEY, OP_ADD, OP_MIN, OP_MAX, OP_OR = 0, 1, 2, 3, 4
T_2025_01_01_16 = 1735747200  # Utc.with_ymd_and_hms(2025, 1, 1, 16, 0, 0)

# test_explode_ipfix_repeating_ie_fields (tests.rs:755-827): set 400, obs domain 300,
# peer 172.16.0.1:4739; key_select / agg_select with FieldRef indices
REPEAT_TEMPLATE = [(8, 4), (8, 4), (12, 4), (4, 1), (4, 1), (4, 1), (1, 8), (1, 8)]
REPEAT_RECORD = (struct.pack(">IIIBBBQQ", 0x0A000001, 0x64646401, 0x0A000002, 41, 4, 17, 100, 200))
REPEAT_FIELDS = [(0, 8, 1, OP_KEY), (0, 12, 0, OP_KEY), (0, 4, 0, OP_KEY), (0, 4, 2, OP_KEY),
                 (0, 1, 0, OP_ADD), (0, 1, 1, OP_ADD)]
REPEAT_EXPECTED = dict(key=(0x64646401, 0x0A000002, 41, 17), vals=(100, 200), record_count=1,
                       ports={4739}, domains={300}, templates={(10, 400)},
                       min_export=T_2025_01_01_16, max_export=T_2025_01_01_16, max_sysup=0)

# test_explode_ipfix_missing_fields (tests.rs:830-893) shape: a selected IE the record
# lacks is None (key and agg)
MISSING_TEMPLATE = [(8, 4), (1, 8)]
MISSING_RECORD = struct.pack(">IQ", 0x0A000001, 1000)
MISSING_FIELDS = [(0, 8, 0, OP_KEY), (0, 12, 0, OP_KEY), (0, 1, 0, OP_ADD), (0, 2, 0, OP_ADD)]
MISSING_EXPECTED = dict(key=(0x0A000001, None), vals=(1000, None), record_count=1)

# test_reduce_add_operations (tests.rs:244-337): record1 + record2 -> expected
REDUCE_FIELDS = [(0, 1, 0, OP_ADD), (0, 2, 0, OP_ADD), (0, 52, 0, OP_MIN), (0, 53, 0, OP_MAX),
                 (0, 7, 0, OP_MIN), (0, 11, 0, OP_MAX), (0, 6, 0, OP_OR), (0, 197, 0, OP_OR)]
REDUCE_R1 = (1000, 10, 64, 128, 80, None, 0x03, None)
REDUCE_R2 = (2000, 20, 32, 255, None, 22, 0xC0, None)
REDUCE_EXPECTED = (3000, 30, 32, 255, 80, 22, 0xC3, None)
# as wire records: template 256 carries sourceTransportPort, 257 destinationTransportPort
REDUCE_TEMPLATE_1 = [(1, 8), (2, 8), (52, 1), (53, 1), (7, 2), (6, 2)]
REDUCE_TEMPLATE_2 = [(1, 8), (2, 8), (52, 1), (53, 1), (11, 2), (6, 2)]
REDUCE_WIRE_1 = struct.pack(">QQBBHH", 1000, 10, 64, 128, 80, 0x03)
REDUCE_WIRE_2 = struct.pack(">QQBBHH", 2000, 20, 32, 255, 22, 0xC0)

# test_explode_simple_netflowv9_packet (tests.rs:946-1017): NetFlowV9Packet::new(sys_up_time 1000,
# 2025-01-01 12:00:00, seq 1, source_id 100), data set 256, peer 192.168.1.1:9995, collection
# time 2025-01-01 10:00:00
T_2025_01_01_12 = 1735732800
T_2025_01_01_10_MS = 1735725600000
NF_TEMPLATE = [(8, 4), (12, 4), (7, 2), (11, 2), (1, 8), (2, 8)]
NF_RECORD = struct.pack(">IIHHQQ", 0x0A000001, 0x0A000002, 80, 443, 1000, 10)
NF_FIELDS = [(0, 8, 0, OP_KEY), (0, 12, 0, OP_KEY), (0, 7, 0, OP_KEY), (0, 11, 0, OP_KEY),
             (0, 1, 0, OP_ADD), (0, 2, 0, OP_ADD)]
NF_EXPECTED = dict(flow_type=9, key=(0x0A000001, 0x0A000002, 80, 443), vals=(1000, 10), record_count=1,
                   ports={9995}, domains={100}, templates={(9, 256)}, min_export=T_2025_01_01_12,
                   max_export=T_2025_01_01_12, max_sysup=1000, min_coll=T_2025_01_01_10_MS,
                   max_coll=T_2025_01_01_10_MS)


def nf_packet():
    """The test's packet as NetFlow v9 wire bytes: template flowset + data flowset, count 2."""
    tpl = struct.pack(">HH", 256, len(NF_TEMPLATE)) + b"".join(struct.pack(">HH", i, n) for i, n in NF_TEMPLATE)
    tset = struct.pack(">HH", 0, 4 + len(tpl)) + tpl
    dset = struct.pack(">HH", 256, 4 + len(NF_RECORD)) + NF_RECORD
    return struct.pack(">HHIIII", 9, 2, 1000, T_2025_01_01_12, 1, 100) + tset + dset


# ---------------------------------------------------------------------------------------------
# The rest of aggregator/tests.rs (:72-1377) and the window tests of analytics/src/aggregation.rs
# (:579-789), restated as wire-level scenarios: every AggFlowInfo / FlowInfo / TestItem of a test
# becomes IPFIX or NetFlow v9 datagrams that decode to exactly its fields, pushed as sent by the
# test's peer (IP, port) at the test's collection time; the expected groups are the test's
# expected cache entries / windows.  Where a test builds items with different field sets under one
# template id (a None in agg_fields), the template is redefined between the items' messages, so the
# group's template set stays the test's.  Times: the tests' Utc.with_ymd_and_hms / RFC 3339 values.
# ---------------------------------------------------------------------------------------------
T10, T11, T12, T13 = 1735725600, 1735729200, 1735732800, 1735736400
T14_30, T15, T16, T18, T20 = 1735741800, 1735743600, 1735747200, 1735754400, 1735761600
T_JUL2_10, T_JUL2_10_05 = 1751450400, 1751450405  # 2025-07-02T10:00:00Z / 10:00:05Z
T_2025 = 1735689600                                  # 2025-01-01T00:00:00Z

SRC4, DST4, SPORT, DPORT, OCTETS, PACKETS = 8, 12, 7, 11, 1, 2
MIN_TTL, MAX_TTL, TCP_FLAGS, SRC6 = 52, 53, 6, 27


def ip4(a, b, c, d):
    return (a << 24) | (b << 16) | (c << 8) | d


def tcp(fin, syn, rst, psh, ack, urg, ece, cwr):
    """TCPHeaderFlags::new(fin, syn, rst, psh, ack, urg, ece, cwr) as its u8 (FIN = bit 0)."""
    return sum(1 << i for i, b in enumerate((fin, syn, rst, psh, ack, urg, ece, cwr)) if b)


ENC = {SRC4: ">I", DST4: ">I", SPORT: ">H", DPORT: ">H", OCTETS: ">Q", PACKETS: ">Q", MIN_TTL: ">B",
       MAX_TTL: ">B", TCP_FLAGS: ">H", SRC6: None}


def record(fields):
    """[(IE, value)] -> (template field list, record bytes)."""
    tpl, b = [], b""
    for ie, v in fields:
        if ie == SRC6:
            tpl.append((ie, 16))
            b += v
        else:
            tpl.append((ie, struct.calcsize(ENC[ie])))
            b += struct.pack(ENC[ie], v)
    return tpl, b


def ipfix_msg(sets, export_time, seq=1, domain=7):
    body = b"".join(sets)
    return struct.pack(">HHIII", 10, 16 + len(body), export_time, seq, domain) + body


def tset(tid, fields):
    body = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, n) for i, n in fields)
    return struct.pack(">HH", 2, 4 + len(body)) + body


def dset(tid, recs):
    body = b"".join(recs)
    return struct.pack(">HH", tid, 4 + len(body)) + body


def ipfix_packet(tid, records, export_time, seq, domain):
    """IpfixPacket::new(export_time, seq, domain, [Set::Data{id: tid, records}]) on the wire: the
    template set, then the data set (records: lists of (IE, value), one shape)."""
    shapes = [record(r) for r in records]
    assert all(s[0] == shapes[0][0] for s in shapes)
    return ipfix_msg([tset(tid, shapes[0][0]), dset(tid, [b for _, b in shapes])], export_time, seq, domain)


def nf_packet_of(tid, records, sys_up_time, unix_time, seq, source_id):
    """NetFlowV9Packet::new(sys_up_time, unix_time, seq, source_id, [Set::Data{id: tid, records}]):
    a template flowset and a data flowset (count = 1 template + the records)."""
    shapes = [record(r) for r in records]
    tpl = shapes[0][0]
    t = struct.pack(">HH", tid, len(tpl)) + b"".join(struct.pack(">HH", i, n) for i, n in tpl)
    ts = struct.pack(">HH", 0, 4 + len(t)) + t
    data = b"".join(b for _, b in shapes)
    ds = struct.pack(">HH", tid, 4 + len(data)) + data
    return struct.pack(">HHIIII", 9, 1 + len(records), sys_up_time, unix_time, seq, source_id) + ts + ds


def G(peer, window_start, key, vals, flow_type=10, count=1, export=None, coll_ms=None, sysup=0,
      templates=(), ports=(), domains=()):
    """An expected group (FlowCacheKey + FlowCacheRecord) in the oracle's / device's canonical form."""
    export = window_start if export is None else export
    return dict(peer=peer, window_start=window_start, flow_type=flow_type, key=tuple(key), vals=tuple(vals),
                record_count=count, min_export=export if not isinstance(export, tuple) else export[0],
                max_export=export if not isinstance(export, tuple) else export[1], max_sysup=sysup,
                min_coll=coll_ms if not isinstance(coll_ms, tuple) else coll_ms[0],
                max_coll=coll_ms if not isinstance(coll_ms, tuple) else coll_ms[1],
                templates=set(templates), ports=set(ports), domains=set(domains))


def minute(t):
    return t - t % 60


# A scenario: fields, pushes [(peer_ip, peer_port, collection_ms, [datagrams])], the groups each
# push's closed windows emit (None: not checked), the groups of the final flush, late records.
def _s(name, src, fields, pushes, flush, emits=None, late=0, window_s=60, lateness_s=10):
    return dict(name=name, src=src, fields=fields, pushes=pushes, flush=flush, emits=emits, late=late,
                window_s=window_s, lateness_s=lateness_s)


K2 = [(0, SRC4, 0, OP_KEY), (0, DST4, 0, OP_KEY)]
P192_1 = "192.168.1.1"
T10_MS = T10 * 1000
k_10_1, k_10_2 = ip4(10, 0, 0, 1), ip4(10, 0, 0, 2)

SCENARIOS = [
    # test_aggregator_init (:72-82) / test_explode_ipfix_empty_selectors (:895-944): no selectors
    _s("empty_selectors", "tests.rs:895-944", [],
       [("198.51.100.1", 2055, T16 * 1000,
         [ipfix_packet(600, [[(SRC4, k_10_1), (OCTETS, 300)]], T20, 20, 500)])],
       [G("198.51.100.1", T20, (), (), coll_ms=T16 * 1000, templates={(10, 600)}, ports={2055}, domains={500})]),
    # test_aggregator_push_new_ipfix_flow (:84-127)
    _s("push_new_ipfix_flow", "tests.rs:84-127",
       K2 + [(0, OCTETS, 0, OP_ADD), (0, PACKETS, 0, OP_ADD), (0, MIN_TTL, 0, OP_MIN), (0, MAX_TTL, 0, OP_MAX)],
       [(P192_1, 9995, T10_MS, [ipfix_packet(256, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 1000),
                                                     (PACKETS, 10), (MIN_TTL, 64), (MAX_TTL, 128)]], T10, 1, 100)])],
       [G(P192_1, T10, (k_10_1, k_10_2), (1000, 10, 64, 128), coll_ms=T10_MS, templates={(10, 256)}, ports={9995},
          domains={100})]),
    # test_aggregator_push_ipfix_duplicate_flow_key (:129-194): three items of one key; template 256
    # redefined between them (the items' agg fields are (Some, None), (Some, Some), (None, Some))
    _s("push_ipfix_duplicate_flow_key", "tests.rs:129-194",
       K2 + [(0, OCTETS, 0, OP_ADD), (0, TCP_FLAGS, 0, OP_OR)],
       [(P192_1, 9995, T10_MS, [ipfix_packet(256, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 1000)]], T10, 1, 100)]),
        (P192_1, 9995, T10_MS, [ipfix_packet(256, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 500),
                                                     (TCP_FLAGS, tcp(1, 1, 0, 0, 0, 0, 0, 0))]], T10, 2, 100)]),
        (P192_1, 9995, T10_MS, [ipfix_packet(256, [[(SRC4, k_10_1), (DST4, k_10_2),
                                                     (TCP_FLAGS, tcp(0, 1, 0, 0, 0, 0, 1, 1))]], T10, 3, 100)])],
       [G(P192_1, T10, (k_10_1, k_10_2), (1500, tcp(1, 1, 0, 0, 0, 0, 1, 1)), count=3, coll_ms=T10_MS,
          templates={(10, 256)}, ports={9995}, domains={100})]),
    # test_aggregator_push_ipfix_different_flow_keys (:196-241)
    _s("push_ipfix_different_flow_keys", "tests.rs:196-241",
       K2 + [(0, OCTETS, 0, OP_ADD), (0, TCP_FLAGS, 0, OP_OR)],
       [(P192_1, 9995, T10_MS, [ipfix_packet(256, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 1000)]], T10, 1, 100)]),
        (P192_1, 9995, T10_MS, [ipfix_packet(256, [[(SRC4, ip4(20, 0, 0, 1)), (DST4, ip4(20, 0, 0, 2)),
                                                     (OCTETS, 1000)]], T10, 2, 100)])],
       [G(P192_1, T10, (k_10_1, k_10_2), (1000, None), coll_ms=T10_MS, templates={(10, 256)}, ports={9995},
          domains={100}),
        G(P192_1, T10, (ip4(20, 0, 0, 1), ip4(20, 0, 0, 2)), (1000, None), coll_ms=T10_MS, templates={(10, 256)},
          ports={9995}, domains={100})]),
    # test_explode_simple_ipfix_packet (:588-658)
    _s("explode_simple_ipfix_packet", "tests.rs:588-658",
       K2 + [(0, SPORT, 0, OP_KEY), (0, DPORT, 0, OP_KEY), (0, OCTETS, 0, OP_ADD), (0, PACKETS, 0, OP_ADD)],
       [(P192_1, 9995, T10_MS, [ipfix_packet(256, [[(SRC4, k_10_1), (DST4, k_10_2), (SPORT, 80), (DPORT, 443),
                                                     (OCTETS, 1000), (PACKETS, 10)]], T12, 1, 100)])],
       [G(P192_1, T12, (k_10_1, k_10_2, 80, 443), (1000, 10), coll_ms=T10_MS, templates={(10, 256)}, ports={9995},
          domains={100})]),
    # test_explode_ipfix_multiple_records (:660-752): an IPv6 peer
    _s("explode_ipfix_multiple_records", "tests.rs:660-752", K2 + [(0, OCTETS, 0, OP_ADD)],
       [("2001:db8::1", 2055, T11 * 1000,
         [ipfix_packet(300, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 500)],
                             [(SRC4, ip4(10, 0, 0, 3)), (DST4, ip4(10, 0, 0, 4)), (OCTETS, 750)]], T14_30, 5, 200)])],
       [G("2001:db8::1", T14_30, (k_10_1, k_10_2), (500,), coll_ms=T11 * 1000, templates={(10, 300)}, ports={2055},
          domains={200}),
        G("2001:db8::1", T14_30, (ip4(10, 0, 0, 3), ip4(10, 0, 0, 4)), (750,), coll_ms=T11 * 1000,
          templates={(10, 300)}, ports={2055}, domains={200})]),
    # test_explode_ipfix_missing_fields (:829-893), with its sourceIPv6Address c:a:f:e::
    _s("explode_ipfix_missing_fields", "tests.rs:829-893",
       [(0, SRC4, 0, OP_KEY), (0, DST4, 0, OP_KEY), (0, SRC6, 0, OP_KEY), (0, OCTETS, 0, OP_ADD),
        (0, PACKETS, 0, OP_ADD)],
       [("203.0.113.1", 9996, T15 * 1000,
         [ipfix_packet(500, [[(SRC4, k_10_1), (OCTETS, 500), (SRC6, struct.pack(">8H", 0xc, 0xa, 0xf, 0xe, 0, 0, 0, 0))]],
                       T18, 15, 400)])],
       [G("203.0.113.1", T18, (k_10_1, None, struct.pack(">8H", 0xc, 0xa, 0xf, 0xe, 0, 0, 0, 0)), (500, None),
          coll_ms=T15 * 1000, templates={(10, 500)}, ports={9996}, domains={400})]),
    # test_explode_netflowv9_multiple_records (:1018-1110)
    _s("explode_netflowv9_multiple_records", "tests.rs:1018-1110", K2 + [(0, OCTETS, 0, OP_ADD)],
       [("2001:db8::1", 2055, T11 * 1000,
         [nf_packet_of(300, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 500)],
                             [(SRC4, ip4(10, 0, 0, 3)), (DST4, ip4(10, 0, 0, 4)), (OCTETS, 750)]], 2000, T14_30, 5, 200)])],
       [G("2001:db8::1", T14_30, (k_10_1, k_10_2), (500,), flow_type=9, coll_ms=T11 * 1000, sysup=2000,
          templates={(9, 300)}, ports={2055}, domains={200}),
        G("2001:db8::1", T14_30, (ip4(10, 0, 0, 3), ip4(10, 0, 0, 4)), (750,), flow_type=9, coll_ms=T11 * 1000,
          sysup=2000, templates={(9, 300)}, ports={2055}, domains={200})]),
    # test_explode_netflowv9_missing_fields (:1112-1176)
    _s("explode_netflowv9_missing_fields", "tests.rs:1112-1176",
       [(0, SRC4, 0, OP_KEY), (0, DST4, 0, OP_KEY), (0, SRC6, 0, OP_KEY), (0, OCTETS, 0, OP_ADD),
        (0, PACKETS, 0, OP_ADD)],
       [("203.0.113.1", 9996, T15 * 1000,
         [nf_packet_of(500, [[(SRC4, k_10_1), (OCTETS, 500), (SRC6, struct.pack(">8H", 0xc, 0xa, 0xf, 0xe, 0, 0, 0, 0))]],
                       3000, T18, 15, 400)])],
       [G("203.0.113.1", T18, (k_10_1, None, struct.pack(">8H", 0xc, 0xa, 0xf, 0xe, 0, 0, 0, 0)), (500, None),
          flow_type=9, coll_ms=T15 * 1000, sysup=3000, templates={(9, 500)}, ports={9996}, domains={400})]),
    # test_aggregator_push_netflowv9_and_ipfix_different_flow_types (:1178-1261)
    _s("push_netflowv9_and_ipfix_different_flow_types", "tests.rs:1178-1261", K2 + [(0, OCTETS, 0, OP_ADD)],
       [(P192_1, 9995, T10_MS, [ipfix_packet(256, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 1000)]], T10, 1, 100)]),
        (P192_1, 9996, T10_MS, [nf_packet_of(300, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 2000)]], 0, T10, 1, 200)])],
       [G(P192_1, T10, (k_10_1, k_10_2), (1000,), coll_ms=T10_MS, templates={(10, 256)}, ports={9995},
          domains={100}),
        G(P192_1, T10, (k_10_1, k_10_2), (2000,), flow_type=9, coll_ms=T10_MS, templates={(9, 300)}, ports={9996},
          domains={200})]),
    # test_aggregator_push_netflowv9_duplicate_flow_key (:1263-1377)
    _s("push_netflowv9_duplicate_flow_key", "tests.rs:1263-1377", K2 + [(0, OCTETS, 0, OP_ADD), (0, TCP_FLAGS, 0, OP_OR)],
       [(P192_1, 9995, T10_MS, [nf_packet_of(256, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 1000)]], 0, T10, 1, 100)]),
        (P192_1, 9996, T10_MS, [nf_packet_of(257, [[(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, 500),
                                                     (TCP_FLAGS, tcp(1, 1, 0, 0, 0, 0, 0, 0))]], 0, T10, 2, 101)])],
       [G(P192_1, T10, (k_10_1, k_10_2), (1500, tcp(1, 1, 0, 0, 0, 0, 0, 0)), flow_type=9, count=2, coll_ms=T10_MS,
          templates={(9, 256), (9, 257)}, ports={9995, 9996}, domains={100, 101})]),
]


# analytics/src/aggregation.rs window tests: TestItem{key "key1", ts, value} -> one IPFIX message with
# one octetDeltaCount record (the value) per item, all from one peer; TestAggregator's sum is Add.
def _item(ts, value, seq):
    return ipfix_packet(256, [[(OCTETS, value)]], ts, seq, 1)


def window_scenario(name, src, items, emits, flush, late=0):
    peer = "10.11.12.13"
    pushes = [(peer, 4739, 0, [_item(ts, v, i)]) for i, (ts, v) in enumerate(items)]
    grp = lambda ws, total, n, export: G(peer, ws, (), (total,), count=n, export=export, coll_ms=0,  # noqa: E731
                                         templates={(10, 256)}, ports={4739}, domains={1})
    return _s(name, src, [(0, OCTETS, 0, OP_ADD)], pushes,
              [grp(*g) for g in flush], emits=[[grp(*g) for g in e] for e in emits], late=late)


_m = lambda mm, ss=0: T_2025 + 60 * mm + ss  # noqa: E731  2025-01-01T00:mm:ss
_B = 1738671601  # DateTime::from_timestamp_millis(1738671601000), test_buffer_order
WINDOW_SCENARIOS = [
    # get_test_input (:498-576) through test_window_aggregator / _iterator / _stream (:578-683): windows
    # [0:00, 0:01) = 1 + 2, [0:01, 0:02) = 3 + 4 closed by the items at 0:01:30 and 0:02:10, the 0:01:40
    # item late (more than 10 s behind 0:02:10), [0:02, 0:03) = 5 closed by 0:03:10, [0:03, 0:04) = 5 flushed
    window_scenario("window_aggregator", "aggregation.rs:498-683",
                    [(_m(0), 1), (_m(1), 3), (_m(0, 55), 2), (_m(1, 30), 4), (_m(2, 10), 5), (_m(1, 40), 5),
                     (_m(3, 10), 5)],
                    [[], [], [], [(_m(0), 3, 2, (_m(0), _m(0, 55)))], [(_m(1), 7, 2, (_m(1), _m(1, 30)))], [],
                     [(_m(2), 5, 1, _m(2, 10))]],
                    [(_m(3), 5, 1, _m(3, 10))], late=1),
    # test_buffer_order (:685-744)
    window_scenario("buffer_order", "aggregation.rs:685-744",
                    [(_B, 1), (_B + 30, 2), (_B + 30, 3), (_B + 60, 4), (_B + 180, 5)],
                    [[], [], [], [], [(minute(_B), 6, 3, (_B, _B + 30)), (minute(_B) + 60, 4, 1, _B + 60)]],
                    [(minute(_B) + 180, 5, 1, _B + 180)]),
    # test_empty_windows (:746-788): no window for the empty minute between the items
    window_scenario("empty_windows", "aggregation.rs:746-788", [(_m(0), 1), (_m(2), 2)],
                    [[], [(_m(0), 1, 1, _m(0))]], [(_m(2), 2, 1, _m(2))]),
]

# test_reduce_add_operations (:243-337) in full: FlowCacheRecord::reduce of record1 with record2
# (the windowed device path never merges records an hour apart; this pins the oracle's reduce,
# and the device's values through REDUCE_* above)
REDUCE_FULL_R1 = dict(ports={9995, 1234}, domains={100, 105}, templates={(10, 256)}, min_export=T10, max_export=T10,
                      min_coll=T10_MS, max_coll=T10_MS, max_sysup=1000, count=5)
REDUCE_FULL_R2 = dict(ports={9996}, domains={101}, templates={(10, 257)}, min_export=T11, max_export=T11,
                      min_coll=T11 * 1000, max_coll=T11 * 1000, max_sysup=2000, count=1)
REDUCE_FULL_EXPECTED = dict(ports={9995, 1234, 9996}, domains={100, 105, 101}, templates={(10, 256), (10, 257)},
                            min_export=T10, max_export=T11, min_coll=T10_MS, max_coll=T11 * 1000, max_sysup=2000,
                            count=6)

# test_ipfix_into_flowinfo_with_extra_fields (:339-460) / test_netflowv9_... (:462-586): the group
# (ports {9995, 9996}, domains {1, 2}, templates {256, 257}, 3 records, octets 1000, packets 10,
# export 2025-07-02T10:00:00Z, collection 10:00:05Z, NetFlow v9 sys-up time 5000) as two pushes;
# shard 5, sequence number 42.  Expected fields: the test's (key, agg, originalFlowsPresent,
# min/maxExportSeconds, collectionTimeMilliseconds, windowStart/End, the sets), plus the
# originalExporterIPv4Address the actor adds (actor.rs:222-225) for the peer 192.168.1.100.
FLOWINFO_PEER = "192.168.1.100"


def flowinfo_scenario(flow_type):
    fields = K2 + [(0, OCTETS, 0, OP_ADD), (0, PACKETS, 0, OP_ADD)]
    r = lambda o, p: [(SRC4, k_10_1), (DST4, k_10_2), (OCTETS, o), (PACKETS, p)]  # noqa: E731
    if flow_type == 10:
        a = ipfix_packet(256, [r(500, 5)], T_JUL2_10, 1, 1)
        b = ipfix_packet(257, [r(300, 3), r(200, 2)], T_JUL2_10, 2, 2)
    else:
        a = nf_packet_of(256, [r(500, 5)], 5000, T_JUL2_10, 1, 1)
        b = nf_packet_of(257, [r(300, 3), r(200, 2)], 4000, T_JUL2_10, 2, 2)
    coll = T_JUL2_10_05 * 1000
    return fields, [(FLOWINFO_PEER, 9995, coll, [a]), (FLOWINFO_PEER, 9996, coll, [b])]


def _dt(t):
    import datetime
    return datetime.datetime.fromtimestamp(t, datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


FLOWINFO_EXPECTED_FIELDS = [
    {"sourceIPv4Address": "10.0.0.1"}, {"destinationIPv4Address": "10.0.0.2"},
    {"octetDeltaCount": 1000}, {"packetDeltaCount": 10},
    {"originalFlowsPresent": 3}, {"minExportSeconds": _dt(T_JUL2_10)}, {"maxExportSeconds": _dt(T_JUL2_10)},
    {"collectionTimeMilliseconds": _dt(T_JUL2_10_05)},
    {"NetGauze": {"windowStart": "2025-07-02T10:00:00Z"}}, {"NetGauze": {"windowEnd": "2025-07-02T10:01:00Z"}},
    {"NetGauze": {"originalExporterTransportPort": 9995}}, {"NetGauze": {"originalExporterTransportPort": 9996}},
    {"originalObservationDomainId": 1}, {"originalObservationDomainId": 2},
    {"NetGauze": {"originalTemplateId": 256}}, {"NetGauze": {"originalTemplateId": 257}},
    {"originalExporterIPv4Address": FLOWINFO_PEER},  # actor.rs:222-225
]


# ---------------------------------------------------------------------------------------------
# Field arithmetic KATs of crates/flow-pkt/src/lib.rs:359-615: Field::{add,min,max,bitwise_or}_field
# (and the *_assign_field forms, same results) on two fields of one IE, and the
# FieldOperationError::Inapplicable* pair for a field of another IE.  IEs as (pen, id, name):
# VMware (PEN 6876) averageLatency 958 unsigned32, algControlFlowId 955 unsigned64 identifier.
# Each entry: (test, src, op, ie, lhs, rhs, expected, other_ie, error variant).
# ---------------------------------------------------------------------------------------------
IE_OCTETS = (0, 1, "octetDeltaCount")
IE_PACKETS = (0, 2, "packetDeltaCount")
IE_TCP_FLAGS = (0, 6, "tcpControlBits")
IE_PROTOCOL = (0, 4, "protocolIdentifier")
IE_VMW_LATENCY = (6876, 958, "averageLatency")
IE_VMW_ALG_FLOW = (6876, 955, "algControlFlowId")
ICMP, IGMP = 1, 2  # protocolIdentifier::ICMP / IGMP

FIELD_OP_KATS = [
    ("test_field_add", "lib.rs:359-382", OP_ADD, IE_OCTETS, 100, 200, 300, IE_PACKETS, "InapplicableAdd"),
    ("test_field_min", "lib.rs:383-406", OP_MIN, IE_OCTETS, 100, 200, 100, IE_PACKETS, "InapplicableMin"),
    ("test_field_max", "lib.rs:407-430", OP_MAX, IE_OCTETS, 100, 200, 200, IE_PACKETS, "InapplicableMax"),
    ("test_field_bitwise_or", "lib.rs:431-454", OP_OR, IE_OCTETS, 100, 200, 236, IE_PACKETS, "InapplicableBitwise"),
    ("test_field_bitwise_or_tcp_control_bits", "lib.rs:455-478", OP_OR, IE_TCP_FLAGS, 0x01, 0x02, 0x03, IE_PACKETS,
     "InapplicableBitwise"),
    ("test_field_bitwise_or_protocol_identifier", "lib.rs:479-502", OP_OR, IE_PROTOCOL, ICMP, IGMP, 0x03, IE_PACKETS,
     "InapplicableBitwise"),
    ("test_vmware_ops", "lib.rs:503-526", OP_ADD, IE_VMW_LATENCY, 100, 200, 300, IE_VMW_ALG_FLOW, "InapplicableAdd"),
    ("test_vendor_field_add", "lib.rs:527-548", OP_ADD, IE_VMW_LATENCY, 100, 200, 300, IE_VMW_ALG_FLOW,
     "InapplicableAdd"),
    ("test_vendor_field_min", "lib.rs:549-570", OP_MIN, IE_VMW_LATENCY, 100, 200, 100, IE_VMW_ALG_FLOW,
     "InapplicableMin"),
    ("test_vendor_field_max", "lib.rs:571-592", OP_MAX, IE_VMW_LATENCY, 100, 200, 200, IE_VMW_ALG_FLOW,
     "InapplicableMax"),
    ("test_vendor_field_bitwise_or", "lib.rs:593-615", OP_OR, IE_VMW_ALG_FLOW, 100, 200, 236, IE_VMW_LATENCY,
     "InapplicableBitwise"),
]

# IE::supports_{arithmetic,bitwise,comparison}_ops asserts of lib.rs:267-358, by IE name:
# (arithmetic, bitwise, comparison); None where the reference test asserts nothing.
SUPPORTS_KATS = {
    "mplsLabelStackSection": (False, True, False), "paddingOctets": (False, True, False),
    "destinationIPv4PrefixLength": (True, True, True), "flowActiveTimeout": (True, True, True),
    "distinctCountOfSourceIPv4Address": (True, True, True), "postMCastPacketDeltaCount": (True, True, True),
    "ipv6ExtensionHeadersFull": (False, True, False), "mibObjectValueInteger": (True, True, True),
    "absoluteError": (True, None, None),
    "ipClassOfService": (False, True, True), "egressInterface": (False, True, True),
    "forwardingStatus": (False, True, True), "dataRecordsReliability": (False, True, False),
    "observationTimeSeconds": (False, False, True), "observationTimeMilliseconds": (False, False, True),
    "observationTimeNanoseconds": (False, False, True), "observationTimeMicroseconds": (False, False, True),
    "sourceIPv4Address": (False, True, True), "sourceIPv6Address": (False, True, True),
    "bgpSourceCommunityList": (False, None, None), "ipv6ExtensionHeaderTypeCountList": (False, None, None),
    "subTemplateMultiList": (False, None, None),
}

_WIDTH = {(0, 1): 8, (0, 2): 8, (0, 6): 2, (0, 4): 1, (6876, 958): 4, (6876, 955): 8}


def etset(tid, fields):
    """An IPFIX template set of (pen, id, length) specifiers (enterprise bit set for pen != 0)."""
    spec = b"".join(struct.pack(">HH", i | 0x8000, n) + struct.pack(">I", p) if p else struct.pack(">HH", i, n)
                    for p, i, n in fields)
    body = struct.pack(">HH", tid, len(fields)) + spec
    return struct.pack(">HH", 2, 4 + len(body)) + body


def _field_record(ie, v):
    w = _WIDTH[ie[:2]]
    return struct.pack(">I", k_10_1) + v.to_bytes(w, "big")


def field_op_scenario(kat):
    """One FIELD_OP_KATS entry as two records of one group: key sourceIPv4Address, the IE under the
    KAT's op; lhs arrives first (Ord::min keeps it on equality, Ord::max takes the rhs).  Then the
    Inapplicable pair: an aggregator with the op on both IEs, one record carrying only the first
    IE and one only the other -- the reduce never combines two IEs (FieldRef lookup, types.rs:82-100;
    aggregator.rs:159-198), so each keeps its own value."""
    name, src, op, ie, lhs, rhs, exp, other, _err = kat
    p, i, _ = ie
    tpl = [(0, SRC4, 4), (p, i, _WIDTH[ie[:2]])]
    msg = ipfix_msg([etset(300, tpl), dset(300, [_field_record(ie, lhs), _field_record(ie, rhs)])], T10, 1, 100)
    same = _s("fieldop_" + name, src, [(0, SRC4, 0, OP_KEY), (p, i, 0, op)],
              [(P192_1, 9995, T10_MS, [msg])],
              [G(P192_1, T10, (k_10_1,), (exp,), count=2, coll_ms=T10_MS, templates={(10, 300)}, ports={9995},
                 domains={100})])
    op2 = other[:2]
    # algControlFlowId has identifier semantics: no Add (generator.rs:1176-1181); Max there instead
    other_op = OP_MAX if (op == OP_ADD and other == IE_VMW_ALG_FLOW) else op
    tpl2 = [(0, SRC4, 4), (op2[0], op2[1], _WIDTH[op2])]
    msg2 = ipfix_msg([etset(300, tpl), etset(301, tpl2), dset(300, [_field_record(ie, lhs)]),
                      dset(301, [_field_record(other, rhs)])], T10, 2, 100)
    pair = _s("fieldop_pair_" + name, src, [(0, SRC4, 0, OP_KEY), (p, i, 0, op), (op2[0], op2[1], 0, other_op)],
              [(P192_1, 9995, T10_MS, [msg2])],
              [G(P192_1, T10, (k_10_1,), (lhs, rhs), count=2, coll_ms=T10_MS, templates={(10, 300), (10, 301)},
                 ports={9995}, domains={100})])
    return [same, pair]


FIELD_OP_SCENARIOS = [s for kat in FIELD_OP_KATS for s in field_op_scenario(kat)]

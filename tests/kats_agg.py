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

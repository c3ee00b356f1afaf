"""GPU parity of the device flow aggregation (include/ngz/flow_aggregate.h) against
oracle/ngz_agg_oracle.py, a restatement of the collector's FlowAggregator /
WindowAggregator (aggregator.rs:68-354, analytics/src/aggregation.rs:124-185),
pinned by the reference's aggregation unit tests (tests/kats_agg.py).

Every comparison is exact: group set, key values, aggregated values (adds wrap at the
IE's Rust width), record counts, export/collection time bounds, sys-up time and the
template / port / observation-domain sets."""
import os
import struct
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import golden_io  # noqa: E402
import kats_agg as K  # noqa: E402
import ngz_agg_oracle as A  # noqa: E402

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

OK, ADD, MN, MX, OR = K.OP_KEY, K.OP_ADD, K.OP_MIN, K.OP_MAX, K.OP_OR
# rendering of flushed values per IE (pen, id): byte-like IEs stay bytes
KINDS = {(0, 27): "bytes", (0, 28): "bytes", (0, 56): "bytes", (0, 80): "bytes"}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.aggregate import FlowAggregator  # noqa: F401  (loads libngz.so, fails loudly)
    return torch.device("cuda:0")


def ipfix_msg(sets, export_time, seq=1, domain=7):
    body = b"".join(sets)
    return struct.pack(">HHIII", 10, 16 + len(body), export_time, seq, domain) + body


def tset(tid, fields):
    body = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, n) for i, n in fields)
    return struct.pack(">HH", 2, 4 + len(body)) + body


def dset(tid, recs):
    body = b"".join(recs)
    return struct.pack(">HH", tid, 4 + len(body)) + body


def norm(groups):
    out = {}
    for g in groups:
        k = (g["window_start"], g["flow_type"], tuple(g["key"]))
        assert k not in out, k
        out[k] = (tuple(g["vals"]), g["record_count"], g["min_export"], g["max_export"], g["max_sysup"],
                  g["min_coll"], g["max_coll"], frozenset(g["templates"]), frozenset(g["ports"]),
                  frozenset(g["domains"]))
    return out


def run_device(fields, batches, port=4739, coll=1_700_000_000_000, lateness_s=10, capacity=1 << 16):
    """batches: list of lists of datagrams, decoded in order on one codec (one peer)."""
    from netgauze_amd.aggregate import FlowAggregator
    from netgauze_amd.flow import FlowInfoCodec
    codec = FlowInfoCodec()
    agg = FlowAggregator(fields, lateness_s=lateness_s, capacity=capacity, kinds=KINDS)
    late = 0
    for b in batches:
        batch = codec.decode_datagrams(b)
        late += agg.push(batch, port, coll)
    groups = agg.flush()
    assert agg.n_groups() == 0
    agg.close()
    codec.close()
    return groups, late


def run_oracle(fields, batches, port=4739, coll=1_700_000_000_000, lateness_s=10):
    o = A.aggregate_datagrams(fields, [d for b in batches for d in b], peer_port=port, collection_ms=coll,
                              lateness_s=lateness_s)
    late = o.late
    return o.flush(), late


def check(fields, batches, **kw):
    g_dev, late_dev = run_device(fields, batches, **kw)
    kw.pop("capacity", None)
    g_ref, late_ref = run_oracle(fields, batches, **kw)
    assert late_dev == late_ref
    a, b = norm(g_dev), norm(g_ref)
    assert set(a) == set(b), (len(a), len(b), sorted(set(a) ^ set(b))[:5])
    for k in b:
        assert a[k] == b[k], (k, a[k], b[k])
    return g_dev


def test_kat_repeating_ie_fields(dev):
    d = [ipfix_msg([tset(400, K.REPEAT_TEMPLATE), dset(400, [K.REPEAT_RECORD])], K.T_2025_01_01_16, domain=300)]
    (g,) = check(K.REPEAT_FIELDS, [d])
    for k, v in K.REPEAT_EXPECTED.items():
        assert g[k] == v, k


def test_kat_missing_fields(dev):
    d = [ipfix_msg([tset(300, K.MISSING_TEMPLATE), dset(300, [K.MISSING_RECORD])], 1_700_000_000)]
    (g,) = check(K.MISSING_FIELDS, [d])
    for k, v in K.MISSING_EXPECTED.items():
        assert g[k] == v, k


def test_kat_reduce_operations(dev):
    d = [ipfix_msg([tset(256, K.REDUCE_TEMPLATE_1), tset(257, K.REDUCE_TEMPLATE_2),
                    dset(256, [K.REDUCE_WIRE_1]), dset(257, [K.REDUCE_WIRE_2])], 1_700_000_000)]
    (g,) = check(K.REDUCE_FIELDS, [d])
    assert g["vals"] == K.REDUCE_EXPECTED and g["record_count"] == 2


def test_wrapping_add_and_signed_min_max(dev):
    # u8 adds wrap (ipTTL-like unsigned8 IE 192 ipTTL), signed32 IE 434 (mibObjectValueInteger) min/max
    tpl = [(192, 1), (434, 4), (1, 8)]
    recs = [struct.pack(">BiQ", 200, -5, 1), struct.pack(">BiQ", 100, 7, 2), struct.pack(">BiQ", 250, -9, 3)]
    d = [ipfix_msg([tset(500, tpl), dset(500, recs)], 1_700_000_000)]
    fields = [(0, 192, 0, ADD), (0, 434, 0, MN), (0, 434, 0, MX), (0, 1, 0, ADD)]
    kinds = dict(KINDS)
    from netgauze_amd.aggregate import FlowAggregator
    from netgauze_amd.flow import FlowInfoCodec
    codec = FlowInfoCodec()
    agg = FlowAggregator(fields, kinds={**kinds, (0, 434): "sint"})
    agg.push(codec.decode_datagrams(d))
    (g,) = agg.flush()
    assert g["vals"] == ((200 + 100 + 250) & 0xFF, -9, 7, 6)
    o = A.aggregate_datagrams(fields, d).flush()
    assert o[0]["vals"] == g["vals"]


def t20_datagrams(n, rec_per_msg, times, seed_first=0):
    from netgauze_amd import synth
    rec = synth.t20_records(n, first=seed_first)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64, rec_per_msg=rec_per_msg)
    b = bytes(buf.numpy())
    out = []
    for i, (o, ln) in enumerate(zip(offs.tolist(), lens.tolist())):
        m = bytearray(b[o:o + ln])
        m[4:8] = struct.pack(">I", times[i % len(times)] + 60 * (i // len(times)))
        out.append(bytes(m))
    return [synth.template_message()] + out


T20_AGG = [(0, 1, 0, ADD), (0, 2, 0, ADD), (0, 6, 0, OR), (0, 22, 0, MN), (0, 21, 0, MX), (0, 16, 0, MX),
           (0, 10, 0, MN)]


@pytest.mark.parametrize("keys", [
    [(0, 4, 0, OK), (0, 61, 0, OK)],                    # 6 groups per window: heavy atomic contention
    [(0, 11, 0, OK)],                                   # destination port: mostly singleton groups
    [(0, 8, 0, OK), (0, 12, 0, OK), (0, 7, 0, OK), (0, 11, 0, OK), (0, 4, 0, OK)],  # 5-tuple
])
def test_t20_groups_windows_lateness(dev, keys):
    """T20 messages whose export times go back and forth: late messages dropped, minute windows."""
    times = [1_700_000_010, 1_700_000_030, 1_700_000_015, 1_700_000_045, 1_700_000_020, 1_700_000_050,
             1_700_000_061, 1_700_000_049]
    d = t20_datagrams(6000, 100, times)
    g = check(keys + T20_AGG, [d[:25], d[25:]])
    assert len(g) > 1


def test_t20_multi_port_collection_times(dev):
    """Two pushes with different peer ports and collection times: port sets and collection bounds."""
    from netgauze_amd.aggregate import FlowAggregator
    from netgauze_amd.flow import FlowInfoCodec
    keys = [(0, 4, 0, OK)]
    d = t20_datagrams(3000, 300, [1_700_000_000])
    codec = FlowInfoCodec()
    agg = FlowAggregator(keys + T20_AGG, kinds=KINDS)
    agg.push(codec.decode_datagrams(d[:6]), 1000, 5_000)
    agg.push(codec.decode_datagrams(d[6:]), 2000, 9_000)
    o = A.FlowAggregatorOracle(keys + T20_AGG)
    import ngz_oracle as O
    oc = O.FlowInfoCodec()
    for i, x in enumerate(d):
        pkt = oc.decode(bytearray(x))
        if pkt is not None:
            o.push_packet(pkt, 1000 if i < 6 else 2000, 5_000 if i < 6 else 9_000)
    assert norm(agg.flush()) == norm(o.flush())


def peers_of(name):
    groups = {}
    for src, sp, dst, dp, payload in golden_io.datagrams(name):
        groups.setdefault((src, sp, dst, dp), []).append(payload)
    return groups


GOLDEN_AGG = [(0, 8, 0, OK), (0, 12, 0, OK), (0, 27, 0, OK), (0, 4, 0, OK), (0, 10, 0, OK),
              (0, 1, 0, ADD), (0, 2, 0, ADD), (0, 6, 0, OR), (0, 22, 0, MN), (0, 21, 0, MX), (0, 7, 0, MX),
              (0, 56, 0, OR)]


# a key that packs into the 63-bit tag (exact, no verify pass): protocol + source port
GOLDEN_AGG_PACKED = [(0, 4, 0, OK), (0, 7, 0, OK), (0, 1, 0, ADD), (0, 2, 0, ADD), (0, 6, 0, OR),
                     (0, 22, 0, MN), (0, 21, 0, MX)]


@pytest.mark.parametrize("fields", ["wide", "packed"])
@pytest.mark.parametrize("name", [c[0] for c in golden_io.cases()])
def test_reference_captures(dev, name, fields):
    """Every reference capture, per exporter peer (IPFIX and NetFlow v9, options data,
    several templates and observation domains), in two batches."""
    from netgauze_amd.aggregate import AggError
    sel = GOLDEN_AGG if fields == "wide" else GOLDEN_AGG_PACKED
    for key, dgrams in peers_of(name).items():
        h = len(dgrams) // 2
        try:
            check(sel, [dgrams[:h], dgrams[h:]], port=key[1], lateness_s=60)
        except AggError as e:
            # selected fields that are variable-length in some template are not on the device yet
            assert "variable-length" in str(e), e


def test_wave_preaggregation_bytes_and_presence(dev):
    """Low-cardinality keys (wave pre-aggregation path) with a byte-wise OR (mac), a
    signed min and fields present in only one of two templates."""
    import random
    rnd = random.Random(7)
    t1 = [(8, 4), (56, 6), (1, 8), (434, 4)]
    t2 = [(8, 4), (2, 8)]
    r1 = [struct.pack(">I6sQi", rnd.choice([1, 2]), bytes(rnd.getrandbits(8) for _ in range(6)),
                      rnd.getrandbits(64), rnd.randint(-2**31, 2**31 - 1)) for _ in range(700)]
    r2 = [struct.pack(">IQ", rnd.choice([1, 2, 3]), rnd.getrandbits(64)) for _ in range(500)]
    d = [ipfix_msg([tset(600, t1), tset(601, t2)], 1_700_000_000)]
    for i in range(0, 700, 100):
        d.append(ipfix_msg([dset(600, r1[i:i + 100]), dset(601, r2[i:i + 100] if i < 500 else [])]
                           if i < 500 else [dset(600, r1[i:i + 100])], 1_700_000_000 + i // 100))
    fields = [(0, 8, 0, OK), (0, 56, 0, OR), (0, 1, 0, ADD), (0, 2, 0, MX), (0, 434, 0, MN)]
    from netgauze_amd.aggregate import FlowAggregator
    from netgauze_amd.flow import FlowInfoCodec
    codec = FlowInfoCodec()
    agg = FlowAggregator(fields, kinds={**KINDS, (0, 434): "sint"})
    agg.push(codec.decode_datagrams(d))
    got = norm(agg.flush())
    ref = norm(A.aggregate_datagrams(fields, d, collection_ms=0).flush())
    assert set(got) == set(ref) and len(got) == 3
    for k in ref:
        assert got[k] == ref[k], (k, got[k], ref[k])


def test_table_full_and_flush_buffer_errors(dev):
    """A group table that fills up reports NGZ_AGG_E_OVERFLOW (no hang); a flush buffer that is
    too small is refused without emptying the table."""
    import numpy as np
    from netgauze_amd import _lib
    from netgauze_amd.aggregate import AggError, FlowAggregator, lib
    from netgauze_amd.flow import FlowInfoCodec
    d = t20_datagrams(5000, 500, [1_700_000_000])
    codec = FlowInfoCodec()
    agg = FlowAggregator([(0, 8, 0, OK), (0, 12, 0, OK)] + T20_AGG, capacity=16)  # 2048 slots
    with pytest.raises(AggError, match="group table full"):
        agg.push(codec.decode_datagrams(d))
    agg2 = FlowAggregator([(0, 4, 0, OK)] + T20_AGG)
    agg2.push(codec.decode_datagrams(d[:3]))
    n = agg2.n_groups()
    assert n == 6  # 3 protocols x 2 minute windows (the two data messages are 60 s apart)
    rb = agg2.layout()[0]
    buf = np.zeros(rb * n - 1, dtype=np.uint8)
    assert lib().ngz_agg_flush(agg2._h, buf.ctypes.data, buf.nbytes) == -1  # NGZ_E_INVALID
    assert agg2.n_groups() == n
    assert len(agg2.flush()) == n and agg2.n_groups() == 0


def test_kat_netflowv9_explode(dev):
    (g,) = check(K.NF_FIELDS, [[K.nf_packet()]], port=9995, coll=K.T_2025_01_01_10_MS)
    for k, v in K.NF_EXPECTED.items():
        assert g[k] == v, k


def test_flow_type_separates_groups(dev):
    """The same key exported over NetFlow v9 and IPFIX by one peer makes two groups
    (FlowCacheKey.flow_type; reference test_aggregator_push_netflowv9_and_ipfix_different_flow_types,
    aggregator/tests.rs:1179-1262)."""
    ipfix = ipfix_msg([tset(256, K.NF_TEMPLATE), dset(256, [K.NF_RECORD, K.NF_RECORD])], K.T_2025_01_01_12,
                      domain=100)
    g = check(K.NF_FIELDS, [[K.nf_packet(), ipfix]], port=9995, coll=K.T_2025_01_01_10_MS)
    assert sorted((x["flow_type"], x["record_count"], x["vals"]) for x in g) == [(9, 1, (1000, 10)),
                                                                                 (10, 2, (2000, 20))]

"""CPU: the aggregation oracle reproduces the reference's aggregation unit tests
(tests/kats_agg.py, from aggregator/tests.rs) and the window/lateness rules of
analytics/src/aggregation.rs:124-172."""
import os
import struct
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import kats_agg as K  # noqa: E402
import ngz_agg_oracle as A  # noqa: E402


def ipfix_msg(sets, export_time, seq=1, domain=7):
    body = b"".join(sets)
    return struct.pack(">HHIII", 10, 16 + len(body), export_time, seq, domain) + body


def tset(tid, fields):
    body = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, n) for i, n in fields)
    return struct.pack(">HH", 2, 4 + len(body)) + body


def dset(tid, recs):
    body = b"".join(recs)
    return struct.pack(">HH", tid, 4 + len(body)) + body


def test_repeating_ie_fields():
    d = [ipfix_msg([tset(400, K.REPEAT_TEMPLATE), dset(400, [K.REPEAT_RECORD])], K.T_2025_01_01_16, domain=300)]
    (g,) = A.aggregate_datagrams(K.REPEAT_FIELDS, d, peer_port=4739).flush()
    for k, v in K.REPEAT_EXPECTED.items():
        assert g[k] == v, k


def test_missing_fields():
    d = [ipfix_msg([tset(300, K.MISSING_TEMPLATE), dset(300, [K.MISSING_RECORD])], 1_700_000_000)]
    (g,) = A.aggregate_datagrams(K.MISSING_FIELDS, d).flush()
    for k, v in K.MISSING_EXPECTED.items():
        assert g[k] == v, k


def test_reduce_add_operations():
    d = [ipfix_msg([tset(256, K.REDUCE_TEMPLATE_1), tset(257, K.REDUCE_TEMPLATE_2),
                    dset(256, [K.REDUCE_WIRE_1]), dset(257, [K.REDUCE_WIRE_2])], 1_700_000_000)]
    (g,) = A.aggregate_datagrams(K.REDUCE_FIELDS, d).flush()
    assert g["vals"] == K.REDUCE_EXPECTED
    assert g["record_count"] == 2 and g["templates"] == {(10, 256), (10, 257)}


def test_add_wraps_at_rust_width():
    # release-mode `*lhs += *rhs` on u8 / i8 wraps
    ie_u8 = type("IE", (), {"dtype": "unsigned8"})()
    ie_i8 = type("IE", (), {"dtype": "signed8"})()
    assert A.reduce_value(ie_u8, A.OP_ADD, 200, 100) == 44
    assert A.reduce_value(ie_i8, A.OP_ADD, 100, 100) == -56
    assert A.reduce_value(ie_u8, A.OP_OR, b"\x01\x02", b"\x10\x20\x30") == b"\x11\x22"


def test_lateness_and_minute_windows():
    t = [tset(256, K.MISSING_TEMPLATE)]
    rec = [dset(256, [K.MISSING_RECORD])]
    times = [1_700_000_150, 1_700_000_180, 1_700_000_165, 1_700_000_169, 1_700_000_171]
    d = [ipfix_msg(t + rec, times[0])] + [ipfix_msg(rec, x) for x in times[1:]]
    agg = A.aggregate_datagrams(K.MISSING_FIELDS, d, lateness_s=10)
    assert agg.late == 2  # 165 and 169 are more than 10 s behind 180
    # event time 180: cutoff = get_window_start(180 - 10) - 60 = 100 closes the first window
    # (aggregation.rs:154-160); the second stays active until the flush
    closed = [(g["window_start"], g["record_count"]) for g in agg.emit()]
    assert closed == [(1_700_000_100, 1)] and agg.emit() == []
    got = sorted((g["window_start"], g["record_count"]) for g in agg.flush())
    assert got == [(1_700_000_160, 2)]  # minute floors


def test_netflowv9_explode():
    agg = A.aggregate_datagrams(K.NF_FIELDS, [K.nf_packet()], peer_port=9995, collection_ms=K.T_2025_01_01_10_MS)
    (g,) = agg.flush()
    for k, v in K.NF_EXPECTED.items():
        assert g[k] == v, k


def test_float_and_enum_orders():
    """Min / Max follow the Rust Ord of each Field type; Ord::min keeps the group's value
    on equality, Ord::max takes the record's."""
    import ngz_oracle as O
    f64 = next(ie for ie in O.REGISTRY.by_key.values() if ie.dtype == "float64")
    nan = float("nan")
    assert A.reduce_value(f64, A.OP_MIN, 1.0, nan) == 1.0          # NaN is the greatest
    assert A.reduce_value(f64, A.OP_MAX, 1.0, nan) != A.reduce_value(f64, A.OP_MAX, 1.0, nan)  # -> NaN
    import math
    assert math.copysign(1, A.reduce_value(f64, A.OP_MIN, 0.0, -0.0)) == 1    # equal: keep lhs
    assert math.copysign(1, A.reduce_value(f64, A.OP_MAX, 0.0, -0.0)) == -1   # equal: take rhs
    f32ie = type("IE", (), {"dtype": "float32", "kind": "iana", "id": 0, "subreg": None})()  # no float32 IE is registered
    assert A.reduce_value(f32ie, A.OP_ADD, 16777216.0, 1.0) == 16777216.0  # f32 rounding
    assert A.reduce_value(f64, A.OP_ADD, 16777216.0, 1.0) == 16777217.0
    proto = O.REGISTRY.lookup(0, 4)  # protocolIdentifier: sub-registry enum
    unassigned = next(v for v in range(256) if v not in {x for x, _ in proto.subreg["entries"]})
    assert A.reduce_value(proto, A.OP_MAX, 200 if 200 in {x for x, _ in proto.subreg["entries"]} else 6,
                          unassigned) == unassigned  # Unassigned(x) after every registered variant
    assert A.reduce_value(proto, A.OP_MIN, 147, unassigned) == 147  # registered 147 < Unassigned(148)
    assert A.reduce_value(proto, A.OP_MIN, 250, unassigned) == unassigned  # Unassigned(148) < Unassigned(250)
    tcp = O.REGISTRY.lookup(0, 6)
    assert A.reduce_value(tcp, A.OP_MAX, 0x01, 0x80) == 0x01  # FIN (bit 0) outranks CWR (bit 7)
    assert A.reduce_value(tcp, A.OP_MIN, 0x02, 0x01) == 0x02  # {SYN} < {FIN}


def test_nested_and_byte_orders():
    """forwardingStatus (nested reason codes, generator_sub_registries.rs:96-140): the outer
    variant per 64-value group, then the reason enum's discriminant (Unassigned(x) = last
    declared reason + 1), then x; values from 256 are the outer Unassigned(x), after every
    group.  Box<[u8]> (lists) order lexicographically, a prefix first; octet-array OR keeps
    the group's length (zip)."""
    import ngz_oracle as O
    fwd = O.REGISTRY.lookup(0, 89)
    assert fwd.subreg["kind"] == "nested"
    mn = lambda a, b: A.reduce_value(fwd, A.OP_MIN, a, b)  # noqa: E731
    mx = lambda a, b: A.reduce_value(fwd, A.OP_MAX, a, b)  # noqa: E731
    assert mn(69, 68) == 68          # Forwarded: reason 68 < Unassigned(69)
    assert mn(100, 128) == 100       # Forwarded(..) < Dropped(..)
    assert mx(300, 255) == 300       # Unassigned(300) after Consumed(Unassigned(255))
    assert mn(3, 64) == 3            # Unknown(Unassigned(3)) < Forwarded(Unknown)
    assert mx(144, 143) == 144       # Dropped: Unassigned(144) > Hardware (143)
    blist = O.REGISTRY.lookup(0, 291)
    assert A.reduce_value(blist, A.OP_MIN, b"\x01\x02", b"\x01") == b"\x01"      # a prefix is less
    assert A.reduce_value(blist, A.OP_MAX, b"\x02", b"\x01\xff\xff") == b"\x02"  # first byte decides
    octets = O.REGISTRY.lookup(0, 210)
    assert A.reduce_value(octets, A.OP_OR, b"\x01\x00", b"\x10\x20\x30") == b"\x11\x20"
    assert A.reduce_value(octets, A.OP_OR, b"\x01\x00\x00", b"\x02") == b"\x03\x00\x00"


def run_oracle_scenario(sc):
    """Pushes of a kats_agg scenario through the oracle (one codec per peer address, one shard)."""
    import ngz_oracle as O
    agg = A.FlowAggregatorOracle(sc["fields"], sc["window_s"], sc["lateness_s"])
    codecs, emits = {}, []
    for ip, port, coll, dgrams in sc["pushes"]:
        codec = codecs.setdefault((ip, port), O.FlowInfoCodec())
        A.aggregate_datagrams(sc["fields"], dgrams, port, coll, peer_ip=ip, agg=agg, codec=codec)
        emits.append(agg.emit())
    return agg, emits, agg.flush()


def _sorted(groups):
    return sorted(groups, key=lambda g: repr((g["peer"], g["window_start"], g["flow_type"], g["key"])))


@pytest.mark.parametrize("sc", K.SCENARIOS + K.WINDOW_SCENARIOS, ids=lambda s: s["name"])
def test_reference_scenarios(sc):
    """aggregator/tests.rs and analytics aggregation.rs tests, as wire-level scenarios: the
    expected cache entries / windows, the late items, and the windows each push closes."""
    agg, emits, flushed = run_oracle_scenario(sc)
    assert agg.late == sc["late"]
    assert _sorted(flushed) == _sorted(sc["flush"])
    if sc["emits"] is not None:
        assert len(emits) == len(sc["emits"])
        for got, exp in zip(emits, sc["emits"]):
            assert _sorted(got) == _sorted(exp)


def test_reduce_full_reference_vector():
    """test_reduce_add_operations (tests.rs:243-337) in full: sets, time bounds, sys-up time,
    count and the aggregated values of FlowCacheRecord::reduce."""
    import ngz_oracle as O
    o = A.FlowAggregatorOracle(K.REDUCE_FIELDS)
    ies = [O.REGISTRY.lookup(0, ie) for _p, ie, _i, _op in K.REDUCE_FIELDS]
    lhs = dict(K.REDUCE_FULL_R1, vals=[None if v is None else (ie, v) for ie, v in zip(ies, K.REDUCE_R1)])
    rhs = dict(K.REDUCE_FULL_R2, vals=[None if v is None else (ie, v) for ie, v in zip(ies, K.REDUCE_R2)])
    lhs = {k: (set(v) if isinstance(v, set) else v) for k, v in lhs.items()}
    o.reduce(lhs, rhs)
    for k, v in K.REDUCE_FULL_EXPECTED.items():
        assert lhs[k] == v, k
    assert tuple(None if v is None else v[1] for v in lhs["vals"]) == K.REDUCE_EXPECTED


@pytest.mark.parametrize("flow_type", [10, 9])
def test_into_flowinfo_with_extra_fields(flow_type):
    """test_ipfix / test_netflowv9_into_flowinfo_with_extra_fields (tests.rs:339-586): the fields of
    the one record, compared sorted (the test sorts: HashSet order is unspecified), plus the
    exporter IP the actor appends; header sequence number / observation domain (shard) /
    sys-up time."""
    import json
    fields, pushes = K.flowinfo_scenario(flow_type)
    sc = dict(fields=fields, pushes=pushes, window_s=60, lateness_s=10)
    _agg, _emits, (g,) = run_oracle_scenario(sc)
    pkt = json.loads(_agg.flowinfo_json(g, shard_id=5, seq=42, export_time_ms=K.T_JUL2_10 * 1000))
    body = pkt["IPFIX" if flow_type == 10 else "NetFlowV9"]
    assert body["sequence_number"] == 42
    assert body["observation_domain_id" if flow_type == 10 else "source_id"] == 5
    if flow_type == 9:
        assert body["sys_up_time"] == 5000
    (st,) = body["sets"]
    (rec,) = st["Data"]["records"]
    assert st["Data"]["id"] == 65535 and rec["scope_fields"] == []
    key = lambda f: json.dumps(f, sort_keys=True)  # noqa: E731
    assert sorted(rec["fields"], key=key) == sorted(K.FLOWINFO_EXPECTED_FIELDS, key=key)


def _ie(pen, ie_id):
    import ngz_oracle as O
    return O.REGISTRY.lookup(pen, ie_id | (0x8000 if pen else 0))


@pytest.mark.parametrize("kat", K.FIELD_OP_KATS, ids=lambda k: k[0])
def test_field_op_kats(kat):
    """lib.rs:359-615: Field::{add,min,max,bitwise_or}_field of two fields of one IE gives the
    test's value; with a field of another IE it is FieldOperationError::Inapplicable*(lhs IE,
    rhs IE) -- for the VMware fields too, whose vendor error maps into the same variant."""
    name, src, op, ie, lhs, rhs, exp, other, err = kat
    a, b = _ie(*ie[:2]), _ie(*other[:2])
    assert (a.name, b.name) == (ie[2], other[2])
    assert A.field_op(op, a, lhs, a, rhs) == exp
    with pytest.raises(A.FieldOperationError) as e:
        A.field_op(op, a, lhs, b, rhs)
    assert (e.value.variant, e.value.lhs, e.value.rhs) == (err, a, b)


def test_supports_ops_kats():
    """IE::supports_{arithmetic,bitwise,comparison}_ops asserts of lib.rs:267-358 on the oracle's
    restatement (generator.rs:1176-1272)."""
    import ngz_oracle as O
    by_name = {ie.name: ie for ie in O.REGISTRY.by_key.values() if ie.pen == 0}
    for name, (arith, bit, cmp_) in K.SUPPORTS_KATS.items():
        ie = by_name[name]
        for op, want in ((K.OP_ADD, arith), (K.OP_OR, bit), (K.OP_MIN, cmp_), (K.OP_MAX, cmp_)):
            if want is not None:
                assert A.supports(ie, op) == want, (name, op)


@pytest.mark.parametrize("sc", K.FIELD_OP_SCENARIOS, ids=lambda s: s["name"])
def test_field_op_scenarios(sc):
    """The field-op KATs as two-record aggregation scenarios on the oracle."""
    agg, _emits, flushed = run_oracle_scenario(sc)
    assert _sorted(flushed) == _sorted(sc["flush"])

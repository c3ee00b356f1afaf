"""Pin the CPU oracle to the reference's packet-level and SliceReader KATs
(tests/kats_packets.py, wires from crates/flow-pkt/src/wire/tests/{ipfix,
netflow}.rs, benches/serde_benchmark.rs and parse-utils/src/reader.rs)."""
import pytest

import kat_runner
import kats_packets as K
import ngz_oracle as O


def run_case(case):
    """[[(status, value, consumed)]] per map, asserting every pinned step."""
    results = []
    for m in case:
        tmap = {}
        kat_runner.preload(tmap, m.get("preload", {}))
        got = []
        for kind, w, (ek, ev) in m["steps"]:
            wire = kat_runner.step_wire(w)
            st, val, consumed = kat_runner.oracle_step(kind, wire, tmap)
            if ek in ("ok", "ok?", "same"):
                assert st == "ok", (w, val)
                assert consumed == len(wire), "parsed completely: %d of %d" % (consumed, len(wire))
                if ek == "ok":
                    assert val == ev, (w, val)
                if ek == "same":
                    assert val == got[ev][1]
            else:
                assert st == "err", (w, val)
                if ek == "err":
                    assert val == ev
            got.append((st, val, consumed))
        for tid, n in m.get("counts", {}).items():
            assert tmap[tid].processed_count == n
        results.append(got)
    return results


@pytest.mark.parametrize("name", sorted(K.CASES))
def test_packet_kat_oracle(name):
    res = run_case(K.CASES[name])
    for cname, (ma, sa), (mb, sb) in K.SAME_ACROSS:
        if cname == name:
            assert res[ma][sa][1] == res[mb][sb][1]


def test_bench_data_only_records():
    """serde_benchmark.rs:73-161: the data-only packet is 34 records of
    template 1024 (40 B each) that the mixed packet defines."""
    tmap = {}
    O.parse_ipfix_packet(O.Reader(K.wire(K.B + "IPFIX_PKT_MIXED")), tmap)
    pkt = O.parse_ipfix_packet(O.Reader(K.wire(K.B + "IPFIX_PKT_DATA_PKT_ONLY")), tmap)
    assert [(k, sid, len(r)) for k, sid, r in pkt.sets] == [("Data", 1024, 34)]


def _reader_op(r, op, args):
    try:
        if op == "u8":
            return r.read_u8()
        if op in ("u16", "u32"):
            return r.read_uint({"u16": 2, "u32": 4}[op])
        if op == "peek16":
            return r.peek_uint(2)
        if op == "offset":
            return r.offset()
        if op == "remaining":
            return r.remaining()
        if op == "rest":
            return bytes(r.buf[r.pos:r.end])
        if op == "take":
            s = r.take_slice(args[0])
            return (s.offset(), bytes(s.buf[s.pos:s.end]))
        if op == "padded":
            n, ln = args
            return r.read_padded(ln, n)
        if op == "uint32":
            return r.read_unsigned_be(args[0], 4)
        if op == "uint64":
            return r.read_unsigned_be(args[0], 8)
        if op == "int32":
            return r.read_signed_be(args[0], 4)
        if op == "int64":
            return r.read_signed_be(args[0], 8)
    except O.ParseFail as e:
        (k, v), = e.err["Parse"].items()
        if k == "UnexpectedEof":
            return ("eof", v["offset"], v["needed"], v["available"])
        return ("pad", v["offset"], v["requested"], v["ret_len"])
    raise AssertionError(op)


@pytest.mark.parametrize("name,ops", K.READER_KATS, ids=[k[0] for k in K.READER_KATS])
def test_reader_kat(name, ops):
    r = O.Reader(bytearray(K.wire(K.R_ + name + ":data")))
    for op, args, exp in ops:
        assert _reader_op(r, op, args) == exp, (name, op, args)


def test_reader_shortened_and_too_wide():
    for w in K.READER_SHORTENED:
        for op in ("uint32", "uint64"):
            r = O.Reader(bytearray(w))
            assert _reader_op(r, op, (len(w),)) == 0xABCD and r.remaining() == 0
    for op, ln, exp in K.READER_TOO_WIDE:
        r = O.Reader(bytearray(16))
        assert _reader_op(r, op, (ln,)) == exp and r.offset() == 0


@pytest.mark.parametrize("name", sorted(n for n, c in K.CASES.items()
                                        if any(k in kat_runner.IPFIX_WRAPPED for m in c for k, _, _ in m["steps"])))
def test_wrapped_item_kats_at_packet_level(name):
    """The item-level KATs (mod.rs TemplateRecord / FieldSpecifier / DataRecord
    / Set) wrapped into the message the device tests send: the oracle's packet
    parse of it equals the reference value nested as its types nest it
    (kat_runner.ipfix_wrapped_expect), errors included with absolute offsets."""
    for m in K.CASES[name]:
        tmap = {}
        kat_runner.preload(tmap, m.get("preload", {}))
        tid = next(iter(m.get("preload", {})), None)
        pre, steps = kat_runner.codec_datagrams(m)
        for (i, dgram), (kind, w, (ek, ev)) in zip(steps, m["steps"]):
            st, val, consumed = kat_runner.oracle_step("ipfix", dgram, tmap)
            exp = kat_runner.ipfix_wrapped_expect(kind, ek, ev, tid)
            assert st == ("ok" if ek == "ok" else "err"), (name, i, val)
            assert val == exp, (name, i, val, exp)
            if st == "ok":
                assert consumed == len(dgram)


def test_codec_partial_messages_kat():
    """codec.rs:226-249 on the oracle codec: Ok(None) for both partial buffers, nothing consumed."""
    oc = O.FlowInfoCodec()
    for key, want in K.CODEC_PARTIAL:
        buf = bytearray(K.WIRES[key])
        n0 = len(buf)
        assert oc.decode(buf) is want
        assert len(buf) == n0
    assert len(K.WIRES[K.CODEC_PARTIAL[0][0]]) == 18 and K.WIRES[K.CODEC_PARTIAL[1][0]] == b"\x01"

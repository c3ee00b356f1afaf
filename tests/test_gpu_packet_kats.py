"""The reference's packet-level KATs through the HIP path (C ABI), in both
decode kernel paths.

Each map of a case gets one product FlowInfoCodec; templates a Rust test
inserts into its TemplatesMap directly are fed as a synthesized template
message first; then every step's wire is one datagram batch (so data-only
steps go through the device framing with the template state of the earlier
batches).  The product must give, per datagram:
  * exactly the oracle codec's result (status, serde JSON text, consumed), and
  * where the KAT pins it, the reference's own value: the FlowInfo JSON
    {"IPFIX": packet} / {"NetFlowV9": packet}, or the error
    {"IpfixParsingError": e} / {"NetFlowV9ParingError": e} (codec.rs:155-159,
    178-183) whenever the codec hands the bytes to the packet parser.
"""
import json

import pytest

import kat_runner
import parity
import kats_packets as K
import ngz_oracle as O
from netgauze_amd import _lib as L

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.flow import FlowInfoCodec  # noqa: F401  (loads libngz.so, fails loudly if missing)
    return torch.device("cuda:0")


@pytest.fixture(params=["specialized", "generic"])
def specialize(request):
    return request.param == "specialized"


def oracle_codec_step(oc, dgram):
    buf = bytearray(dgram)
    n0 = len(buf)
    try:
        m = oc.decode(buf)
    except O.ParseFail as e:
        return L.NGZ_DG_ERROR, O.dumps(e.err), n0 - len(buf)
    if m is None:
        return L.NGZ_DG_NEED_MORE, None, 0
    return L.NGZ_DG_OK, O.dumps(m.to_json()), n0 - len(buf)


def product_step(codec, dgram):
    batch = codec.decode_datagrams([dgram])
    st = int(batch.dgram_headers()[0]["status"])
    lines = batch.json_lines()
    if st == L.NGZ_DG_NEED_MORE:
        assert lines == []
        return st, None, 0
    assert len(lines) == 1 and lines[0][1] == st
    assert batch.json(0) == lines[0][2]
    if st == L.NGZ_DG_ERROR:  # the structured error (ngz_dgram_error) says the same
        parity.check_error_struct(batch, 0, json.loads(lines[0][2]))
    return st, lines[0][2], lines[0][3]


def wrap_pinned(kind, ek, ev, dgram, tid=None):
    """The reference value the codec-level JSON must equal, or None when the
    KAT pins nothing at this level."""
    if kind in kat_runner.IPFIX_WRAPPED:
        v = kat_runner.ipfix_wrapped_expect(kind, ek, ev, tid)
        return None if v is None else {"IPFIX" if ek == "ok" else "IpfixParsingError": v}
    proto = 10 if kind == "ipfix" else 9
    version = (dgram[0] << 8) | dgram[1]
    if ek == "ok":
        if kind == "nf9set":
            return {"NetFlowV9": dict(kat_runner.NF9_WRAP_HDR, sets=[ev])}
        return {"IPFIX": ev} if proto == 10 else {"NetFlowV9": ev}
    if ek == "err" and version == proto:
        return {"IpfixParsingError": ev} if proto == 10 else {"NetFlowV9ParingError": ev}
    return None


@pytest.mark.parametrize("name", sorted(K.CASES))
def test_packet_kat_gpu(dev, specialize, name):
    from netgauze_amd.flow import FlowInfoCodec
    results = []
    for m in K.CASES[name]:
        codec = FlowInfoCodec(0, specialize=specialize)
        oc = O.FlowInfoCodec()
        pre, steps = kat_runner.codec_datagrams(m)
        proto = 9 if m["steps"][0][0].startswith("nf9") else 10
        if pre:
            batch = codec.decode_datagrams(pre)
            for i, d in enumerate(pre):
                assert oracle_codec_step(oc, d)[0] == L.NGZ_DG_OK
                assert int(batch.dgram_headers()[i]["status"]) == L.NGZ_DG_OK
        got = []
        for (i, dgram), (kind, w, (ek, ev)) in zip(steps, m["steps"]):
            exp = oracle_codec_step(oc, dgram)
            res = product_step(codec, dgram)
            assert res == exp, "%s step %d (%s):\n got %s\n exp %s" % (name, i, w, res, exp)
            pinned = wrap_pinned(kind, ek, ev, dgram, next(iter(m.get("preload", {})), None))
            if pinned is not None:
                assert json.loads(res[1]) == pinned, (name, i)
            if ek in ("ok", "ok?", "same"):
                assert res[0] == L.NGZ_DG_OK and res[2] == len(dgram), (name, i, res[0], res[2])
            if ek == "same":
                assert res[1] == got[ev][1]
            if ek in ("err", "err?") and exp[0] != L.NGZ_DG_NEED_MORE:
                assert res[0] == L.NGZ_DG_ERROR
            got.append(res)
        counts = codec.template_counts(proto)
        tmap = oc.ipfix_templates if proto == 10 else oc.netflow_templates
        assert counts == {t: v.processed_count for t, v in tmap.items()}
        for tid, n in m.get("counts", {}).items():
            assert counts[tid] == n
        results.append(got)
    for cname, (ma, sa), (mb, sb) in K.SAME_ACROSS:
        if cname == name:
            assert results[ma][sa][1] == results[mb][sb][1]


def test_nf9_zero_length_fields_past_count_gate(dev, specialize):
    """netflow.rs:756-770 must be Err.  FlowInfoCodec::decode first waits for
    buf.len() >= the u16 at [2..4], which for v9 is the record *count*
    (codec.rs:200-206; 0x4b09 here), so the bare wire is Ok(None) at codec
    level.  Zero bytes appended past the failing set reach the parser with the
    same packet-level error the oracle restates (offset 41), on the device."""
    from netgauze_amd.flow import FlowInfoCodec
    wire = K.wire(K.N + "test_zero_length_fields:good_template_wire")
    count = (wire[2] << 8) | wire[3]
    dgram = wire + bytes(count - len(wire))
    oc = O.FlowInfoCodec()
    exp = oracle_codec_step(oc, dgram)
    st, val, _ = kat_runner.oracle_step("nf9", wire, {})
    assert st == "err" and json.loads(exp[1]) == {"NetFlowV9ParingError": val}
    codec = FlowInfoCodec(0, specialize=specialize)
    assert product_step(codec, dgram) == exp


def test_bench_data_only_steady_state(dev, specialize):
    """serde_benchmark.rs:225-230: templates from the mixed packet, then the
    34-record data-only packet decoded again and again (one batch of 64
    copies) - every copy is the same FlowInfo, and processed_count (+1 per
    set, ipfix.rs:223) counts them all."""
    from netgauze_amd.flow import FlowInfoCodec
    mixed = K.wire(K.B + "IPFIX_PKT_MIXED")
    data = K.wire(K.B + "IPFIX_PKT_DATA_PKT_ONLY")
    codec = FlowInfoCodec(0, specialize=specialize)
    oc = O.FlowInfoCodec()
    codec.decode_datagrams([mixed])
    oracle_codec_step(oc, mixed)
    exp = oracle_codec_step(oc, data)
    batch = codec.decode_datagrams([data] * 64)
    lines = batch.json_lines()
    assert len(lines) == 64 and all(ln[1:] == exp for ln in lines)
    for _ in range(63):
        oracle_codec_step(oc, data)
    assert codec.template_counts(10) == {t: v.processed_count for t, v in oc.ipfix_templates.items()}
    assert codec.template_counts(10)[1024] == 1 + 64


def test_codec_partial_messages_kat(dev, specialize):
    """codec.rs:226-249 (test_decode_partial_messages) through the C ABI: the 18-byte IPFIX buffer
    whose header announces 116 bytes, then the 1-byte buffer, each decoded as its own batch on one
    context, are NGZ_DG_NEED_MORE (Ok(None)) with nothing consumed and no template state touched;
    so is the pair as one batch, and a complete message decodes normally afterwards."""
    from netgauze_amd.flow import FlowInfoCodec
    codec = FlowInfoCodec(0, specialize=specialize)
    oc = O.FlowInfoCodec()
    wires = [K.WIRES[k] for k, _ in K.CODEC_PARTIAL]
    for w in wires:
        assert product_step(codec, w) == oracle_codec_step(oc, w) == (L.NGZ_DG_NEED_MORE, None, 0)
    batch = codec.decode_datagrams(wires)
    assert [int(s) for s in batch.dgram_headers()["status"]] == [L.NGZ_DG_NEED_MORE] * 2
    assert batch.json_lines() == []
    assert codec.template_counts(10) == {} and codec.template_counts(9) == {}
    full = bytes.fromhex("000a0010583de05900000ee400000000")  # the same header, length 16, no sets
    assert product_step(codec, full) == oracle_codec_step(oc, full)
    assert product_step(codec, full)[0] == L.NGZ_DG_OK

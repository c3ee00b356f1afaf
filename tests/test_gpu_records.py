"""GPU: the per-record typed view at the boundary (ngz_record_fields) against the oracle's
`Field` values -- DataRecord::parse -> Box<[Field]> (ipfix.rs:335-370, 419-424; NFv9
ScopeField netflow.rs:443-475): per field the IE (pen, id), its data type and decode rule, the
scope / string / vendor / unknown / sub-registry flags and the typed value, on every reference
golden capture, config 4 (NFv9 313 + the variable-length / enterprise template 900) and the
all-decode-rules template of the fuzz corpus."""
import types

import pytest

import fuzz_corpus as F
import golden_io
import ngz_oracle as O
import parity
from netgauze_amd import _lib as L

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

DTYPES = ["octetArray", "unsigned8", "unsigned16", "unsigned32", "unsigned64", "signed8", "signed16", "signed32",
          "signed64", "float32", "float64", "boolean", "macAddress", "string", "dateTimeSeconds",
          "dateTimeMilliseconds", "dateTimeMicroseconds", "dateTimeNanoseconds", "ipv4Address", "ipv6Address",
          "basicList", "subTemplateList", "subTemplateMultiList", "unsigned256"]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.flow import FlowInfoCodec  # noqa: F401  (loads libngz.so, fails loudly if missing)
    return torch.device("cuda:0")


def expected(fv, width, kind):
    """The oracle Field -> (pen, ie_id, dtype, flags, value bytes) the view must give."""
    scope = isinstance(fv, O.ScopeFieldValue)
    ie = fv.ie
    if scope:
        pen, ie_id, dtype = ie.pen, ie.id, 0
        flags = L.FV_SCOPE
    else:
        pen, ie_id, dtype = ie.pen, ie.id, DTYPES.index(ie.dtype) if ie.kind not in ("unknown", "vendor_unknown") else 0
        flags = 0
        if ie.kind in ("vendor", "vendor_unknown"):
            flags |= L.FV_VENDOR
        if ie.kind in ("unknown", "vendor_unknown"):
            flags |= L.FV_UNKNOWN
    v = fv.value
    if isinstance(v, str):
        flags |= L.FV_STRING
        val = v.encode("utf-8")
    elif kind == L.K_VLEN:
        val = bytes(v)
    else:
        val = parity.canon(fv, types.SimpleNamespace(kind=kind, width=width))
    return pen, ie_id, dtype, flags, val


def check_records(batch, oracle):
    sets = batch.sets()
    first = {}
    for i in range(len(sets)):
        first.setdefault(int(sets[i]["dgram"]), []).append(int(sets[i]["slot"]))
    widths = {(d, k): [fi.width for fi in batch.slots[slot].fields]
              for d, slots in first.items() for k, slot in enumerate(slots)}
    n = 0
    for d, (k, m) in enumerate(oracle):
        if k != "ok":
            if k == "err":
                with pytest.raises(Exception):
                    batch.record_fields(d, 0, 0)
            continue
        data = [s for s in m.sets if s[0] == "Data"]
        for si, (_, sid, recs) in enumerate(data):
            for r, (scope, fields) in enumerate(recs):
                got = batch.record_fields(d, si, r)
                allf = list(scope) + list(fields)
                assert len(got) == len(allf), (d, si, r)
                for f, (g, fv) in enumerate(zip(got, allf)):
                    pen, ie_id, kind, dtype, flags, wl, woff, val = g
                    width = widths[(d, si)][f]
                    e_pen, e_id, e_dtype, e_flags, e_val = expected(fv, width, kind)
                    assert (pen, ie_id) == (e_pen, e_id), (d, si, r, f, g[:2], (e_pen, e_id))
                    if f < len(scope) and not isinstance(fv, O.ScopeFieldValue):
                        e_flags |= L.FV_SCOPE
                    assert flags & (L.FV_SCOPE | L.FV_STRING | L.FV_VENDOR | L.FV_UNKNOWN) == e_flags, (d, si, r, f,
                                                                                                   flags, e_flags)
                    if not flags & L.FV_UNKNOWN and not isinstance(fv, O.ScopeFieldValue):
                        assert dtype == e_dtype, (d, si, r, f, dtype, e_dtype)
                    assert val == e_val, (d, si, r, f, kind, val[:40].hex(), e_val[:40].hex())
                    n += 1
        # a set index past the datagram's data sets is refused
        with pytest.raises(Exception):
            batch.record_fields(d, len(data), 0)
    return n


def run(dgrams, specialize=True):
    from netgauze_amd.flow import FlowInfoCodec
    codec = FlowInfoCodec(0, specialize=specialize)
    batch = codec.decode_datagrams(dgrams)
    oracle, _ = parity.oracle_datagrams(dgrams)
    return check_records(batch, oracle), batch, codec


def test_record_fields_on_reference_goldens(dev):
    total = 0
    for name, kind, _ in golden_io.cases():
        peers = {}
        for src, sp, dst, dp, payload in golden_io.datagrams(name):
            peers.setdefault((src, sp, dst, dp), []).append(payload)
        for dgs in peers.values():
            n, *_ = run(dgs)
            total += n
    assert total > 50_000


def test_record_fields_cfg4_and_all_decode_rules(dev):
    from netgauze_amd import synth
    n, *_ = run(synth.cfg4_datagrams(3000))
    assert n > 3000 * 14
    name, tm, msgs = F._zoo()
    n, *_ = run(tm + msgs, specialize=False)
    assert n > 200 * len(F.ZOO)


def test_record_fields_wire_offsets(dev):
    """wire_offset points at the field's bytes in its datagram: for fixed numeric fields the
    big-endian wire value re-reads to the decoded one (config 4, variable-length records
    included: the offsets come from the set's own record walk)."""
    from netgauze_amd import synth
    dgrams = synth.cfg4_datagrams(400)
    from netgauze_amd.flow import FlowInfoCodec
    codec = FlowInfoCodec(0)
    batch = codec.decode_datagrams(dgrams)
    oracle, _ = parity.oracle_datagrams(dgrams)
    checked = 0
    for d, (k, m) in enumerate(oracle):
        if k != "ok":
            continue
        for si, (_, sid, recs) in enumerate([s for s in m.sets if s[0] == "Data"]):
            for r in range(len(recs)):
                for pen, ie_id, kind, dtype, flags, wl, woff, val in batch.record_fields(d, si, r):
                    wire = dgrams[d][woff:woff + (len(val) if kind == L.K_VLEN else wl)]
                    if kind == L.K_VLEN:
                        assert wire == val
                    elif kind == L.K_UINT:
                        assert int.from_bytes(wire, "big") == int.from_bytes(val, "little"), (d, si, r, ie_id)
                    checked += 1
    assert checked > 400 * 10

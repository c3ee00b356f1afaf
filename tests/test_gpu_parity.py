"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle.

Bit-exact on every decoded field, every header, every error text.
"""
import ctypes
import struct

import numpy as np
import pytest

import golden_io
import ngz_oracle as O
import parity
from netgauze_amd import _lib as L

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.flow import FlowInfoCodec  # noqa: F401  (loads libngz.so, fails loudly if missing)
    return torch.device("cuda:0")


_SPECIALIZE = [True]


@pytest.fixture(autouse=True, params=["specialized", "generic"])
def kernel_path(request):
    """Every parity test runs through both decode paths: the per-template
    run-time-compiled kernels and the generic field-table kernel."""
    _SPECIALIZE[0] = request.param == "specialized"
    yield request.param
    _SPECIALIZE[0] = True


# ngz_ctx_set_option values a test forces on every context it creates (monkeypatch.setitem);
# they choose how a batch runs, never its results
CTX_OPTIONS = {}


def new_codec():
    from netgauze_amd.flow import FlowInfoCodec
    return FlowInfoCodec(0, specialize=_SPECIALIZE[0], options=dict(CTX_OPTIONS))


def run_both(dgrams):
    codec = new_codec()
    batch = codec.decode_datagrams(dgrams)
    oracle, ocodec = parity.oracle_datagrams(dgrams)
    stats = parity.check_batch(batch, oracle)
    return stats, batch, codec, ocodec


def t20_stream(n, rec_per_msg=1023, seed=None):
    from netgauze_amd import synth
    rec = synth.t20_records(n, seed=seed or synth.SEED_CFG2)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64, rec_per_msg=rec_per_msg)
    b = bytes(buf.numpy())
    return [synth.template_message()] + [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]


def test_t20_small(dev):
    stats, batch, codec, oc = run_both(t20_stream(2500))
    assert stats["ok"] == 4 and stats["records"] == 2500 and stats["unsupported"] == 0
    assert batch.n_template_dgrams == 1


def test_t20_mtu_messages(dev):
    # MTU-sized messages: 21 records per set, set starts not window aligned
    stats, *_ = run_both(t20_stream(1000, rec_per_msg=21))
    assert stats["records"] == 1000


def test_t20_steady_state_batches(dev):
    """Templates learnt in one batch are used by the next (per-peer state)."""
    from netgauze_amd import synth
    codec = new_codec()
    tm = synth.template_message()
    codec.decode_datagrams([tm])
    data = t20_stream(3000)[1:]
    batch = codec.decode_datagrams(data)
    assert batch.n_template_dgrams == 0
    oc = O.FlowInfoCodec()
    oc.decode(bytearray(tm))
    oracle, _ = parity.oracle_datagrams(data, oc)
    stats = parity.check_batch(batch, oracle)
    assert stats["records"] == 3000
    # processed_count: +1 per data set (ipfix.rs:223)
    assert codec.template_counts(10) == {256: oc.ipfix_templates[256].processed_count}


def test_steady_state_active_templates_change(dev):
    """Batches after the first launch the decode kernels of the templates
    that had records in the previous batch without a host round trip; a
    template that gains records (or loses them) in a later batch must still
    decode bit-exact, with processed counts and statuses redone."""
    from netgauze_amd import synth
    tpls = synth.CFG3_TEMPLATES[:3]
    codec = new_codec()
    oc = O.FlowInfoCodec()
    tm = synth.templates_message(tpls)
    codec.decode_datagrams([tm])
    oc.decode(bytearray(tm))

    def stream(ids, n, seed):
        dgrams = []
        for i, tid in enumerate(ids):
            fields = dict(tpls)[tid]
            rec = synth.template_records(fields, n, seed + i)
            _, rl = synth.field_offsets(fields)
            buf, offs, lens = synth.ipfix_data_stream(rec, rl, tid=tid, rec_per_msg=max(1, 60000 // rl))
            b = bytes(buf.numpy())
            dgrams += [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]
        return dgrams

    for ids, seed in (([256], 11), ([256], 12), ([256, 347], 13), ([348], 14), ([256, 347, 348], 15)):
        data = stream(ids, 3000, seed)
        batch = codec.decode_datagrams(data)
        oracle, _ = parity.oracle_datagrams(data, oc)
        stats = parity.check_batch(batch, oracle)
        assert stats["records"] == 3000 * len(ids), (ids, stats)
        assert codec.template_counts(10) == {t: oc.ipfix_templates[t].processed_count for t, _ in tpls}


def test_t20_device_resident_large(dev):
    """Full-column check at 10^6 records against big-endian numpy views."""
    from netgauze_amd import synth
    n = 1_000_000
    codec = new_codec()
    codec.decode_datagrams([synth.template_message()])
    rec = synth.t20_records(n, device=dev)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64)
    torch.cuda.synchronize()
    batch = codec.decode_batch(buf, offs, lens)
    assert batch.n_records == n
    hdr = batch.dgram_headers()
    assert (hdr["status"] == 0).all()
    slot = [s for s in batch.slots if s.template_id == 256][0]
    r = rec.cpu().numpy()
    offs_f, _ = synth.field_offsets(synth.T20)
    for f, ((ie, ln), off) in enumerate(zip(synth.T20, offs_f)):
        got = slot.column_bytes(f)
        raw = r[:, off:off + ln]
        if ie == 6:  # tcpControlBits -> u8 = low byte
            exp = raw[:, 1:2]
        else:
            exp = raw[:, ::-1]  # big endian -> little endian, same width
        assert np.array_equal(got, exp), "field %d (ie %d)" % (f, ie)


def column_on_device(slot, f, rows):
    """Device copy (torch, uint8 [rows, width]) of one decoded column: the
    full-size checks compare on the GPU instead of shipping GBs to the host."""
    from netgauze_amd import _lib
    w = slot.fields[f].width
    out = torch.empty(rows * w, dtype=torch.uint8, device="cuda")
    if rows * w:
        hip = _lib.hip()
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        assert hip.hipMemcpy(out.data_ptr(), slot.column_ptr(f), rows * w, 3) == 0  # D2D
    return out.view(rows, w)


def expected_column(rec, fi):
    """Canonical column of a fixed-width unsigned / ipv4 / tcpControlBits /
    raw-bytes / dateTimeMilliseconds field, from the wire bytes (torch, on the
    records' device): the big-endian value re-laid little-endian at the
    column width (SURVEY.md §8(a) column table)."""
    off, ln, w = fi.wire_offset, fi.wire_length, fi.width
    raw = rec[:, off:off + ln]
    if fi.kind == L.K_BYTES:
        return raw
    if fi.kind == L.K_TCPFLAGS:
        return raw[:, ln - 1:ln]
    assert fi.kind in (L.K_UINT, L.K_DTMS), fi.kind
    out = torch.zeros(rec.shape[0], w, dtype=torch.uint8, device=rec.device)
    out[:, :ln] = torch.flip(raw, dims=[1])
    return out


def check_slot_full(slot, rec):
    n = rec.shape[0]
    assert slot.n_records == n
    for f, fi in enumerate(slot.fields):
        got = column_on_device(slot, f, n)
        exp = expected_column(rec, fi)
        if not torch.equal(got, exp):
            bad = torch.nonzero((got != exp).any(dim=1)).flatten()
            raise AssertionError("template %d field %d: %d rows differ, first %s last %s; got %s exp %s" % (
                slot.template_id, f, bad.numel(), bad[:8].tolist(), bad[-4:].tolist(),
                got[bad[:2]].tolist(), exp[bad[:2]].tolist()))


def test_t20_full_size_1e8(dev):
    """North-star size: 10^8 T20 records, every column byte compared on the GPU."""
    from netgauze_amd import synth
    n = 100_000_000
    codec = new_codec()
    codec.decode_datagrams([synth.template_message()])
    rec = synth.t20_records(n, device=dev)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64)
    torch.cuda.synchronize()
    batch = codec.decode_batch(buf, offs, lens)
    del buf
    hdr = batch.dgram_headers()
    assert (hdr["status"] == 0).all() and len(hdr) == offs.numel()
    check_slot_full([s for s in batch.slots if s.template_id == 256][0], rec)
    assert codec.template_counts(10) == {256: offs.numel()}  # one processed_count per data set


def test_cfg4_full_size_batch_over_2gib(dev):
    """Config 4 at 1.6e7 records: the batch spans more than 2 GiB, so row-mode groups whose
    records lie more than 2 GiB apart go one record per pass (ngz_dev.h row_group), and the
    staged variable-length decode and the record map work above 2 GiB.  Every datagram
    decodes, the per-template record counts hold, every NetFlow v9 column equals its re-laid
    wire bytes (on the GPU), and the FlowInfo JSON of datagrams sampled at the start, the
    middle and past 2 GiB equals the oracle's."""
    from netgauze_amd import synth
    n = 16_000_000
    seed = synth.SEED_CFG4 + 99
    dg = synth.cfg4_datagrams(n, seed=seed)
    codec = new_codec()
    codec.decode_datagrams(dg[:2])
    data = dg[2:]
    buf, offs, lens = synth.host_batch(data, device=dev)
    assert buf.numel() > (1 << 31)
    batch = codec.decode_batch(buf, offs, lens)
    hdr = batch.dgram_headers()
    assert (hdr["status"] == 0).all() and len(hdr) == len(data)
    by_tid = {s.template_id: s for s in batch.slots}
    assert by_tid[synth.NF313_ID].n_records == n // 2 and by_tid[synth.V900_ID].n_records == n - n // 2
    nf = synth.template_records(synth.NF313, n // 2, seed, dev)
    slot = by_tid[synth.NF313_ID]
    for f, fi in enumerate(slot.fields):
        if fi.kind not in (L.K_UINT, L.K_DTMS, L.K_BYTES, L.K_TCPFLAGS):
            continue
        got = column_on_device(slot, f, n // 2)
        assert torch.equal(got, expected_column(nf, fi)), f
    del nf
    oc = O.FlowInfoCodec()
    for t in dg[:2]:
        oc.decode(bytearray(t))
    past = int(torch.searchsorted(offs, torch.tensor([1 << 31], device=offs.device)).item())
    sample = list(range(0, 40)) + list(range(len(data) // 2, len(data) // 2 + 40)) + list(range(past, past + 40)) + \
        list(range(len(data) - 40, len(data)))
    for d in sample:
        exp = O.dumps(oc.decode(bytearray(data[d])).to_json())
        assert batch.json(d) == exp, d


def test_cfg4_vlen_columns_full_size(dev):
    """Config 4 at 1.6e7 records: every column of the IPFIX variable-length / enterprise template
    900 (8e6 records) checked on the GPU against the generator's ground truth.  Each
    variable-length column entry {u64 batch offset, u32 length, 0} must equal the value's span
    in the batch as the generator wrote it (u8 length prefix, 255 + 3-byte escape every 97th
    record; generator.rs:1775-1793), and every fixed field -- those after variable-length
    fields included -- must equal its wire bytes re-laid at the column width."""
    from netgauze_amd import synth
    n = 16_000_000
    seed = synth.SEED_CFG4 + 99
    dg, lay = synth.cfg4_datagrams(n, seed=seed, layout=True)
    codec = new_codec()
    codec.decode_datagrams(dg[:2])
    data = dg[2:]
    buf, offs, lens = synth.host_batch(data, device=dev)
    batch = codec.decode_batch(buf, offs, lens)
    assert (batch.dgram_headers()["status"] == 0).all()
    slot = [s for s in batch.slots if s.template_id == synth.V900_ID][0]
    nv = n - n // 2
    assert slot.n_records == nv and len(slot.fields) == len(synth.V900)
    # batch offset of every record: its message's batch offset + 20 (message + set header)
    # + its offset inside the message's records
    rec_len = lay["rec_len"]
    starts = np.zeros(nv + 1, dtype=np.int64)
    starts[1:] = np.cumsum(rec_len)
    first = np.asarray(lay["v_first"], dtype=np.int64)
    per = np.diff(np.append(first, nv))
    msg_off = offs.cpu().numpy()[np.asarray(lay["v_pos"], dtype=np.int64) - 2].astype(np.int64)
    rec_batch = np.repeat(msg_off + 20 - starts[first], per) + starts[:-1]
    flat = torch.from_numpy(lay["flat"]).to(dev)
    checked = {"vlen": 0, "fixed": 0}
    for f, fi in enumerate(slot.fields):
        start, ln = lay["spans"][f]
        got = column_on_device(slot, f, nv)
        if fi.kind == L.K_VLEN:
            exp_off = torch.from_numpy(rec_batch + (start - starts[:-1])).to(dev)
            g = got.contiguous().view(torch.int64).view(nv, 2)
            assert torch.equal(g[:, 0], exp_off), f
            assert torch.equal(g[:, 1] & 0xFFFFFFFF, torch.from_numpy(ln).to(dev)), f
            assert torch.equal(g[:, 1] >> 32, torch.zeros_like(g[:, 1])), f
            checked["vlen"] += 1
            continue
        w = int(ln[0])
        idx = torch.from_numpy(start).to(dev)[:, None] + torch.arange(w, device=dev)[None, :]
        raw = flat[idx]  # [nv, wire length] big-endian wire bytes
        if fi.kind == L.K_BYTES:
            exp = raw
        else:
            assert fi.kind in (L.K_UINT, L.K_DTMS), (f, fi.kind)
            exp = torch.zeros(nv, fi.width, dtype=torch.uint8, device=dev)
            exp[:, :w] = torch.flip(raw, dims=[1])
        assert torch.equal(got, exp), f
        checked["fixed"] += 1
    assert checked == {"vlen": 5, "fixed": 9}, checked


def test_cfg3_mixed_templates_1e8(dev):
    """Config 3 at its full size, 10^8 records over 8 templates (1.25e7 each): every column of
    every template compared on the GPU with the wire bytes re-laid."""
    from netgauze_amd import synth
    codec = new_codec()
    codec.decode_datagrams([synth.templates_message(synth.CFG3_TEMPLATES)])
    b, o, ln, recs = synth.mixed_stream(100_000_000, device=dev)
    torch.cuda.synchronize()
    batch = codec.decode_batch(b, o, ln)
    del b
    assert batch.n_records == 100_000_000
    assert (batch.dgram_headers()["status"] == 0).all()
    by_tid = {s.template_id: s for s in batch.slots if s.n_records}
    assert set(by_tid) == set(recs)
    for tid in list(recs):
        check_slot_full(by_tid[tid], recs.pop(tid))


def test_cfg5_shard_full_size(dev):
    """One config-5 shard at its full size: 1.25e8 records over the 16 templates (rank 0 of
    10^9 over 8 GPUs, the stream bench.py --workload cfg5 decodes), every column of every
    template compared on the GPU with the wire bytes re-laid, and the per-template
    processed counts (one per data set) equal to the messages of each template."""
    from netgauze_amd import synth
    n = 125_000_000
    codec = new_codec()
    codec.decode_datagrams([synth.templates_message(synth.CFG5_TEMPLATES)])
    b, o, ln, recs = synth.mixed_stream(n, templates=synth.CFG5_TEMPLATES, seed=synth.SEED_CFG5, device=dev)
    torch.cuda.synchronize()
    batch = codec.decode_batch(b, o, ln)
    del b
    assert batch.n_records == n
    assert (batch.dgram_headers()["status"] == 0).all()
    by_tid = {s.template_id: s for s in batch.slots if s.n_records}
    assert set(by_tid) == set(recs) and len(recs) == 16
    msgs = {}
    for tid, fields in synth.CFG5_TEMPLATES:
        per = (65535 - 20) // synth.field_offsets(fields)[1]
        msgs[tid] = -(-recs[tid].shape[0] // per)
    for tid in list(recs):
        check_slot_full(by_tid[tid], recs.pop(tid))
    assert codec.template_counts(10) == msgs


@pytest.mark.parametrize("group", ["0", "1"])
def test_cfg3_mixed_templates_oracle(dev, group, monkeypatch):
    """Config 3 shape (8 templates, 40-153 B records, interleaved messages)
    against the oracle, every field; one launch per template or one
    multi-template launch per workgroup shape (NGZ_OPT_GROUP)."""
    monkeypatch.setitem(CTX_OPTIONS, L.NGZ_OPT_GROUP, int(group))
    from netgauze_amd import synth
    b, o, ln, _ = synth.mixed_stream(24_000)
    bb = bytes(b.numpy())
    dgrams = [synth.templates_message(synth.CFG3_TEMPLATES)] + [bb[x:x + y] for x, y in zip(o.tolist(), ln.tolist())]
    stats, batch, codec, oc = run_both(dgrams)
    assert stats["records"] == 24_000 and stats["unsupported"] == 0
    assert codec.template_counts(10) == {t: oc.ipfix_templates[t].processed_count for t, _ in synth.CFG3_TEMPLATES}


@pytest.mark.parametrize("group", ["0", "1"])
def test_cfg5_sixteen_templates_sharded(dev, group, monkeypatch):
    """Config 5 shape (16 templates: config 3 + width permutations) against
    the oracle, decoded as two shards on two contexts (ranks) as bench.py
    --gpus N does; the shards' processed counts add up to the oracle's.  One
    launch per template or per workgroup shape (NGZ_OPT_GROUP)."""
    monkeypatch.setitem(CTX_OPTIONS, L.NGZ_OPT_GROUP, int(group))
    from netgauze_amd import dist, synth
    b, o, ln, _ = synth.mixed_stream(32_000, templates=synth.CFG5_TEMPLATES, seed=synth.SEED_CFG5)
    bb = bytes(b.numpy())
    data = [bb[x:x + y] for x, y in zip(o.tolist(), ln.tolist())]
    tm = synth.templates_message(synth.CFG5_TEMPLATES)
    oc = O.FlowInfoCodec()
    oc.decode(bytearray(tm))
    total = {}
    for rank in range(2):
        lo, hi = dist.shard_range(len(data), rank, 2)
        codec = new_codec()
        codec.decode_datagrams([tm])
        shard = data[lo:hi]
        batch = codec.decode_datagrams(shard)
        oracle, _ = parity.oracle_datagrams(shard, oc)
        stats = parity.check_batch(batch, oracle)
        assert stats["unsupported"] == 0 and stats["err"] == 0
        for t, c in codec.template_counts(10).items():
            total[t] = total.get(t, 0) + c
    assert total == {t: oc.ipfix_templates[t].processed_count for t, _ in synth.CFG5_TEMPLATES}


@pytest.mark.parametrize("group", ["0", "1"])
def test_cfg3_mixed_templates_1e7(dev, group, monkeypatch):
    """Config 3 at 10^7 records (1.25e6 per template): every column of every
    template compared on the GPU with the wire bytes re-laid, one launch per
    template or per workgroup shape (NGZ_OPT_GROUP)."""
    monkeypatch.setitem(CTX_OPTIONS, L.NGZ_OPT_GROUP, int(group))
    from netgauze_amd import synth
    codec = new_codec()
    codec.decode_datagrams([synth.templates_message(synth.CFG3_TEMPLATES)])
    b, o, ln, recs = synth.mixed_stream(10_000_000, device=dev)
    torch.cuda.synchronize()
    batch = codec.decode_batch(b, o, ln)
    assert batch.n_records == 10_000_000
    assert (batch.dgram_headers()["status"] == 0).all()
    by_tid = {s.template_id: s for s in batch.slots if s.n_records}
    assert set(by_tid) == set(recs)
    for tid, rec in recs.items():
        check_slot_full(by_tid[tid], rec)


def peers_of(name):
    groups = {}
    for src, sp, dst, dp, payload in golden_io.datagrams(name):
        groups.setdefault((src, sp, dst, dp), []).append(payload)
    return groups


GOLDEN = [c[0] for c in golden_io.cases()]


@pytest.mark.parametrize("name", GOLDEN)
def test_reference_captures_datagram_mode(dev, name):
    """Every datagram of the reference's captures, per exporter peer."""
    for key, dgrams in peers_of(name).items():
        stats, *_ = run_both(dgrams)
        assert stats["ok"] + stats["unsupported"] + stats["err"] + stats["none"] == len(dgrams)


# ---------------------------------------------------------------------------
# hand-built messages: framing errors, record errors, template state
# ---------------------------------------------------------------------------
def ipfix_msg(sets, export_time=1_700_000_000, seq=1, domain=7):
    body = b"".join(sets)
    return struct.pack(">HHIII", 10, 16 + len(body), export_time, seq, domain) + body


def ipfix_set(sid, payload):
    return struct.pack(">HH", sid, 4 + len(payload)) + payload


def tmpl(tid, fields):
    out = struct.pack(">HH", tid, len(fields))
    for f in fields:
        if len(f) == 2:
            out += struct.pack(">HH", f[0], f[1])
        else:
            out += struct.pack(">HHI", f[0] | 0x8000, f[1], f[2])
    return out


def nf_msg(sets, count, sys_up=1000, unix=1_700_000_000, seq=5, src=9):
    return struct.pack(">HHIIII", 9, count, sys_up, unix, seq, src) + b"".join(sets)


def test_framing_errors(dev):
    t = ipfix_msg([ipfix_set(2, tmpl(300, [(8, 4), (7, 2)]))])
    rec = bytes([10, 0, 0, 1, 0, 80])
    dgrams = [
        t,
        b"\x00\x0a\x00",                                   # shorter than 16: Ok(None)
        ipfix_msg([ipfix_set(300, rec * 3)])[:30],          # shorter than its length: Ok(None)
        struct.pack(">HHIII", 11, 16, 0, 0, 0),            # unsupported version
        struct.pack(">HHIII", 10, 12, 0, 0, 0) + b"\0" * 4,  # length < 16
        ipfix_msg([ipfix_set(5, b"")]),                     # invalid set id
        ipfix_msg([struct.pack(">HH", 300, 2)]),            # set length < 4
        ipfix_msg([struct.pack(">HH", 300, 40) + rec]),     # set longer than message
        ipfix_msg([ipfix_set(301, rec)]),                   # no template
        ipfix_msg([ipfix_set(300, rec * 2 + b"\x01")]),     # leftover ignored (IPFIX)
        ipfix_msg([ipfix_set(300, rec), b"\x01"]),          # 1 trailing byte: eof on set id
        ipfix_msg([ipfix_set(300, rec), b"\x01\x2c\x00"]),  # eof on set length
        ipfix_msg([ipfix_set(300, rec)]) + b"trailing",     # bytes after the message: ignored
    ]
    stats, *_ = run_both(dgrams)
    assert stats["err"] >= 8 and stats["none"] == 2


def test_record_errors(dev):
    # dateTimeMilliseconds (152), dateTimeMicroseconds (154), interfaceName string (82)
    t = ipfix_msg([ipfix_set(2, tmpl(400, [(152, 8), (154, 8), (82, 8), (7, 2)]))])

    def rec(ms, secs, frac, s, port=1):
        return struct.pack(">QII", ms, secs, frac) + s + struct.pack(">H", port)

    good = rec(1_700_000_000_123, 1_700_000_000, 12345, b"eth0\0\0\0\0")
    dgrams = [
        t,
        ipfix_msg([ipfix_set(400, good * 4)]),
        ipfix_msg([ipfix_set(400, good + rec(2**63 + 5, 1, 1, b"ok\0\0\0\0\0\0"))]),       # millis out of range
        ipfix_msg([ipfix_set(400, good * 2 + rec(1, 1_700_000_000, 0xFFFFFFFF, b"x" * 8))]),  # leap ns, sec%60!=59
        ipfix_msg([ipfix_set(400, rec(1, 1_700_000_039, 0xFFFFFFFF, b"ok\0\xff\xfe\0\0\0"))]),  # :59 leap accepted, junk after NUL ok
        ipfix_msg([ipfix_set(400, good + rec(1, 1, 1, b"ab\xc3\x28\0\0\0\0"))]),           # invalid utf-8
        ipfix_msg([ipfix_set(400, rec(1, 1, 1, b"ab\xe2\x82\0\0\0\0"))]),                 # truncated utf-8 before NUL
        ipfix_msg([ipfix_set(400, rec(2**63, 1, 1, b"\xff" * 8) * 2)]),                   # first error wins
        ipfix_msg([ipfix_set(400, good), ipfix_set(400, rec(1, 1, 1, b"\x80" * 8))]),     # error in 2nd set
    ]
    stats, batch, codec, oc = run_both(dgrams)
    assert stats["err"] == 6 and stats["ok"] == 3
    assert codec.template_counts(10) == {400: oc.ipfix_templates[400].processed_count}


def vl(b):
    """RFC 7011 s7 variable-length encoding as the reference reads it:
    u8 length, or 255 + 3-byte length (generator.rs:1775-1793)."""
    return (bytes([len(b)]) if len(b) < 255 else b"\xff" + len(b).to_bytes(3, "big")) + b


def test_variable_length_fields(dev):
    """IPFIX variable-length (65535) IEs on the device: strings (UTF-8
    checked, no NUL truncation), octet arrays, vendor-unknown IEs, the 255
    escape, fields after a vlen field at per-record offsets, and every
    UnexpectedEof a record walk can hit."""
    fields = [(8, 4), (82, 65535), (7, 2), (313, 65535), (152, 8), (4, 1), (1000, 65535, 2011)]
    t = ipfix_msg([ipfix_set(2, tmpl(500, fields))])

    def rec(name, blob, ms=1_700_000_000_000, ven=b"hw", port=443, proto=6, ip=0x0A000001):
        return (struct.pack(">I", ip) + vl(name) + struct.pack(">H", port) + vl(blob) + struct.pack(">QB", ms, proto)
                + vl(ven))

    goods = [rec(("if%d" % i).encode() * (i % 7), bytes(range(i % 64)), ms=1_700_000_000_000 + i,
                 port=i & 0xFFFF, ven=b"v" * (300 if i % 97 == 0 else i % 13)) for i in range(700)]
    assert len(b"".join(goods[40:700])) < 65000
    dgrams = [
        t,
        ipfix_msg([ipfix_set(500, b"".join(goods[:40]))]),
        ipfix_msg([ipfix_set(500, b"".join(goods[40:700]))]),                      # > 256 records: several chunks
        ipfix_msg([ipfix_set(500, rec("grüße €".encode(), b"", ven=b"") + rec(b"a\0b", b"\x00" * 300))]),
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x") + b"\0\0\0")]),                  # zero padding after records
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x") + rec(b"\xc3\x28", b"y"))]),       # invalid utf-8 (vlen: no NUL cut)
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x") + rec(b"ok", b"y", ms=2**63 + 1))]),  # dt-ms after vlen fields
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x") + struct.pack(">I", 1) + b"\xc8" + b"n" * 20)]),      # data EOF
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x") + rec(b"ok", b"y", ven=b"")[:-1] + b"\xff\x00\x01")]),  # escape EOF
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x") + struct.pack(">I", 1) + vl(b"e" * 14))]),              # u16 EOF
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x") + struct.pack(">I", 1) + b"\xff\x00\x00\x05abcd" + b"\0" * 8)]),
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x")), ipfix_set(500, rec(b"ok", b"\x01" * 40)[:-3])]),   # 2nd set EOF
        ipfix_msg([ipfix_set(500, rec(b"ok", b"x")) + ipfix_set(2, tmpl(501, [(8, 4), (82, 65535)]))]),
        ipfix_msg([ipfix_set(501, struct.pack(">I", 7) + vl(b"z" * 1000)), ipfix_set(500, rec(b"q", b"r"))]),
    ]
    stats, batch, codec, oc = run_both(dgrams)
    assert stats["unsupported"] == 0
    assert stats["records"] == 700 + 2 + 1 + 1 + 2
    assert stats["err"] == 7
    assert codec.template_counts(10) == {t: oc.ipfix_templates[t].processed_count for t in (500, 501)}


def test_variable_length_utf8_randomized(dev):
    """UTF-8 of variable-length strings at every byte alignment and length (0-300, both length
    forms): ASCII, valid 2-4 byte sequences, and one invalid byte (lone continuation, truncated
    sequence, overlong, surrogate, > U+10FFFF) placed at the first, a middle and the last byte, in
    messages of 60 records (the staged 64-row groups) and a lone-record message (unstaged); every
    datagram against the oracle (ipfix.rs:335-370, generator.rs:1775-1793: vlen strings are
    UTF-8 checked over all their bytes, no NUL cut)."""
    import random
    rnd = random.Random(29)
    fields = [(8, 4), (82, 65535), (7, 2), (96, 65535), (4, 1), (83, 65535)]
    t = ipfix_msg([ipfix_set(2, tmpl(502, fields))])
    good = ["", "a", "ab", "abc", "abcd", "gr\u00fc\u00dfe", "\u20ac\u20ac", "\U0001f600x", "\u00e9" * 40]
    bad = [b"\x80", b"\xc3", b"\xe2\x82", b"\xc0\xaf", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xff"]

    def text():
        k = rnd.random()
        n = rnd.choice([0, 1, 2, 3, 5, 17, 40, 63, 64, 65, 254, 255, 300])
        base = "".join(rnd.choice("abcdefghij") for _ in range(n)).encode()
        if k < 0.5:
            return base
        if k < 0.75:
            return base + rnd.choice(good).encode()
        b = rnd.choice(bad)
        at = rnd.choice([0, len(base) // 2, len(base)])
        return base[:at] + b + base[at:]

    def rec():
        return (struct.pack(">I", rnd.getrandbits(32)) + vl(text()) + struct.pack(">H", rnd.getrandbits(16)) +
                vl(text()) + bytes([rnd.getrandbits(8)]) + vl(text()))
    dgrams = [t]
    for m in range(40):
        dgrams.append(ipfix_msg([ipfix_set(502, b"".join(rec() for _ in range(60 if m % 4 else 1)))]))
    stats, batch, codec, oc = run_both(dgrams)
    assert stats["unsupported"] == 0 and stats["err"] > 5 and stats["ok"] > 1


def test_reference_field_kats(dev):
    """The reference's field-level unit vectors (tests/kats.py) through the
    device: each wrapped as [sourceIPv4Address, field, sourceTransportPort]
    records of its own template, 3 records per message.  (The InvalidLength
    vectors call Field::parse directly in the reference; on the wire their
    templates are already rejected by FieldSpecifier::new, so they are pinned
    on the oracle only, tests/test_oracle_kat.py.)"""
    import kats
    dgrams = []
    good = [k for k in kats.KATS if not isinstance(k[4], dict)]
    for i, (name, ie_id, length, wire, _) in enumerate(good):
        tid = 600 + i
        recs = b"".join(struct.pack(">I", 0x0A000000 + k) + wire + struct.pack(">H", 1000 + k) for k in range(3))
        dgrams += [ipfix_msg([ipfix_set(2, tmpl(tid, [(8, 4), (ie_id, length), (7, 2)]))]),
                   ipfix_msg([ipfix_set(tid, recs)])]
    stats, *_ = run_both(dgrams)
    assert stats["err"] == 0 and stats["ok"] == 2 * len(good) and stats["records"] == 3 * len(good)


def test_cfg4_split_framing_steady_state(dev, kernel_path, monkeypatch):
    """Steady-state config-4 batches (NFv9 313 + IPFIX variable-length 900) with split framing
    (NGZ_OPT_SPLIT 1; off by default, it measured slower): from the second batch on, the record
    walk of the variable-length sets runs on its own stream beside the NFv9 framing and decode
    (specialised kernels); every batch equals the
    oracle, processed counts included.  A batch with a variable-length record that runs past
    its set (the UnexpectedEof only the split walk sees; phase A went past it) runs again
    unsplit and equals the oracle too, and so does the batch after it."""
    from netgauze_amd import synth
    monkeypatch.setitem(CTX_OPTIONS, L.NGZ_OPT_SPLIT, 1)
    dg = synth.cfg4_datagrams(9000)
    codec = new_codec()
    oc = O.FlowInfoCodec()
    codec.decode_datagrams(dg[:2])
    parity.oracle_datagrams(dg[:2], oc)
    data = dg[2:]
    third = len(data) // 3
    infos = []
    for k in range(3):
        part = data[k * third:(k + 1) * third]
        batch = codec.decode_datagrams(part)
        oracle, _ = parity.oracle_datagrams(part, oc)
        stats = parity.check_batch(batch, oracle)
        assert stats["err"] == 0 and stats["records"] > 0
        infos.append(codec.last_batch_info())
    if kernel_path == "specialized":
        assert infos[1] & L.NGZ_BATCH_SPLIT and infos[2] & L.NGZ_BATCH_SPLIT, infos
    else:
        assert not any(i & L.NGZ_BATCH_SPLIT for i in infos), infos
    bad = list(data[:400])
    i = next(j for j, d in enumerate(bad) if d[1] == 10 and j > 40)
    b = bytearray(bad[i])
    b[28:32] = b"\xff\xff\xff\xff"  # the first record's first string: 0xFF escape, length 2^24 - 1
    bad[i] = bytes(b)
    for part in (bad, data[400:800]):
        batch = codec.decode_datagrams(part)
        oracle, _ = parity.oracle_datagrams(part, oc)
        stats = parity.check_batch(batch, oracle)
        assert stats["err"] == (1 if part is bad else 0)
        if part is bad and kernel_path == "specialized":
            assert codec.last_batch_info() & L.NGZ_BATCH_RERUN
    assert codec.template_counts(10) == {900: oc.ipfix_templates[900].processed_count}
    assert codec.template_counts(9) == {313: oc.netflow_templates[313].processed_count}


def test_cfg4_netflow_v9_and_variable_length(dev):
    """Config 4 shape: NetFlow v9 (the reference capture's template 313, 130 B)
    interleaved with IPFIX records carrying variable-length strings/octets and
    VMware / Huawei enterprise IEs, against the oracle."""
    from netgauze_amd import synth
    dgrams = synth.cfg4_datagrams(6000)
    stats, batch, codec, oc = run_both(dgrams)
    assert stats["records"] == 6000 and stats["err"] == 0 and stats["unsupported"] == 0
    assert codec.template_counts(10) == {900: oc.ipfix_templates[900].processed_count}
    assert codec.template_counts(9) == {313: oc.netflow_templates[313].processed_count}


def test_unknown_pen_65535_is_eof(dev):
    """IE::Unknown (unregistered PEN) with length 65535 is read as 65535 fixed
    bytes (generator.rs:2971-2974): every record hits UnexpectedEof."""
    t = ipfix_msg([ipfix_set(2, tmpl(510, [(8, 4), (5, 65535, 213)]))])
    dgrams = [t, ipfix_msg([ipfix_set(510, struct.pack(">I", 1) + b"abc")])]
    stats, *_ = run_both(dgrams)
    assert stats["err"] == 1 and stats["unsupported"] == 0


def test_template_errors_and_redefinition(dev):
    rec_a = struct.pack(">IH", 0x0A000001, 80)
    rec_b = struct.pack(">HIB", 443, 0xC0A80001, 6)
    dgrams = [
        ipfix_msg([ipfix_set(2, tmpl(310, [(8, 4), (7, 2)]))]),
        ipfix_msg([ipfix_set(310, rec_a * 5)]),
        ipfix_msg([ipfix_set(2, tmpl(310, [(7, 2), (8, 4), (4, 1)])), ipfix_set(310, rec_b * 3)]),  # redefine + use
        ipfix_msg([ipfix_set(310, rec_b * 2)]),
        ipfix_msg([ipfix_set(2, tmpl(311, [(8, 4), (999, 4)]))]),       # UndefinedIANAIE
        ipfix_msg([ipfix_set(2, tmpl(312, [(8, 5)]))]),                 # length outside length_range
        ipfix_msg([ipfix_set(2, tmpl(100, [(8, 4)]))]),                 # template id < 256
        ipfix_msg([ipfix_set(2, tmpl(313, [(8, 4)]) + b"\x01")]),       # truncated template record
        ipfix_msg([ipfix_set(2, tmpl(314, [(8, 4), (2011, 2, 2011), (1234, 3, 99999)]))]),  # vendor / unknown PEN
        ipfix_msg([ipfix_set(314, struct.pack(">I", 1) + b"\x00\x07" + b"abc")]),
        ipfix_msg([ipfix_set(3, struct.pack(">HHH", 320, 2, 1) + struct.pack(">HHHH", 10, 4, 8, 4) + b"\0\0")]),
        ipfix_msg([ipfix_set(320, struct.pack(">II", 7, 0x01020304) * 2)]),
        ipfix_msg([ipfix_set(3, struct.pack(">HHH", 321, 1, 2) + struct.pack(">HH", 10, 4))]),  # scope > total
        ipfix_msg([ipfix_set(3, struct.pack(">HHH", 322, 1, 1) + struct.pack(">HH", 10, 4) + b"\0\x05")]),  # padding
        ipfix_msg([ipfix_set(310, rec_b)]),
    ]
    stats, batch, codec, oc = run_both(dgrams)
    assert stats["ok"] >= 7 and stats["err"] >= 5
    assert codec.templates(10) == [{"id": k, **_tjson(v)} for k, v in sorted(oc.ipfix_templates.items())]
    assert codec.template_counts(10) == {k: v.processed_count for k, v in oc.ipfix_templates.items()}


def _tjson(t):
    return {"scope_field_specifiers": [s.to_json() for s in t.scope],
            "field_specifiers": [f.to_json() for f in t.fields]}


def test_template_after_failing_record_is_not_applied(dev):
    """A record error stops the message: a template set after it must not be
    learnt (ipfix.rs:94-96 + :314-320)."""
    t = ipfix_msg([ipfix_set(2, tmpl(330, [(82, 4)]))])
    dgrams = [
        t,
        ipfix_msg([ipfix_set(330, b"\xff\xff\xff\xff"), ipfix_set(2, tmpl(331, [(8, 4)]))]),
        ipfix_msg([ipfix_set(331, b"\x01\x02\x03\x04")]),  # -> NoTemplateDefinedFor
        ipfix_msg([ipfix_set(330, b"ok\0\0"), ipfix_set(2, tmpl(332, [(8, 4)]))]),
        ipfix_msg([ipfix_set(332, b"\x01\x02\x03\x04")]),
    ]
    stats, *_ = run_both(dgrams)
    assert stats["err"] == 2 and stats["ok"] == 3


def test_netflow_v9(dev):
    tset = struct.pack(">HH", 0, 4 + 4 + 16) + struct.pack(">HH", 260, 4) + struct.pack(">HHHHHHHH", 8, 4, 1, 4, 7, 2, 6, 1)
    # options template: scope System(1) len 4, Interface(2) len 2; option samplingInterval(34) len 4
    oset = struct.pack(">HH", 1, 4 + 6 + 8 + 4 + 2) + struct.pack(">HHH", 270, 8, 4) + \
        struct.pack(">HHHH", 1, 4, 2, 2) + struct.pack(">HH", 34, 4) + b"\0\0"
    rec = struct.pack(">IIHB", 0x0A000001, 1500, 80, 0x12)  # octetDeltaCount reduced to 4 bytes
    orec = struct.pack(">IHI", 77, 3, 1000)
    dgrams = [
        nf_msg([tset, oset], count=2),
        nf_msg([struct.pack(">HH", 260, 4 + 11 * 3 + 3) + rec * 3 + b"\0\0\0"], count=3),
        nf_msg([struct.pack(">HH", 270, 4 + 10 * 2) + orec * 2], count=2),
        nf_msg([struct.pack(">HH", 260, 4 + 11 * 2 + 1) + rec * 2 + b"\x01"], count=2),  # bad padding
        nf_msg([struct.pack(">HH", 260, 4 + 11 * 3) + rec * 3], count=2),                # InvalidCount
        nf_msg([struct.pack(">HH", 260, 4 + 11) + rec, struct.pack(">HH", 260, 4 + 11) + rec], count=1),  # count stops
        nf_msg([struct.pack(">HH", 261, 4 + 11) + rec], count=1),                        # no template
        nf_msg([], count=0)[:18],                                                        # header eof
        nf_msg([struct.pack(">HH", 3, 4)], count=1),                                     # invalid set id
    ]
    stats, batch, codec, oc = run_both(dgrams)
    assert stats["ok"] >= 4 and stats["err"] >= 4
    assert codec.template_counts(9) == {k: v.processed_count for k, v in oc.netflow_templates.items()}


def test_all_field_kinds(dev):
    """One template with every fixed-width data type the registry uses."""
    fields = [(8, 4), (27, 16), (56, 6), (70, 3), (152, 8), (154, 8), (156, 8), (150, 4), (82, 8),
              (1, 3), (2, 5), (6, 1), (4, 1), (89, 1), (61, 1), (434, 4), (276, 1), (320, 8),
              (9, 1), (210, 3), (7, 1), (18, 16), (138, 8), (500, 2)]
    ies = O.REGISTRY
    fields = [f for f in fields if (0, f[0]) in ies.by_key]
    t = ipfix_msg([ipfix_set(2, tmpl(340, fields))])
    rl = sum(ln for _, ln in fields)
    rng = np.random.default_rng(5)
    offs, o = [], 0
    for _, ln in fields:
        offs.append(o)
        o += ln
    data = []
    for m in range(6):
        recs = bytearray(rng.integers(0, 256, size=rl * 50, dtype=np.uint8).tobytes())
        if m < 4:  # keep dates in range and strings printable so records decode
            for r in range(50):
                for (ie, ln), off in zip(fields, offs):
                    b = r * rl + off
                    dt = O.REGISTRY.by_key[(0, ie)].dtype
                    if dt == "dateTimeMilliseconds":
                        recs[b:b + 8] = int(rng.integers(0, 2**41)).to_bytes(8, "big")
                    elif dt == "string":
                        recs[b:b + ln] = bytes(rng.integers(32, 127, size=ln, dtype=np.uint8))
        data.append(ipfix_msg([ipfix_set(340, bytes(recs))], seq=m))
    stats, *_ = run_both([t] + data)
    assert stats["ok"] + stats["err"] == 7


def test_wide_templates_no_field_cap(dev):
    """Templates of 200 and 600 fields (no field cap; the reference has none,
    ipfix.rs:384-413): the 200-field one gets a generated kernel, the 600-field
    one (> NGZ_RTC_MAX_FIELDS) the generic kernel, whose descriptors past the
    first 128 come through scalar loads.  NFv9 too."""
    rng = np.random.default_rng(17)
    kinds = [(7, 2), (8, 4), (1, 8), (4, 1), (27, 16), (152, 8), (82, 6), (2, 3), (61, 1), (210, 5)]
    dgrams = []
    for tid, nf in ((700, 200), (701, 600)):
        fields = [kinds[i % len(kinds)] for i in range(nf)]
        rl = sum(ln for _, ln in fields)
        dgrams.append(ipfix_msg([ipfix_set(2, tmpl(tid, fields))]))
        per = max(1, 60000 // rl)
        for m in range(3):
            recs = bytearray()
            for _ in range(per):
                for ie, ln in fields:
                    if ie == 152:
                        recs += int(rng.integers(0, 2**41)).to_bytes(8, "big")
                    elif ie == 82:
                        recs += bytes(rng.integers(97, 123, size=ln, dtype=np.uint8))
                    else:
                        recs += bytes(rng.integers(0, 256, size=ln, dtype=np.uint8))
            dgrams.append(ipfix_msg([ipfix_set(tid, bytes(recs))], seq=m))
    # NetFlow v9, 300 fields
    nfields = [kinds[i % 5] for i in range(300)]
    nrl = sum(ln for _, ln in nfields)
    tset = struct.pack(">HH", 0, 8 + 4 * len(nfields)) + struct.pack(">HH", 710, len(nfields)) + \
        b"".join(struct.pack(">HH", ie, ln) for ie, ln in nfields)
    dgrams.append(nf_msg([tset], count=1))
    for m in range(2):
        body = bytearray()
        for _ in range(20):
            for ie, ln in nfields:
                body += (int(rng.integers(0, 2**41)).to_bytes(8, "big") if ie == 152
                         else bytes(rng.integers(0, 256, size=ln, dtype=np.uint8)))
        dgrams.append(nf_msg([struct.pack(">HH", 710, 4 + len(body)) + bytes(body)], count=20))
    stats, batch, codec, oc = run_both(dgrams)
    assert stats["unsupported"] == 0 and stats["err"] == 0
    assert {s.template_id: len(s.fields) for s in batch.slots} == {700: 200, 701: 600, 710: 300}
    assert {s.template_id: batch.out.slots[i].n_fields for i, s in enumerate(batch.slots)} == \
        {700: 200, 701: 600, 710: 300}
    assert stats["records"] == sum(3 * max(1, 60000 // sum(ln for _, ln in [kinds[i % 10] for i in range(n)]))
                                   for n in (200, 600)) + 40


def test_template_counts_device(dev):
    """ngz_template_counts_device writes the (id, processed_count) table for a
    collective in one stream-ordered copy; ids ascending, tail zeroed, reset
    as ngz_template_counts (flow_actor.rs:362-381)."""
    from netgauze_amd import synth
    tpls = synth.CFG3_TEMPLATES[:3]
    codec = new_codec()
    oc = O.FlowInfoCodec()
    dgrams = [synth.templates_message(tpls)]
    for i, (tid, fields) in enumerate(tpls):
        rec = synth.template_records(fields, 500 * (i + 1), 40 + i)
        _, rl = synth.field_offsets(fields)
        buf, offs, lens = synth.ipfix_data_stream(rec, rl, tid=tid, rec_per_msg=37)
        b = bytes(buf.numpy())
        dgrams += [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]
    codec.decode_datagrams(dgrams)
    parity.oracle_datagrams(dgrams, oc)
    exp = sorted((k, v.processed_count) for k, v in oc.ipfix_templates.items())
    table = torch.full((8, 2), -1, dtype=torch.int64, device="cuda:0")
    assert codec.template_counts_device(10, table.data_ptr(), 8) == 3
    torch.cuda.synchronize()
    got = table.cpu().tolist()
    assert [tuple(r) for r in got[:3]] == exp and got[3:] == [[0, 0]] * 5
    small = torch.zeros((2, 2), dtype=torch.int64, device="cuda:0")
    assert codec.template_counts_device(10, small.data_ptr(), 2, reset=True) == 3  # > cap: re-agree the size
    torch.cuda.synchronize()
    assert [tuple(r) for r in small.cpu().tolist()] == exp[:2]
    assert codec.template_counts(10) == dict(exp)  # too small a table resets nothing
    assert codec.template_counts_device(10, table.data_ptr(), 8, reset=True) == 3
    assert codec.template_counts(10) == {k: 0 for k, _ in exp}  # reset
    assert codec.template_counts_device(9, table.data_ptr(), 8) == 0
    torch.cuda.synchronize()
    assert table.abs().sum().item() == 0


def test_columns_to_host_async(dev, kernel_path):
    """ngz_columns_to_host_async: the column blocks copied by a copy engine or by the CUs' stores
    to pinned host memory (NGZ_D2H_KERNEL) on another stream equal the synchronous copy, and the
    context's next decode waits for the copy before it reuses the columns."""
    from netgauze_amd import synth
    from netgauze_amd.flow import NgzError
    codec = new_codec()
    dgrams = synth.cfg4_datagrams(4000) + t20_stream(5000)  # three templates, NFv9 and IPFIX
    batch = codec.decode_datagrams(dgrams)
    assert sum(1 for s in batch.slots if s.n_records) == 3
    cap = sum(s.block_bytes() + 256 for s in batch.slots)
    side = torch.cuda.Stream(dev)
    again = t20_stream(3000)[1:]
    for kernel in (True, False):
        ref = np.zeros(cap, dtype=np.uint8)
        n = codec.columns_to_host(ref.ctypes.data, cap)
        assert n > 0
        out = torch.zeros(cap + 64, dtype=torch.uint8).pin_memory()
        for shift in (0, 3):  # 16-byte and byte copies
            out.zero_()
            got = codec.columns_to_host_async(out.data_ptr() + shift, cap, stream=side.cuda_stream, kernel=kernel)
            assert got == n
            side.synchronize()
            assert np.array_equal(out.numpy()[shift:shift + n], ref[:n])
        # queued, then straight into the next decode on the same context: the copy still sees this
        # batch's columns (the decode waits for it)
        out.zero_()
        codec.columns_to_host_async(out.data_ptr(), cap, stream=side.cuda_stream, kernel=kernel)
        b2 = codec.decode_datagrams(again)
        assert b2.n_records == 3000
        side.synchronize()
        assert np.array_equal(out.numpy()[:n], ref[:n])
        batch = codec.decode_datagrams(dgrams[2:])  # the same records, templates known
        cap = max(cap, sum(s.block_bytes() + 256 for s in batch.slots))
    with pytest.raises(NgzError):
        codec.columns_to_host_async(out.data_ptr(), 16, stream=side.cuda_stream, kernel=True)  # too small
    pageable = np.zeros(cap, dtype=np.uint8)
    with pytest.raises(NgzError):
        codec.columns_to_host_async(pageable.ctypes.data, cap, kernel=True)  # not mapped for the device


def test_columns_to_host_async_two_streams_then_decode(dev):
    """Two queued column copies of one batch on two different streams (one by the CUs, one by a
    copy engine), then the context's next decode: the decode waits for both (one event chained
    over every queued copy), so both buffers hold the first batch's columns.  A too-small
    destination queues nothing and leaves the earlier copies tracked; the synchronous copy after
    an asynchronous one on another stream waits for both."""
    from netgauze_amd.flow import NgzError
    codec = new_codec()
    first = t20_stream(400_000)
    batch = codec.decode_datagrams(first)
    cap = sum(s.block_bytes() + 256 for s in batch.slots)
    ref = np.zeros(cap, dtype=np.uint8)
    n = codec.columns_to_host(ref.ctypes.data, cap)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    a = torch.zeros(cap, dtype=torch.uint8).pin_memory()
    b = torch.zeros(cap, dtype=torch.uint8).pin_memory()
    assert codec.columns_to_host_async(a.data_ptr(), cap, stream=s1.cuda_stream, kernel=True) == n
    assert codec.columns_to_host_async(b.data_ptr(), cap, stream=s2.cuda_stream, kernel=False) == n
    with pytest.raises(NgzError):
        codec.columns_to_host_async(b.data_ptr(), 16, stream=s2.cuda_stream)
    b2 = codec.decode_datagrams(t20_stream(300_000, seed=99)[1:])  # other records into the same columns
    assert b2.n_records == 300_000
    assert np.array_equal(a.numpy()[:n], ref[:n]) and np.array_equal(b.numpy()[:n], ref[:n])
    # synchronous copy after an asynchronous one on another stream
    batch = codec.decode_datagrams(first[1:])
    a.zero_()
    codec.columns_to_host_async(a.data_ptr(), cap, stream=s1.cuda_stream, kernel=True)
    c = np.zeros(cap, dtype=np.uint8)
    assert codec.columns_to_host(c.ctypes.data, cap) == n
    # (rows past the batch's records in each column are not rewritten: compare the two copies)
    assert np.array_equal(a.numpy()[:n], c[:n])


def test_contexts_decode_concurrently(dev):
    """bench.py --contexts: several contexts, each on its own stream and host thread, decode the
    same device-resident config-4 batch at once (one batch's framing beside another's decode).
    Every context's columns, statuses and processed counts equal one context decoding alone."""
    import threading
    from netgauze_amd import synth
    dg = synth.cfg4_datagrams(200_000)
    buf, offs, lens = synth.host_batch(dg[2:], device=dev)
    torch.cuda.synchronize()

    def column_bytes(codec, batch):
        cap = sum(s.block_bytes() + 256 for s in batch.slots)
        h = np.zeros(cap, dtype=np.uint8)
        n = codec.columns_to_host(h.ctypes.data, cap)
        return h[:n]

    ref = new_codec()
    ref.decode_datagrams(dg[:2])
    b = ref.decode_batch(buf, offs, lens)
    assert b.n_records == 200_000
    want = column_bytes(ref, b)
    last = {}
    codecs = [new_codec() for _ in range(3)]
    for c in codecs:
        c.decode_datagrams(dg[:2])
    streams = [torch.cuda.Stream(dev) for _ in codecs]
    errors = []

    def drive(i):
        try:
            for _ in range(4):
                last[i] = codecs[i].decode_batch(buf, offs, lens, stream=streams[i].cuda_stream)
        except Exception as e:  # surfaced below
            errors.append(e)

    th = [threading.Thread(target=drive, args=(i,)) for i in range(len(codecs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    for i, c in enumerate(codecs):
        assert last[i].n_records == 200_000
        assert np.array_equal(column_bytes(c, last[i]), want)
        assert c.template_counts(10) == {900: 4 * ref.template_counts(10)[900]}
        assert c.template_counts(9) == {313: 4 * ref.template_counts(9)[313]}


def test_netflow_v9_record_lengths_around_staged_limit(dev):
    """NFv9 templates whose records are 26 to 256 bytes, around NGZ_VSTAGE_REC_MAX (160): those up to
    160 bytes decode through the LDS-staged row kernel, longer ones through the chunk kernels; all
    in one batch, interleaved, MTU-style packets of 10 records, against the oracle (both kernel paths).
    A fixed-length interfaceName string pads each record to its length (ASCII, some NUL-truncated)."""
    import random
    rnd = random.Random(913)
    base = [(8, 4), (12, 4), (1, 8), (2, 4), (7, 2), (11, 2), (4, 1), (6, 1)]  # 26 bytes
    lengths = [26, 130, 159, 160, 161, 200, 256]
    tsets, tmpls = b"", {}
    for i, rl in enumerate(lengths):
        tid = 400 + i
        fields = base + ([(82, rl - 26)] if rl > 26 else [])
        body = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", t, n) for t, n in fields)
        tsets += body
        tmpls[tid] = rl
    dgrams = [nf_msg([struct.pack(">HH", 0, 4 + len(tsets)) + tsets], count=len(lengths))]

    def record(rl):
        r = struct.pack(">IIQIHHBB", rnd.getrandbits(32), rnd.getrandbits(32), rnd.getrandbits(64),
                        rnd.getrandbits(32), rnd.getrandbits(16), rnd.getrandbits(16), rnd.choice([6, 17, 1]),
                        rnd.getrandbits(8))
        if rl > 26:
            s = bytes(rnd.choice(b"abcdefghij-_.0123456789") for _ in range(rl - 26))
            if rnd.random() < 0.3:
                k = rnd.randrange(rl - 26)
                s = s[:k] + b"\0" * (rl - 26 - k)
            r += s
        return r

    for p in range(6):
        for tid, rl in tmpls.items():
            recs = b"".join(record(rl) for _ in range(10))
            pad = (-len(recs)) % 4
            dgrams.append(nf_msg([struct.pack(">HH", tid, 4 + len(recs) + pad) + recs + b"\0" * pad], count=10,
                                 seq=100 + p))
    # templates first, then the data as a batch of its own (the steady-state device path)
    codec = new_codec()
    oc = O.FlowInfoCodec()
    codec.decode_datagrams(dgrams[:1])
    parity.oracle_datagrams(dgrams[:1], oc)
    batch = codec.decode_datagrams(dgrams[1:])
    oracle, _ = parity.oracle_datagrams(dgrams[1:], oc)
    stats = parity.check_batch(batch, oracle)
    assert stats["err"] == 0 and stats["records"] == 6 * 10 * len(lengths)
    assert codec.template_counts(9) == {k: v.processed_count for k, v in oc.netflow_templates.items()}


@pytest.mark.parametrize("sizes", [(1, 10, 50, 400), (60, 90, 120)])
def test_netflow_v9_staged_rows_large_packets(dev, sizes):
    """The staged-row NFv9 template kernel on large packets of a 26-byte template: 1-400 records per
    packet make the slot's layout chunk mode (the kernel's chunk branch); 60-120 keep it row mode with
    ~25 000 rows per k_emit workgroup, past its LDS stage (3 072 rows), so the row tables go out by
    direct stores.  Against the oracle, processed counts included."""
    import random
    rnd = random.Random(77 + len(sizes))
    fields = [(8, 4), (12, 4), (1, 8), (2, 4), (7, 2), (11, 2), (4, 1), (6, 1)]
    tset = struct.pack(">HH", 420, len(fields)) + b"".join(struct.pack(">HH", t, n) for t, n in fields)
    dgrams = [nf_msg([struct.pack(">HH", 0, 4 + len(tset)) + tset], count=1)]
    for p in range(900):
        n = rnd.choice(sizes) if p % 3 else sizes[-1]
        recs = b"".join(struct.pack(">IIQIHHBB", rnd.getrandbits(32), rnd.getrandbits(32), rnd.getrandbits(64),
                                    rnd.getrandbits(32), rnd.getrandbits(16), rnd.getrandbits(16), 6, 2)
                        for _ in range(n))
        pad = (-len(recs)) % 4
        dgrams.append(nf_msg([struct.pack(">HH", 420, 4 + len(recs) + pad) + recs + b"\0" * pad], count=n, seq=p))
    codec = new_codec()
    oc = O.FlowInfoCodec()
    codec.decode_datagrams(dgrams[:1])
    parity.oracle_datagrams(dgrams[:1], oc)
    for part in (dgrams[1:], dgrams[1:]):  # twice: the second batch takes the steady-state launches
        batch = codec.decode_datagrams(part)
        oracle, _ = parity.oracle_datagrams(part, oc)
        stats = parity.check_batch(batch, oracle)
        assert stats["err"] == 0 and stats["records"] == sum(struct.unpack(">H", d[2:4])[0] for d in part)
    assert codec.template_counts(9) == {k: v.processed_count for k, v in oc.netflow_templates.items()}

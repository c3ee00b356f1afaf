"""GPU: JSON lines straight from the decoded columns (ngz_dgram_json /
ngz_batch_json), the per-peer collector (ngz_collector_*) and the
`pcap-decoder --protocol flow` path (ngz_pcap_to_jsonl, ngz-pcap-decoder).

The bar is the reference's own golden output, byte for byte: every capture
the reference's flow pcap tests walk (tests/golden/*.jsonl.gz) and the
pcap-decoder integration golden.  Synthetic inputs (config 3/4 shapes, error
paths, stream-framing corner cases) are checked against the CPU oracle's
serde layer and its two drivers (oracle/drivers.py).
"""
import os
import struct
import subprocess

import pytest

import drivers
import golden_io as G
import ngz_oracle as O
from test_gpu_parity import ipfix_msg, ipfix_set, nf_msg, tmpl, vl

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.flow import FlowInfoCodec  # noqa: F401  (loads libngz.so, fails loudly if missing)
    return torch.device("cuda:0")


def oracle_lines(dgrams):
    """Per datagram (datagram mode, one FlowInfoCodec::decode each): the
    oracle's JSON of the FlowInfo or of the error, None for Ok(None)."""
    codec = O.FlowInfoCodec()
    out = []
    for dg in dgrams:
        try:
            m = codec.decode(bytearray(dg))
            out.append(None if m is None else O.dumps(m.to_json()))
        except O.ParseFail as e:
            out.append(O.dumps(e.err))
    return out


def check_batch_json(dgrams, specialize=True):
    from netgauze_amd.flow import FlowInfoCodec
    codec = FlowInfoCodec(0, specialize=specialize)
    batch = codec.decode_datagrams(dgrams)
    exp = oracle_lines(dgrams)
    got = {d: (st, js) for d, st, js, _ in batch.json_lines()}
    for d, e in enumerate(exp):
        if e is None:
            assert d not in got, d
            continue
        assert d in got, "dgram %d: no line, expected %s" % (d, e[:200])
        assert got[d][1] == e, "dgram %d:\n got %s\n exp %s" % (d, got[d][1][:600], e[:600])
    # the per-datagram entry renders the same text
    for d in list(got)[:5]:
        assert batch.json(d) == got[d][1]
    return len(got)


# ---------------------------------------------------------------------------
# reference goldens
# ---------------------------------------------------------------------------
CASES = G.cases()


@pytest.mark.parametrize("name,kind,n", CASES, ids=[c[0] for c in CASES])
def test_collector_matches_reference_golden(dev, name, kind, n):
    """The reference's pcap->JSON goldens through the GPU collector: per-peer
    stream buffers, device decode, JSON rendered from the columns."""
    from netgauze_amd import ingest as I
    mode = I.FLOW_INFO if kind == "pcap_tests" else I.PCAP_DECODER
    col = I.Collector(0, mode)
    for i, (src, sp, dst, dp, payload) in enumerate(G.datagrams(name)):
        col.push(src, sp, dst, dp, payload, tag=i)
    got = [line for _, line in col.flush()]
    exp = G.expected_lines(name)
    assert len(got) == len(exp)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g == e, "line %d:\n got %s\n exp %s" % (i, g[:800], e[:800])


def test_pcap_decoder_502_end_to_end(dev, tmp_path):
    """pcap file -> native capture reader -> GPU -> JSONL, against the
    pcap-decoder integration golden (crates/pcap-decoder/tests/integration_tests.rs)."""
    from netgauze_amd import ingest as I
    pcap = os.path.join(G.GOLDEN, "pcap_decoder__502.pcap")
    exp = G.expected_lines("pcap_decoder__502")
    out = tmp_path / "out.jsonl"
    n = I.pcap_to_jsonl(pcap, [9991], str(out))
    assert n == len(exp)
    assert out.read_text().splitlines() == exp
    # the CLI, flags as the reference's
    cli = os.path.join(ROOT, "netgauze_amd", "bin", "ngz-pcap-decoder")
    r = subprocess.run([cli, "--input", pcap, "--protocol", "flow", "--ports", "9991,9992"],
                       capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode().splitlines() == exp


def test_pcap_decoder_frame_numbers_and_input_count(dev, tmp_path):
    """--show-frame-number wraps {"frame_number","data"}; -c stops at the first
    frame past the count (crates/pcap-decoder/src/lib.rs:98-121)."""
    from netgauze_amd import ingest as I
    pcap = os.path.join(G.GOLDEN, "pcap_decoder__502.pcap")
    exp = G.expected_lines("pcap_decoder__502")
    frames = [f for s, sp, d, dp, proto, pl, f in I.read_pcap(pcap) if proto == I.UDP and dp == 9991]
    assert len(frames) == len(exp)  # one message per datagram in this capture
    out = tmp_path / "f.jsonl"
    I.pcap_to_jsonl(pcap, [9991], str(out), show_frame_number=True)
    assert out.read_text().splitlines() == ['{"frame_number":%d,"data":%s}' % (f, e) for f, e in zip(frames, exp)]
    cut = frames[len(frames) // 2]
    I.pcap_to_jsonl(pcap, [9991], str(out), input_count=cut)
    assert out.read_text().splitlines() == [e for f, e in zip(frames, exp) if f <= cut]
    assert I.pcap_to_jsonl(pcap, [4739], str(out)) == 0


# ---------------------------------------------------------------------------
# synthetic inputs against the oracle's serde layer
# ---------------------------------------------------------------------------
def test_json_t20_and_mixed_templates(dev):
    from netgauze_amd import synth
    rec = synth.t20_records(5000)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64, rec_per_msg=700)
    b = bytes(buf.numpy())
    dgrams = [synth.template_message()] + [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]
    assert check_batch_json(dgrams) == len(dgrams)
    buf, offs, lens, _ = synth.mixed_stream(6000)
    b = bytes(buf.numpy())
    dgrams = [synth.templates_message(synth.CFG3_TEMPLATES)] + [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]
    assert check_batch_json(dgrams) == len(dgrams)


@pytest.mark.parametrize("specialize", [True, False])
def test_json_cfg4_netflow_v9_variable_length(dev, specialize):
    from netgauze_amd import synth
    dgrams = synth.cfg4_datagrams(3000)
    assert check_batch_json(dgrams, specialize) == len(dgrams)


def test_json_errors_and_value_edges(dev):
    """Error lines, leap seconds, NUL-truncated strings, float64 / IPv6 /
    sub-registry / tcpControlBits renderings, vendor and unknown-PEN fields."""
    t = ipfix_msg([ipfix_set(2, tmpl(400, [(152, 8), (154, 8), (82, 8), (7, 2)]))])

    def rec(ms, secs, frac, s, port=1):
        return struct.pack(">QII", ms, secs, frac) + s + struct.pack(">H", port)

    good = rec(1_700_000_000_123, 1_700_000_000, 12345, b"eth0\0\0\0\0")
    fields = [(8, 4), (27, 16), (4, 1), (89, 1), (61, 1), (6, 2), (320, 8), (2011, 2, 2011), (1234, 3, 99999),
              (880, 1, 6876), (138, 8), (276, 1)]
    fields = [f for f in fields if len(f) == 3 or (0, f[0]) in O.REGISTRY.by_key]
    t2 = ipfix_msg([ipfix_set(2, tmpl(401, fields))])
    recs = b""
    for i, v6 in enumerate([b"\0" * 16, b"\x20\x01\x0d\xb8" + b"\0" * 11 + b"\x01", b"\0" * 10 + b"\xff\xff\x0a\0\0\1",
                            bytes(range(16))]):
        parts = []
        for f in fields:
            ie, ln = f[0], f[1]
            if ie == 8:
                parts.append(struct.pack(">I", 0xC0A80000 + i))
            elif ie == 27:
                parts.append(v6)
            elif ie == 4:
                parts.append(bytes([[6, 17, 1, 250][i]]))
            elif ie == 89:
                parts.append(bytes([[64, 66, 130, 255][i]]))
            elif ie == 138 and ln == 8:
                parts.append(struct.pack(">d", [0.1, -2.5e-300, 1e21, 123456789.0][i]))
            else:
                parts.append(bytes((i * 37 + k) & 255 for k in range(ln)))
        recs += b"".join(parts)
    dgrams = [
        t, t2,
        ipfix_msg([ipfix_set(400, good * 3)]),
        ipfix_msg([ipfix_set(400, rec(1, 1_700_000_039, 0xFFFFFFFF, b"ok\0\xff\xfe\0\0\0"))]),  # :59 leap second
        ipfix_msg([ipfix_set(400, good + rec(2**63 + 5, 1, 1, b"ok\0\0\0\0\0\0"))]),       # error line
        ipfix_msg([ipfix_set(400, rec(1, 1, 1, b'q"\\\x01\x1f\x7f\0\0'))]),                   # JSON escapes
        ipfix_msg([ipfix_set(401, recs)]),
        struct.pack(">HHIII", 11, 16, 0, 0, 0),                                              # unsupported version
        b"\x00\x0a\x00",                                                                     # Ok(None): no line
    ]
    assert check_batch_json(dgrams) == len(dgrams) - 1


def test_json_templates_and_netflow_v9(dev):
    tset = struct.pack(">HH", 0, 4 + 4 + 16) + struct.pack(">HH", 260, 4) + struct.pack(">HHHHHHHH", 8, 4, 1, 4, 7, 2, 6, 1)
    oset = struct.pack(">HH", 1, 4 + 6 + 8 + 4 + 2) + struct.pack(">HHH", 270, 8, 4) + \
        struct.pack(">HHHH", 1, 4, 2, 2) + struct.pack(">HH", 34, 4) + b"\0\0"
    rec = struct.pack(">IIHB", 0x0A000001, 1500, 80, 0x12)
    orec = struct.pack(">IHI", 77, 3, 1000)
    dgrams = [
        nf_msg([tset, oset], count=2),
        nf_msg([struct.pack(">HH", 260, 4 + 11 * 3 + 3) + rec * 3 + b"\0\0\0"], count=3),
        nf_msg([struct.pack(">HH", 270, 4 + 10 * 2) + orec * 2, tset], count=3),
        nf_msg([struct.pack(">HH", 260, 4 + 11) + rec, struct.pack(">HH", 260, 4 + 11) + rec], count=1),
        nf_msg([struct.pack(">HH", 260, 4 + 11 * 3) + rec * 3], count=2),  # InvalidCount
        ipfix_msg([ipfix_set(2, tmpl(310, [(8, 4), (7, 2)]) + tmpl(311, [(12, 4)])),
                   ipfix_set(3, struct.pack(">HHH", 320, 2, 1) + struct.pack(">HHHH", 10, 4, 8, 4) + b"\0\0"),
                   ipfix_set(310, struct.pack(">IH", 1, 2) * 2)]),
        ipfix_msg([ipfix_set(320, struct.pack(">II", 7, 0x01020304) * 2), ipfix_set(311, b"\1\2\3\4" + b"\0\0")]),
        ipfix_msg([ipfix_set(2, tmpl(330, [(82, 65535), (7, 2)])),
                   ipfix_set(330, vl(b"ge-0/0/1") + b"\0\x50" + vl("ü".encode()) + b"\0\x51")]),
    ]
    assert check_batch_json(dgrams) == len(dgrams)


# ---------------------------------------------------------------------------
# stream framing (collector speculation) against the oracle drivers
# ---------------------------------------------------------------------------
A = (("v4", 0x0A000001), 4000, ("v4", 0x0A000002), 9991)
B = (("v6", 0x20010DB8 << 96 | 7), 5000, ("v6", 0x20010DB8 << 96 | 1), 9991)


def run_collector(dgrams, mode):
    from netgauze_amd import ingest as I
    col = I.Collector(0, mode)
    for i, (src, sp, dst, dp, pl) in enumerate(dgrams):
        col.push(src, sp, dst, dp, pl, tag=i)
    return [line for _, line in col.flush()], col


def framing_stream():
    t = ipfix_msg([ipfix_set(2, tmpl(300, [(8, 4), (7, 2)]))])
    rec = struct.pack(">IH", 0x0A000001, 80)
    d1 = ipfix_msg([ipfix_set(300, rec * 3)], seq=1)
    d2 = ipfix_msg([ipfix_set(300, rec)], seq=2)
    bad = ipfix_msg([ipfix_set(301, rec)], seq=3)                 # NoTemplateDefinedFor
    nf_t = nf_msg([struct.pack(">HH", 0, 4 + 8) + struct.pack(">HHHH", 260, 1, 8, 4)], count=1)
    nf_d = nf_msg([struct.pack(">HH", 260, 8) + struct.pack(">I", 0x01020304)], count=1)
    return [
        A + (t,),
        A + (d1[:10],), A + (d1[10:],),                           # fragmented message
        A + (d1 + d2,),                                           # two messages in one datagram
        B + (nf_t,), B + (nf_d + b"\x00\x0a",),                   # NFv9 consumed < datagram: 2 bytes carried
        B + (b"\x00\x20" + b"\0" * 12 + d2[:16],),                # ... joined to the next datagram's bytes
        A + (bad + d2,),                                          # error with a tail: decoder clears the buffer
        A + (d2[:3],), A + (d2[3:],),
        A + (struct.pack(">HHIII", 11, 16, 0, 0, 0) + d2,),       # unsupported version + more bytes
        A + (struct.pack(">HHIII", 10, 8, 0, 0, 0) + d2,),        # length < 16 + more bytes
        A + (d2 + t + d1,),
        B + (nf_d + b"\x00\x0a\x00",),                            # 3 carried bytes (remaining > 3 stops parse? no)
        B + (b"\x00\x10" + b"\0" * 40,),
        B + (nf_d,),
    ]


@pytest.mark.parametrize("mode", ["pcap_decoder", "flow_info"])
def test_collector_stream_framing(dev, mode):
    from netgauze_amd import ingest as I
    dg = framing_stream()
    if mode == "pcap_decoder":
        exp = drivers.run_pcap_decoder_driver(dg)
        got, col = run_collector(dg, I.PCAP_DECODER)
    else:
        exp = drivers.run_pcap_tests_driver(dg)
        got, col = run_collector(dg, I.FLOW_INFO)
    assert col.peers() == 2
    assert len(got) == len(exp), (got, exp)
    for i, (g, e) in enumerate(zip(got, exp)):
        assert g == e, "line %d:\n got %s\n exp %s" % (i, g, e)


def test_collector_rollback_discards_speculative_templates(dev):
    """A NetFlow v9 message leaves 2 bytes in the buffer; the next datagram (a
    template) is then misread and the buffer cleared, so the template must not
    be learnt although the speculative batch decoded it."""
    from netgauze_amd import ingest as I
    t = ipfix_msg([ipfix_set(2, tmpl(300, [(8, 4), (7, 2)]))])
    rec = struct.pack(">IH", 0x0A000001, 80)
    nf_t = nf_msg([struct.pack(">HH", 0, 4 + 8) + struct.pack(">HHHH", 260, 1, 8, 4)], count=1)
    nf_d = nf_msg([struct.pack(">HH", 260, 8) + struct.pack(">I", 1)], count=1)
    dg = [A + (nf_t,), A + (nf_d + b"\x01\x02",), A + (t,), A + (ipfix_msg([ipfix_set(300, rec)]),)]
    for mode, drv in ((I.PCAP_DECODER, drivers.run_pcap_decoder_driver), (I.FLOW_INFO, drivers.run_pcap_tests_driver)):
        got, _ = run_collector(dg, mode)
        assert got == drv(dg)
    assert "NoTemplateDefinedFor" in got[-1]


def test_collector_flushes_keep_partial_messages(dev):
    """A message split across flushes stays buffered (BytesMut) and decodes
    once its last datagram arrives."""
    from netgauze_amd import ingest as I
    t = ipfix_msg([ipfix_set(2, tmpl(300, [(8, 4), (7, 2)]))])
    d1 = ipfix_msg([ipfix_set(300, struct.pack(">IH", 7, 9) * 4)])
    col = I.Collector(0, I.PCAP_DECODER)
    col.push(*A, t, tag=1)
    col.push(*A, d1[:20], tag=2)
    first = col.flush()
    col.push(*A, d1[20:], tag=3)
    second = col.flush()
    exp = drivers.run_pcap_decoder_driver([A + (t,), A + (d1[:20],), A + (d1[20:],)])
    assert [l for _, l in first + second] == exp
    assert [tag for tag, _ in first + second] == [1, 3]

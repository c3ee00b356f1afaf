"""CPU tests of the host ingest (include/ngz/flow_ingest.h), no GPU needed:

* the C++ capture reader (≙ netgauze_pcap_reader::PcapIter) on the
  reference's own captures (tests/golden/*.pcap) must yield exactly the
  datagrams the golden fixtures were extracted with (tests/golden/*.dgrams),
  and on synthetic captures (pcap LE/BE, micro/nanosecond, pcapng with
  several interfaces, Linux cooked, raw IP, 802.1Q / QinQ, IPv6, Ethernet
  padding, non-IP frames) the payloads written into them;
* the recvmmsg UDP reader on loopback sockets.
"""
import os
import socket
import struct

import pytest

import golden_io as G

pytestmark = pytest.mark.filterwarnings("ignore")

PCAP_CASES = [(n, k) for n, k, _ in G.cases() if os.path.exists(os.path.join(G.GOLDEN, n + ".pcap"))]


def ingest():
    from netgauze_amd import ingest as I
    return I


@pytest.mark.parametrize("name,kind", PCAP_CASES)
def test_pcap_reader_matches_golden_extraction(name, kind):
    """pcap_tests.rs:80-84 filter (UDP to 9991/9992/10088), pcap-decoder golden: 9991."""
    I = ingest()
    ports = (9991,) if kind == "pcap_decoder" else (9991, 9992, 10088)
    got = [(s, sp, d, dp, pl) for s, sp, d, dp, proto, pl, _ in I.read_pcap(os.path.join(G.GOLDEN, name + ".pcap"))
           if proto == I.UDP and dp in ports]
    exp = G.datagrams(name)
    assert len(got) == len(exp)
    assert got == exp


def test_pcap_reader_frame_counter_counts_every_frame():
    """frame_counter increments for every packet record, extracted or not (lib.rs:150,179)."""
    I = ingest()
    frames = [f for *_, f in I.read_pcap(os.path.join(G.GOLDEN, "pcap_decoder__502.pcap"))]
    assert frames == sorted(frames) and len(set(frames)) == len(frames)
    data = open(os.path.join(G.GOLDEN, "pcap_decoder__502.pcap"), "rb").read()
    pos, n = 24, 0
    while pos + 16 <= len(data):
        pos += 16 + struct.unpack("<I", data[pos + 8:pos + 12])[0]
        n += 1
    assert frames[-1] <= n


# ---------------------------------------------------------------------------
# synthetic captures
# ---------------------------------------------------------------------------
def _csum_free_ipv4(src, dst, proto, l4, pad_total=0):
    total = 20 + len(l4) + pad_total
    return struct.pack(">BBHHHBBH4s4s", 0x45, 0, total, 0, 0, 64, proto, 0, src, dst) + l4 + b"\0" * pad_total


def _udp(sp, dp, payload, extra=0):
    return struct.pack(">HHHH", sp, dp, 8 + len(payload), 0) + payload + b"\xee" * extra


def _ipv6(src, dst, nh, l4):
    return struct.pack(">IHBB16s16s", 6 << 28, len(l4), nh, 64, src, dst) + l4


ETH = b"\x00\x11\x22\x33\x44\x55\x66\x77\x88\x99\xaa\xbb"


def _frames(dgrams):
    """(linktype, frame bytes, expected (src, sp, dst, dp, payload) or None) covering the link/L3 shapes."""
    out = []
    for i, (src, sp, dst, dp, pl) in enumerate(dgrams):
        v = i % 6
        if src[0] == "v4":
            s4, d4 = src[1].to_bytes(4, "big"), dst[1].to_bytes(4, "big")
            # UDP trailer bytes beyond the UDP length are cut (lib.rs:306-321); Ethernet padding too
            ip = _csum_free_ipv4(s4, d4, 17, _udp(sp, dp, pl, extra=3 if v == 1 else 0))
            et = b"\x08\x00"
        else:
            s6, d6 = src[1].to_bytes(16, "big"), dst[1].to_bytes(16, "big")
            ip = _ipv6(s6, d6, 17, _udp(sp, dp, pl))
            et = b"\x86\xdd"
        exp = (src, sp, dst, dp, pl)
        if v == 0:
            out.append((1, ETH + et + ip + b"\0" * 6, exp))
        elif v == 1:
            out.append((1, ETH + b"\x81\x00\x00\x0a" + et + ip, exp))               # 802.1Q (pdu unwraps)
        elif v == 2:
            out.append((1, ETH + b"\x88\xa8\x00\x0b\x81\x00\x00\x0c" + et + ip, exp))  # QinQ (strip_vlan_tags)
        elif v == 3:
            out.append((113, b"\0\0\0\1\0\6" + b"\0" * 8 + et + ip, exp))            # Linux cooked
        elif v == 4:
            out.append((101, ip, exp))                                               # raw IP
        else:
            out.append((1, ETH + b"\x08\x06" + b"\0" * 28, None))                      # ARP: skipped, counted
            out.append((1, ETH + et + ip, exp))
    return out


def _legacy(frames, be=False, nanos=False):
    e = ">" if be else "<"
    magic = 0xA1B23C4D if nanos else 0xA1B2C3D4
    lt = frames[0][0]
    out = struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, 65535, lt)
    for _, fr, _ in frames:
        out += struct.pack(e + "IIII", 1700000000, 5, len(fr), len(fr)) + fr
    return out


def _pcapng(frames):
    def block(t, body):
        body += b"\0" * (-len(body) % 4)
        n = 12 + len(body)
        return struct.pack("<II", t, n) + body + struct.pack("<I", n)
    lts = sorted({lt for lt, _, _ in frames})
    out = block(0x0A0D0D0A, struct.pack("<IHHq", 0x1A2B3C4D, 1, 0, -1))
    for lt in lts:
        out += block(1, struct.pack("<HHI", lt, 0, 65535))
    out += block(5, b"\0" * 8)  # an interface statistics block is skipped
    for lt, fr, _ in frames:
        out += block(6, struct.pack("<IIIII", lts.index(lt), 0, 0, len(fr), len(fr)) + fr)
    return out


@pytest.mark.parametrize("shape", ["ng", "le", "be_ns"])
def test_pcap_reader_link_and_vlan_shapes(tmp_path, shape):
    I = ingest()
    dg = G.datagrams("110-IPFIXv10-NFv9-multiple-sources__traffic-00") + G.datagrams("pcap_decoder__502")[:20]
    frames = _frames(dg)
    if shape == "ng":
        blob = _pcapng(frames)
    else:  # legacy files have one link type: keep the Ethernet frames only
        frames = [f for f in frames if f[0] == 1]
        blob = _legacy(frames, be=shape.startswith("be"), nanos=shape.endswith("ns"))
    p = tmp_path / "x.pcap"
    p.write_bytes(blob)
    got = list(I.read_pcap(str(p)))
    exp = [f[2] for f in frames if f[2] is not None]
    assert [(s, sp, d, dp, pl) for s, sp, d, dp, _, pl, _ in got] == exp
    assert [f for *_, f in got] == [i + 1 for i, f in enumerate(frames) if f[2] is not None]


def test_pcap_reader_rejects_garbage(tmp_path):
    I = ingest()
    p = tmp_path / "bad.pcap"
    p.write_bytes(b"not a capture at all....")
    with pytest.raises(ValueError):
        list(I.read_pcap(str(p)))
    p.write_bytes(_legacy(_frames(G.datagrams("pcap_decoder__502")[:2])[:1])[:-5])  # truncated record
    with pytest.raises(ValueError):
        list(I.read_pcap(str(p)))


def test_udp_recv_batches_loopback_datagrams():
    I = ingest()
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.bind(("127.0.0.1", 0))
    try:
        msgs = [G.datagrams("pcap_decoder__502")[i][4] for i in range(5)] + [b"x" * 9000]
        for m in msgs:
            tx.sendto(m, rx.getsockname())
        got = []
        while len(got) < len(msgs):
            batch = I.udp_recv(rx.fileno(), max_dgrams=4, timeout_ms=2000)
            assert batch, "timeout"
            got += batch
        assert [g[4] for g in got] == msgs
        src = ("v4", int.from_bytes(socket.inet_aton("127.0.0.1"), "big"))
        for s, sp, d, dp, _ in got:
            assert (s, sp) == (src, tx.getsockname()[1])
            assert (d, dp) == (src, rx.getsockname()[1])
        assert I.udp_recv(rx.fileno(), timeout_ms=0) == []
    finally:
        rx.close()
        tx.close()

"""Host ingest over the C ABI of include/ngz/flow_ingest.h.

Mirrors the reference's feeding side of FlowInfoCodec:

* ``read_pcap``   ≙ ``netgauze_pcap_reader::PcapIter`` (crates/pcap-reader/src/lib.rs:141-377):
  yields ``(src_ip, src_port, dst_ip, dst_port, proto, payload, frame)``.
* ``Collector``   ≙ the per-exporter-peer ``(FlowInfoCodec, BytesMut)`` map of the pcap
  decoder (crates/pcap-decoder/src/handlers/flow.rs:37-59, handlers/mod.rs:36-80) and of the
  flow pcap tests (crates/flow-pkt/src/wire/tests/pcap_tests.rs:79-118); decoding runs on
  the GPU, one batch per peer per ``flush``.
* ``udp_recv``    ≙ the collector's UDP socket read, batched with recvmmsg(2).
* ``pcap_to_jsonl`` ≙ ``pcap-decoder --protocol flow`` (crates/pcap-decoder/src/lib.rs:65-127).

IP addresses are ``("v4", int)`` / ``("v6", int)``, as in the test fixtures.
"""
import ctypes

import numpy as np

from netgauze_amd import _lib

UDP, TCP = _lib.NGZ_PROTO_UDP, _lib.NGZ_PROTO_TCP
PCAP_DECODER, FLOW_INFO = _lib.NGZ_COLLECT_PCAP_DECODER, _lib.NGZ_COLLECT_FLOW_INFO

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _lib.load()
    return _LIB


def _ip(fam, raw):
    b = bytes(raw)
    return ("v4", int.from_bytes(b[:4], "big")) if fam == 4 else ("v6", int.from_bytes(b, "big"))


def peer_key(src, sport, dst, dport):
    k = _lib.PeerKey()
    fam = 4 if src[0] == "v4" else 6
    k.family = fam
    n = 4 if fam == 4 else 16
    k.src[:n] = list(src[1].to_bytes(n, "big"))
    k.dst[:n] = list(dst[1].to_bytes(n, "big"))
    k.src_port, k.dst_port = sport, dport
    return k


def read_pcap(path):
    """Every UDP/TCP payload of a capture, in capture order."""
    L = lib()
    h = ctypes.c_void_p()
    rc = L.ngz_pcap_open(path.encode(), ctypes.byref(h))
    if rc:
        raise ValueError("ngz_pcap_open(%s) = %d" % (path, rc))
    try:
        pk = _lib.Packet()
        while True:
            rc = L.ngz_pcap_next(h, ctypes.byref(pk))
            if rc == 0:
                return
            if rc < 0:
                raise ValueError("ngz_pcap_next: malformed capture (%d)" % rc)
            k = pk.key
            payload = ctypes.string_at(pk.payload, pk.len) if pk.len else b""
            yield (_ip(k.family, k.src), k.src_port, _ip(k.family, k.dst), k.dst_port, int(pk.proto), payload,
                   int(pk.frame))
    finally:
        L.ngz_pcap_close(h)


class Collector:
    """One FlowInfoCodec + stream buffer per exporter peer, decoded on the GPU."""

    def __init__(self, device=0, mode=PCAP_DECODER):
        self._h = ctypes.c_void_p()
        rc = lib().ngz_collector_create(device, mode, ctypes.byref(self._h))
        if rc:
            raise RuntimeError("ngz_collector_create = %d" % rc)

    def close(self):
        if self._h:
            lib().ngz_collector_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, src, sport, dst, dport, payload, tag=0):
        k = peer_key(src, sport, dst, dport)
        buf = ctypes.create_string_buffer(bytes(payload), max(1, len(payload)))
        rc = lib().ngz_collector_push(self._h, ctypes.byref(k), buf, len(payload), tag)
        if rc:
            raise RuntimeError("ngz_collector_push = %d: %s" % (rc, lib().ngz_collector_last_error(self._h).decode()))

    def flush(self):
        """Decode everything queued; returns [(tag, line)] in push order."""
        out = []

        def cb(_user, tag, line, n):
            out.append((int(tag), ctypes.string_at(line, n).decode("utf-8")))
            return 0

        fn = _lib.COLLECT_LINE_FN(cb)
        n = lib().ngz_collector_flush(self._h, fn, None)
        if n < 0:
            raise RuntimeError("ngz_collector_flush = %d: %s" % (n, lib().ngz_collector_last_error(self._h).decode()))
        return out

    def peers(self):
        return int(lib().ngz_collector_peers(self._h))


def udp_recv(sock_fd, max_dgrams=64, timeout_ms=100):
    """recvmmsg batch: [(src_ip, src_port, dst_ip, dst_port, payload)]."""
    slot = 65536
    buf = np.empty(slot * max_dgrams, dtype=np.uint8)
    keys = (_lib.PeerKey * max_dgrams)()
    offs = np.zeros(max_dgrams, dtype=np.uint64)
    lens = np.zeros(max_dgrams, dtype=np.uint32)
    n = lib().ngz_udp_recv(sock_fd, buf.ctypes.data, buf.size, keys, offs.ctypes.data, lens.ctypes.data, max_dgrams,
                           timeout_ms)
    if n < 0:
        raise OSError("ngz_udp_recv = %d" % n)
    out = []
    for i in range(n):
        k = keys[i]
        o, ln = int(offs[i]), int(lens[i])
        out.append((_ip(k.family, k.src), k.src_port, _ip(k.family, k.dst), k.dst_port, buf[o:o + ln].tobytes()))
    return out


def pcap_to_jsonl(pcap_path, ports, out_path, device=0, input_count=-1, show_frame_number=False):
    arr = (ctypes.c_uint16 * len(ports))(*ports)
    n = lib().ngz_pcap_to_jsonl(pcap_path.encode(), arr, len(ports), out_path.encode() if out_path else None, device,
                                input_count, 1 if show_frame_number else 0)
    if n < 0:
        raise RuntimeError("ngz_pcap_to_jsonl = %d" % n)
    return n

"""CPU ORACLE helper — test infrastructure only.

Restatement of crates/pcap-reader/src/lib.rs:141-377 for the capture shapes
the reference's flow goldens use (legacy pcap, Ethernet link type, optional
single 802.1Q tag, IPv4/IPv6, UDP): yields
(src_ip, src_port, dst_ip, dst_port, proto, payload).  IPv4 UDP payloads are
trimmed to the UDP length (lib.rs:298-312); IPv6 ones are not (:355-366).
IPs are ('v4', int) / ('v6', int).
"""
import struct

UDP, TCP = "UDP", "TCP"


def _parse_l3(ethertype, data):
    if ethertype == 0x0800:
        return _ipv4(data)
    if ethertype == 0x86DD:
        return _ipv6(data)
    return None


def _ipv4(d):
    if len(d) < 20:
        return None
    ihl = (d[0] & 0x0F) * 4
    total = struct.unpack(">H", d[2:4])[0]
    proto = d[9]
    src = ("v4", struct.unpack(">I", d[12:16])[0])
    dst = ("v4", struct.unpack(">I", d[16:20])[0])
    body = d[ihl:total] if total >= ihl else d[ihl:]
    if proto == 17:
        if len(body) < 8:
            return None
        sp, dp, ulen = struct.unpack(">HHH", body[:6])
        payload = body[8:]
        n = ulen - 8
        assert n <= len(payload), "Invalid UDP payload length calculation"
        return (src, sp, dst, dp, UDP, bytes(payload[:n]))
    if proto == 6:
        if len(body) < 20:
            return None
        sp, dp = struct.unpack(">HH", body[:4])
        off = (body[12] >> 4) * 4
        return (src, sp, dst, dp, TCP, bytes(body[off:]))
    return None


def _ipv6(d):
    if len(d) < 40:
        return None
    nh = d[6]
    plen = struct.unpack(">H", d[4:6])[0]
    src = ("v6", int.from_bytes(d[8:24], "big"))
    dst = ("v6", int.from_bytes(d[24:40], "big"))
    body = d[40:40 + plen]
    if nh == 17:
        if len(body) < 8:
            return None
        sp, dp = struct.unpack(">HH", body[:4])
        return (src, sp, dst, dp, UDP, bytes(body[8:]))
    if nh == 6:
        if len(body) < 20:
            return None
        sp, dp = struct.unpack(">HH", body[:4])
        off = (body[12] >> 4) * 4
        return (src, sp, dst, dp, TCP, bytes(body[off:]))
    return None


def iter_pcap(path):
    with open(path, "rb") as f:
        data = f.read()
    magic = data[:4]
    if magic == b"\xd4\xc3\xb2\xa1":
        end = "<"
    elif magic == b"\xa1\xb2\xc3\xd4":
        end = ">"
    else:
        raise ValueError("not a legacy pcap: %r" % magic)
    linktype = struct.unpack(end + "I", data[20:24])[0]
    if linktype != 1:
        raise ValueError("unsupported link type %d" % linktype)
    pos = 24
    while pos + 16 <= len(data):
        _, _, caplen, _ = struct.unpack(end + "IIII", data[pos:pos + 16])
        frame = data[pos + 16:pos + 16 + caplen]
        pos += 16 + caplen
        if len(frame) < 14:
            continue
        et = struct.unpack(">H", frame[12:14])[0]
        body = frame[14:]
        if et == 0x8100:  # single 802.1Q tag unwrapped by the pdu crate
            if len(body) < 4:
                continue
            et = struct.unpack(">H", body[2:4])[0]
            body = body[4:]
            while et in (0x8100, 0x88A8):  # stacked tags: strip_vlan_tags
                if len(body) < 4:
                    body = None
                    break
                et = struct.unpack(">H", body[2:4])[0]
                body = body[4:]
            if body is None:
                continue
        r = _parse_l3(et, body)
        if r is not None:
            yield r

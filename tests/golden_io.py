"""Readers for the tests/golden/ fixtures (see tests/golden/make_golden.py)."""
import gzip
import os
import struct

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cases():
    out = []
    with open(os.path.join(GOLDEN, "cases.txt")) as f:
        for line in f:
            name, kind, n = line.split()
            out.append((name, kind, int(n)))
    return out


def _ip(ver, raw):
    v = int.from_bytes(raw, "big")
    return ("v4", v & 0xFFFFFFFF) if ver == 4 else ("v6", v)


def datagrams(name):
    """[(src_ip, src_port, dst_ip, dst_port, payload)] in capture order."""
    with open(os.path.join(GOLDEN, name + ".dgrams"), "rb") as f:
        d = f.read()
    out = []
    pos = 0
    while pos < len(d):
        ver = d[pos]
        src = _ip(ver, d[pos + 1:pos + 17])
        sp = struct.unpack(">H", d[pos + 17:pos + 19])[0]
        dst = _ip(ver, d[pos + 19:pos + 35])
        dp = struct.unpack(">H", d[pos + 35:pos + 37])[0]
        n = struct.unpack(">I", d[pos + 37:pos + 41])[0]
        out.append((src, sp, dst, dp, d[pos + 41:pos + 41 + n]))
        pos += 41 + n
    return out


def expected_lines(name):
    with gzip.open(os.path.join(GOLDEN, name + ".jsonl.gz"), "rb") as f:
        return f.read().decode("utf-8").splitlines()

#!/usr/bin/env python3
"""Build tests/golden/ from the reference's own golden data files.

Run in the build container (needs /root/reference, read-only).  For every
flow pcap the reference's pcap_tests.rs walks (assets/pcaps/pmacct-tests/*/
*.pcap and assets/pcaps/flow/*/*.pcap, pcap_tests.rs:27-43) with a non-empty
*-flow.json, and for the pcap-decoder integration golden
(crates/pcap-decoder/tests/data/502-...-flow.jsonl), store:

  <name>.dgrams  the UDP datagrams the reference test driver feeds its codecs
                 (dst port filter 9991/9992/10088 as pcap_tests.rs:80-84, or
                 9991 for the pcap-decoder golden) in capture order, framed as
                 u8 ip-version, 16 B src ip, u16 src port, 16 B dst ip,
                 u16 dst port, u32 payload length, payload
  <name>.jsonl.gz the reference's expected output lines, verbatim (gzip)
  <name>.pcap     (--pcaps) the capture itself, for captures up to 50 kB and the
                 pcap-decoder golden: input of the product's pcap reader

Extraction uses oracle/pcap.py; the goldens then pin both the extraction and
the decoder (a wrong datagram would produce a mismatching line).
"""
import glob
import gzip
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import pcap  # noqa: E402

REF = "/root/reference"


def pack_ip(ip):
    ver, v = ip
    return struct.pack(">B", 4 if ver == "v4" else 6) + v.to_bytes(16, "big")


def write_case(name, pcap_path, ports, json_path):
    out = bytearray()
    n = 0
    for src, sp, dst, dp, proto, payload in pcap.iter_pcap(pcap_path):
        if proto != pcap.UDP or dp not in ports:
            continue
        out += pack_ip(src) + struct.pack(">H", sp) + pack_ip(dst)[1:] + struct.pack(">H", dp)
        out += struct.pack(">I", len(payload)) + payload
        n += 1
    with open(os.path.join(HERE, name + ".dgrams"), "wb") as f:
        f.write(out)
    with open(json_path, "rb") as f:
        text = f.read()
    with open(os.path.join(HERE, name + ".jsonl.gz"), "wb") as raw:
        with gzip.GzipFile(fileobj=raw, mode="wb", mtime=0, filename="") as f:
            f.write(text)
    return n


PCAP_FIXTURE_MAX = 50_000  # copy the small captures themselves (the product's pcap reader reads them)


def copy_pcaps():
    """<name>.pcap: the reference's own capture files (data its tests hold),
    for the captures up to PCAP_FIXTURE_MAX bytes and the pcap-decoder golden."""
    import shutil
    n = 0
    for p in sorted(glob.glob(REF + "/assets/pcaps/pmacct-tests/*/*.pcap") + glob.glob(REF + "/assets/pcaps/flow/*/*.pcap")):
        j = p[:-len(".pcap")] + "-flow.json"
        if not os.path.exists(j) or os.path.getsize(j) == 0 or os.path.getsize(p) > PCAP_FIXTURE_MAX:
            continue
        name = os.path.basename(os.path.dirname(p)) + "__" + os.path.basename(p)[:-5]
        shutil.copyfile(p, os.path.join(HERE, name + ".pcap"))
        n += 1
    shutil.copyfile(REF + "/crates/pcap-decoder/tests/data/502-IPFIXv10-BGP-IPv6-CISCO-SRv6-lcomms.pcap",
                    os.path.join(HERE, "pcap_decoder__502.pcap"))
    print("copied %d captures + pcap_decoder__502.pcap" % n)


def main():
    if "--pcaps" in sys.argv:
        return copy_pcaps()
    cases = []
    for p in sorted(glob.glob(REF + "/assets/pcaps/pmacct-tests/*/*.pcap") + glob.glob(REF + "/assets/pcaps/flow/*/*.pcap")):
        j = p[:-len(".pcap")] + "-flow.json"
        if not os.path.exists(j) or os.path.getsize(j) == 0:
            continue
        name = os.path.basename(os.path.dirname(p)) + "__" + os.path.basename(p)[:-5]
        n = write_case(name, p, (9991, 9992, 10088), j)
        cases.append((name, "pcap_tests", n))
    p = REF + "/crates/pcap-decoder/tests/data/502-IPFIXv10-BGP-IPv6-CISCO-SRv6-lcomms.pcap"
    n = write_case("pcap_decoder__502", p, (9991,), p[:-5] + "-flow.jsonl")
    cases.append(("pcap_decoder__502", "pcap_decoder", n))
    with open(os.path.join(HERE, "cases.txt"), "w") as f:
        for name, kind, n in cases:
            f.write("%s %s %d\n" % (name, kind, n))
    print("\n".join("%s %s %d" % c for c in cases))


if __name__ == "__main__":
    main()

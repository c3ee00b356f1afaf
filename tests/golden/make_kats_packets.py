"""Extract the wire byte arrays of the reference's packet-level unit tests into
a data fixture (tests/golden/kats_packets.json).

Run in the build container, where the reference checkout exists:
    python tests/golden/make_kats_packets.py [/root/reference]

Only the *input* byte arrays are extracted (data, not source): every
`let NAME = [ ... ];` / `const NAME: &[u8] = &[ ... ];` literal inside the
listed test functions (and `let NAME: Vec<u8> = vec![ ... ];`), keyed "file:function:variable", with the line it was
found on.  The expected results those tests assert are restated by hand in
tests/kats_packets.py next to the citation of each assertion.
"""
import json
import os
import re
import sys

FILES = [
    "crates/flow-pkt/src/codec.rs",
    "crates/flow-pkt/src/wire/tests/mod.rs",
    "crates/flow-pkt/src/wire/tests/ipfix.rs",
    "crates/flow-pkt/src/wire/tests/netflow.rs",
    "crates/flow-pkt/benches/serde_benchmark.rs",
    "crates/parse-utils/src/reader.rs",
]

_FN = re.compile(r"^\s*(?:pub\s+)?fn\s+(\w+)\s*\(")
_LET = re.compile(r"^\s*(?:let\s+(?:mut\s+)?(\w+)\s*(?::\s*Vec<u8>\s*=\s*vec!|=\s*)|const\s+(\w+)\s*:\s*&\[u8\]\s*=\s*&)\[(.*)$")
_NUM = re.compile(r"0x[0-9a-fA-F]+|\d+")


def extract(path):
    out = {}
    fn = "<top>"
    lines = open(path, encoding="utf-8").read().split("\n")
    i = 0
    while i < len(lines):
        line = lines[i]
        m = _FN.match(line)
        if m:
            fn = m.group(1)
        m = _LET.match(line)
        if m:
            name = m.group(1) or m.group(2)
            start = i + 1
            body = m.group(3)
            seg = body
            while "]" not in seg.split("//")[0]:
                i += 1
                seg = lines[i]
                body += "\n" + seg
            text = "\n".join(seg.split("//")[0] for seg in body.split("\n"))
            text = text.split("]")[0]
            vals = [int(t, 0) for t in _NUM.findall(text)]
            if vals and all(0 <= v <= 255 for v in vals) and "u8" not in text and "(" not in text:
                out["%s:%s" % (fn, name)] = {"line": start, "hex": bytes(vals).hex()}
        i += 1
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    fixture = {}
    for rel in FILES:
        for k, v in extract(os.path.join(ref, rel)).items():
            fixture["%s:%s" % (os.path.basename(rel), k)] = dict(v, file=rel)
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats_packets.json")
    with open(dst, "w") as f:
        json.dump(fixture, f, indent=1, sort_keys=True)
    print("%d arrays -> %s" % (len(fixture), dst))


if __name__ == "__main__":
    main()

"""Regression vectors for divergences the differential fuzz corpus found (tests/test_gpu_fuzz.py),
kept after their fix and run through both kernel paths by test_fuzz_regressions.  Data only:
datagram batches (hex) a codec decodes in order.  Regenerate with
    python tests/golden/make_fuzz_regressions.py
"""
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.dirname(os.path.dirname(HERE))]

import fuzz_corpus as F  # noqa: E402
from netgauze_amd import synth  # noqa: E402


def ipfix(sets, t=1_700_000_000, seq=1, dom=1):
    body = b"".join(sets)
    return struct.pack(">HHIII", 10, 16 + len(body), t, seq, dom) + body


def dset(tid, payload):
    return struct.pack(">HH", tid, 4 + len(payload)) + payload


def vl(b):
    return (bytes([len(b)]) if len(b) < 255 else b"\xff" + len(b).to_bytes(3, "big")) + b


def v900_record(name, blob=b"x", ven=b"hw", ms=1_700_000_000_000):
    # V900: (8,4) (12,4) (82,vlen str) (7,2) (11,2) (4,1) (1,8) (2,8) (96,vlen str) (880,1,6876)
    #       (951,vlen,6876) (960,vlen,6876) (1000,vlen,2011) (152,8)
    return (struct.pack(">II", 1, 2) + vl(name) + struct.pack(">HHBQQ", 80, 443, 6, 1, 2) + vl(b"app") + b"\x01" +
            vl(b"uuid") + vl(blob) + vl(ven) + struct.pack(">Q", ms))


def main():
    vecs = []
    # 1. an invalid vlen string in a record whose later field runs past the set: the record's error
    #    is the Utf8Error (DataRecord::parse reads the string first), not the UnexpectedEof the walk
    #    meets later (found in stream mode, fixed by ngz_partial_record_err)
    tm = synth._ipfix_template_v900()
    good = v900_record(b"eth0")
    bad = v900_record(b"ab\xc3\x28cd")
    vecs.append({"name": "utf8_before_walk_eof", "proto": 10, "dgrams": [
        tm.hex(),
        ipfix([dset(900, good + bad[:-5])]).hex(),            # bad string, then EOF in the last field
        ipfix([dset(900, good + bad + good[:20])]).hex(),     # complete bad record: Utf8Error as before
        ipfix([dset(900, bad[:30])]).hex(),                    # EOF inside the string's own bytes: EOF
    ]})
    # 2. a dateTimeMilliseconds out of chrono's range before a later EOF in the same record (the
    #    all-decode-rules template of the corpus)
    name, ztm, zmsgs = F._zoo()
    rec = bytearray(zmsgs[0][20:])  # the first message's records (a set of 1 record)
    off = sum(ln for ie, ln, *_ in F.ZOO[:3])  # the 152 field
    rec[off:off + 8] = b"\x7f" * 8
    vecs.append({"name": "dtms_before_walk_eof", "proto": 10, "dgrams": [
        ztm[0].hex() if isinstance(ztm, list) else ztm.hex(),
        ipfix([dset(700, bytes(rec[:-3]))], dom=3).hex(),
    ]})
    # 3. 1100 identical re-announcements of a template between data messages in one batch: each reuses
    #    the current version (the batch held one template version per announcement and failed with
    #    NGZ_E_LIMIT past 1024), and processed_count restarts at every announcement -- across
    #    datagrams and inside one ([data][template][data] counts 1)
    t20 = synth.template_message()
    recs = synth.t20_records(64).numpy().tobytes()
    d = ipfix([dset(256, recs[:128])])
    dg = []
    for k in range(1100):
        dg += [t20, d] if k % 3 else [t20]
    dg.append(ipfix([dset(256, recs[:64]), F_tset(), dset(256, recs[64:192])]))
    vecs.append({"name": "template_reannounced_1100_times", "proto": 10, "dgrams": [x.hex() for x in dg]})
    with open(os.path.join(HERE, "fuzz_regressions.json"), "w") as f:
        json.dump(vecs, f, indent=0)
    print(len(vecs), "vectors")


def F_tset():
    t = synth.template_message()
    return t[16:]  # the template set of the T20 announcement


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Config 1 timing: the pcap-decoder golden capture through the GPU path
(native capture reader -> per-peer GPU batches -> JSON from the columns)
vs the CPU oracle's restatement of the reference pcap-decoder on the same
datagrams.  Correctness is tests/test_gpu_jsonl.py; this prints wall times."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import golden_io as G  # noqa: E402

pcap = os.path.join(G.GOLDEN, "pcap_decoder__502.pcap")
exp = G.expected_lines("pcap_decoder__502")
out = "/tmp/ngz_502.jsonl"
res = {"capture": "crates/pcap-decoder/tests/data/502-IPFIXv10-BGP-IPv6-CISCO-SRv6-lcomms.pcap",
       "lines": len(exp), "bytes_json": sum(len(e) + 1 for e in exp)}
cli = os.path.join(ROOT, "netgauze_amd", "bin", "ngz-pcap-decoder")
t0 = time.perf_counter()
r = subprocess.run([cli, "-i", pcap, "-o", out, "--protocol", "flow", "--ports", "9991"], capture_output=True)
res["cli_wall_s"] = time.perf_counter() - t0
assert r.returncode == 0 and open(out).read().splitlines() == exp, r.stderr
from netgauze_amd import ingest  # noqa: E402
ts = []
for _ in range(5):
    t0 = time.perf_counter()
    ingest.pcap_to_jsonl(pcap, [9991], out)
    ts.append(time.perf_counter() - t0)
assert open(out).read().splitlines() == exp
res["in_process_s"] = {"first": ts[0], "warm_min": min(ts[1:])}
import drivers  # noqa: E402
dg = G.datagrams("pcap_decoder__502")
t0 = time.perf_counter()
got = drivers.run_pcap_decoder_driver(dg)
res["cpu_oracle_python_s"] = time.perf_counter() - t0
assert got == exp
print(json.dumps(res))

#!/usr/bin/env python3
"""Summarize a tools/gpu_profile.sh output directory.

  * per-kernel rocprofv3 --kernel-trace --stats of the bench command;
  * the decode kernel's average duration over the TIMED steps only (the last
    `steps` dispatches in the per-dispatch kernel trace: warm-up launches and
    the first batch's arena placement trials are excluded), to compare with the
    bench line's HIP-event kernel_ms of the same run;
  * per-launch HBM traffic of the decode kernel from the separate --pmc passes
    (FETCH_SIZE doubled on gfx950 per MI355X_MICROARCH.md §HBM; both KiB).

Writes <dir>/traffic.json stamped with the product source hash and the decode
sources' hash (netgauze_amd/buildinfo.py) and, when GIT_SHA is set, the commit.
usage: summarize_profile.py <dir> [decode-kernel-substring ...]
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from netgauze_amd import buildinfo  # noqa: E402

d = sys.argv[1]
DECODE = sys.argv[2:] or ["ngz_tpl", "k_decode_generic"]
bench = None
tb = os.path.join(d, "trace_bench.json")
if os.path.exists(tb):
    bench = json.loads(open(tb).read().strip().splitlines()[-1])

rows = []
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    rows += list(csv.DictReader(open(f)))
print("== rocprofv3 --kernel-trace --stats")
print("%-44s %8s %14s %14s" % ("kernel", "calls", "avg_ns", "total_ns"))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    short = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print("%-44s %8s %14.0f %14s" % (short[:44], r["Calls"], float(r["AverageNs"]), r["TotalDurationNs"]))

timed = None
traces = glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))
if traces and bench:
    disp = []
    for r in csv.DictReader(open(traces[0])):
        if any(k in r["Kernel_Name"] for k in DECODE):
            disp.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    disp.sort()
    steps = bench["steps"]
    # one step may launch several decode kernels (one per active template): group by step is not
    # needed for the average per step; take the last `steps` steps' worth of dispatches
    per_step = max(1, round(len(disp) / max(1, bench["steps"] + bench["warmup"])))
    last = disp[-steps * per_step:]
    if last:
        timed = sum(x for _, x in last) / steps / 1e6  # ms of decode kernel per step
        print("== decode kernel over the %d timed steps: %.4f ms/step (%d dispatches); bench kernel_ms %.4f"
              % (steps, timed, len(last), bench["roofline"]["kernel_ms"]))

out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals, frames = {}, []
    for f in glob.glob(os.path.join(d, "pmc_" + c, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            i = int(r["Dispatch_Id"])
            if "k_frame" in r["Kernel_Name"]:
                frames.append(i)
            if any(k in r["Kernel_Name"] for k in DECODE):
                vals[i] = vals.get(i, 0.0) + float(r["Counter_Value"])
    if vals:
        # one step may launch several decode kernels (one per active template): the
        # decode dispatches after the last step's framing kernel, summed
        last = max(frames) if frames else -1
        out[c] = sum(v for i, v in vals.items() if i > last)
print("== PMC per step's decode launches (the last step's dispatches, summed)")
for c, v in out.items():
    print("%s = %.0f KiB" % (c, v))
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    fetch = out["FETCH_SIZE"] * 1024 * 2  # gfx950: FETCH_SIZE reads half of a wide streaming read
    write = out["WRITE_SIZE"] * 1024
    alg = bench["roofline"]["alg_bytes_per_launch"] if bench else None
    print("traffic_bytes_per_launch = %.0f (fetch %.0f + write %.0f)%s" % (
        fetch + write, fetch, write, "; algorithmic %.0f, ratio %.3f" % (alg, (fetch + write) / alg) if alg else ""))
    json.dump({"fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
               "records": bench["config"]["records_per_gpu"] if bench else None,
               "workload": bench["config"]["workload"] if bench else None,
               "alg_bytes_per_launch": alg, "traffic_over_alg": (fetch + write) / alg if alg else None,
               "timed_kernel_ms_trace": timed, "bench_kernel_ms": bench["roofline"]["kernel_ms"] if bench else None,
               "source_hash": buildinfo.source_hash(), "decode_source_hash": buildinfo.decode_source_hash(),
               "git_sha": os.environ.get("GIT_SHA"),
               "kernel": "decode (every decode dispatch of one step)",
               "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950 "
                         "wide-read correction, MI355X_MICROARCH.md HBM)"},
              open(os.path.join(d, "traffic.json"), "w"), indent=1)

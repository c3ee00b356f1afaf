#!/usr/bin/env python3
"""Summarize a tools/gpu_profile.sh output directory.

  * per-kernel rocprofv3 --kernel-trace --stats of the bench command;
  * the decode kernel time per TIMED step (every decode dispatch from the
    k_frame that starts the first timed step on: warm-up steps and the first
    batch's arena placement trials are excluded), to compare with the bench
    line's HIP-event kernel_ms of the same run; it must not exceed ms_per_step;
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

timed, per_step_disp = None, None
traces = glob.glob(os.path.join(d, "trace", "*kernel_trace.csv"))
if traces and bench:
    disp, frames = [], []
    for r in csv.DictReader(open(traces[0])):
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if any(k in r["Kernel_Name"] for k in DECODE):
            disp.append((t0, t1 - t0))
        if "k_frame" in r["Kernel_Name"]:
            frames.append(t0)
    disp.sort()
    frames.sort()
    steps = bench["steps"]
    # Each ngz_decode_batch starts with its k_frame dispatch, so the timed steps are the last
    # `steps` k_frame starts onwards: warm-up steps and the first batch's placement trials (extra
    # decode dispatches without a k_frame of their own) fall before them.  (r4 guessed the
    # dispatches per step from the total count, which the trials inflate.)
    if len(frames) < steps:
        sys.exit("summarize_profile: %d k_frame dispatches for %d timed steps" % (len(frames), steps))
    start = frames[-steps]
    last = [x for t, x in disp if t >= start]
    if last:
        timed = sum(last) / steps / 1e6  # ms of decode kernel per step
        per_step_disp = len(last) / steps
        print("== decode kernel over the %d timed steps: %.4f ms/step (%d dispatches, %.2f per step); "
              "bench kernel_ms %.4f, ms_per_step %.4f"
              % (steps, timed, len(last), per_step_disp, bench["roofline"]["kernel_ms"], bench["ms_per_step"]))
        if timed > bench["ms_per_step"]:
            sys.exit("summarize_profile: decode time per step %.4f ms exceeds the step %.4f ms -- the step "
                     "delimiting is wrong" % (timed, bench["ms_per_step"]))

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
               "timed_kernel_ms_trace": timed, "timed_dispatches_per_step": per_step_disp,
               "ms_per_step_trace_run": bench["ms_per_step"] if bench else None, "bench_kernel_ms": bench["roofline"]["kernel_ms"] if bench else None,
               "source_hash": buildinfo.source_hash(), "decode_source_hash": buildinfo.decode_source_hash(),
               "git_sha": os.environ.get("GIT_SHA"),
               "kernel": "decode (every decode dispatch of one step)",
               "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950 "
                         "wide-read correction, MI355X_MICROARCH.md HBM)"},
              open(os.path.join(d, "traffic.json"), "w"), indent=1)

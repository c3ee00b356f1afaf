#!/usr/bin/env python3
"""Summarize a tools/gpu_round.sh output directory: per-kernel stats
for the decode pipeline and per-launch HBM traffic of the decode kernel (FETCH_SIZE is
doubled on gfx950 per MI355X_MICROARCH.md §HBM; both are KiB)."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
rows = []
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    rows += list(csv.DictReader(open(f)))
print("== rocprofv3 --kernel-trace --stats (pipeline kernels)")
print("%-40s %8s %14s %14s" % ("kernel", "calls", "avg_ns", "total_ns"))
for r in rows:
    name = r["Name"]
    short = name.replace("(anonymous namespace)::", "").split("(")[0]
    if any(k in name for k in ("k_decode_generic", "ngz_tpl", "k_frame", "k_emit", "k_layout", "k_counts", "k_finalize", "rocprim", "fillBuffer")):
        print("%-40s %8s %14.0f %14s" % (short[:40], r["Calls"], float(r["AverageNs"]), r["TotalDurationNs"]))
out = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = {}
    for f in glob.glob(os.path.join(d, "pmc_" + c, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "ngz_tpl" in r["Kernel_Name"] or "k_decode_generic" in r["Kernel_Name"]:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    if vals:
        big = max(vals.values())
        out[c] = big
print("== PMC per decode-kernel launch (largest dispatch = bench batch)")
for c, v in out.items():
    print("%s = %.0f KiB" % (c, v))
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    fetch = out["FETCH_SIZE"] * 1024 * 2  # gfx950: FETCH_SIZE reads half of a wide streaming read
    write = out["WRITE_SIZE"] * 1024
    print("traffic_bytes_per_launch = %.0f (fetch %.0f + write %.0f)" % (fetch + write, fetch, write))
    rec = None
    tb = os.path.join(d, "trace_bench.json")
    if os.path.exists(tb):
        rec = json.loads(open(tb).read().strip().splitlines()[-1])["config"]["records_per_gpu"]
    json.dump({"fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write, "records": rec,
               "kernel": "ngz_tpl (largest dispatch)", "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, "
               "separate passes; FETCH_SIZE x2 (gfx950 wide-read correction, MI355X_MICROARCH.md HBM)"},
              open(os.path.join(d, "traffic.json"), "w"))

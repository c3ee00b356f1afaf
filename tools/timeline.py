#!/usr/bin/env python3
"""Print one bench step's kernel timeline (gaps between dispatches) from a
rocprofv3 --kernel-trace CSV: tools/timeline.py gpurun_out/<tag>/trace/run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "ngz_tpl" in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
t0 = int(rows[a]["End_Timestamp"])
prev = t0
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f us  dur %8.1f  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, r["Kernel_Name"][:70]))
    prev = e
print("step (decode end to decode end): %.1f us" % ((int(rows[b]["End_Timestamp"]) - t0) / 1e3))

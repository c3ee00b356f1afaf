#!/usr/bin/env python3
"""Per-dispatch durations of one bench step's decode kernels from a rocprofv3
--kernel-trace directory: the dispatches between the last two k_frame launches
(one ngz_decode_batch), with grid, workgroup, LDS and VGPR figures.
usage: tools/dispatches.py gpurun_out/<tag>/trace_<case>"""
import csv
import glob
import re
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
def base(name):
    m = re.search(r"(\w+)\(", name)
    return m.group(1) if m else name.split("::")[-1]


frames = [i for i, r in enumerate(rows) if base(r["Kernel_Name"]) == "k_frame"]
a, b = frames[-2], frames[-1]
t0 = int(rows[a]["Start_Timestamp"])
tot = 0.0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = base(r["Kernel_Name"])[:28]
    get = lambda k: r.get(k, "?")  # noqa: E731
    print("%9.1f us  dur %8.1f  grid %8s  wg %4s  lds %6s  vgpr %4s  %s" % (
        (s - t0) / 1e3, (e - s) / 1e3, get("Grid_Size"), get("Workgroup_Size"), get("LDS_Block_Size"),
        get("VGPR_Count") if "VGPR_Count" in r else get("Arch_VGPR_Count"), name))
    if name.startswith("ngz_tpl"):
        tot += (e - s) / 1e3
print("sum of ngz_tpl durations: %.1f us; step span %.1f us" % (tot, (int(rows[b]["Start_Timestamp"]) - t0) / 1e3))

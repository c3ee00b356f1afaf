#!/usr/bin/env python3
"""Per-dispatch counters of several rocprofv3 --pmc --kernel-trace passes of the same command,
joined by dispatch order, with kernel names and derived rates.  Only the last dispatches of each
kernel name are shown (the timed step).  usage: pmc_table.py REGEX DIR [DIR ...]"""
import collections
import csv
import glob
import re
import sys


def load(d, rx):
    names, durs = {}, {}
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                i = int(r["Dispatch_Id"])
                names[i] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                durs[i] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ctr = collections.defaultdict(dict)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                i = int(r["Dispatch_Id"])
                ctr[i][r["Counter_Name"]] = ctr[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                names.setdefault(i, r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0])
    ids = sorted(names)
    return [(names[i], durs.get(i), ctr.get(i, {})) for i in ids]


def main():
    rx = re.compile(sys.argv[1])
    passes = [load(d, rx) for d in sys.argv[2:]]
    n = min(len(p) for p in passes)
    rows = []
    for k in range(n):
        name = passes[0][k][0]
        c, durs = {}, []
        for p in passes:
            assert p[k][0] == name, (k, p[k][0], name)
            c.update(p[k][2])
            durs.append(p[k][1])
        rows.append((name, durs, c))
    last = {}
    for k, (name, _, _) in enumerate(rows):
        last.setdefault(name, []).append(k)
    show = sorted(k for ks in last.values() for k in ks[-4:])
    for k in show:
        name, durs, c = rows[k]
        us = min(d for d in durs if d) if any(durs) else 0
        line = "%-18s %8.1f us" % (name[:18], us)
        if "FETCH_SIZE" in c:
            gb_f, gb_w = 2 * c["FETCH_SIZE"] * 1024 / 1e9, c.get("WRITE_SIZE", 0) * 1024 / 1e9
            line += "  fetch(x2) %.3f GB write %.3f GB  %.2f TB/s" % (gb_f, gb_w, (gb_f + gb_w) / us * 1e-3 if us else 0)
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            wc = c["SQ_WAVE_CYCLES"]
            line += "  waves %d wait %.0f%% waitinst %.0f%% busy %.3g valu/wave %.0f vmem r/w/wave %.1f/%.1f" % (
                c.get("SQ_WAVES", 0), 100 * c.get("SQ_WAIT_ANY", 0) / wc, 100 * c.get("SQ_WAIT_INST_ANY", 0) / wc,
                c.get("SQ_BUSY_CYCLES", 0), c.get("SQ_INSTS_VALU", 0) / max(1, c.get("SQ_WAVES", 1)),
                c.get("SQ_INSTS_VMEM_RD", 0) / max(1, c.get("SQ_WAVES", 1)),
                c.get("SQ_INSTS_VMEM_WR", 0) / max(1, c.get("SQ_WAVES", 1)))
        if "SQ_INSTS_LDS" in c:
            line += "  lds/wave %.0f bankconf %.3g salu/wave %.0f smem/wave %.0f" % (
                c["SQ_INSTS_LDS"] / max(1, c.get("SQ_WAVES", 1)), c.get("SQ_LDS_BANK_CONFLICT", 0),
                c.get("SQ_INSTS_SALU", 0) / max(1, c.get("SQ_WAVES", 1)),
                c.get("SQ_INSTS_SMEM", 0) / max(1, c.get("SQ_WAVES", 1)))
        print(line)


if __name__ == "__main__":
    main()

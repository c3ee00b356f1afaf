#!/usr/bin/env python3
"""Per-dispatch counters beside per-dispatch durations, from rocprofv3 runs made with
`--pmc ... --kernel-trace --output-format csv` (one directory per pass; the passes run the same
command, so dispatch k of one pass is dispatch k of the next).  Kernels matching REGEX only.
usage: python tools/pmc_dispatch.py REGEX DIR [DIR ...]"""
import csv
import collections
import glob
import re
import sys


def load(d, rx):
    durs = {}
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                durs[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    ctr = collections.defaultdict(dict)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                i = int(r["Dispatch_Id"])
                ctr[i][r["Counter_Name"]] = ctr[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(set(durs) | set(ctr))
    return [(durs.get(i), ctr.get(i, {})) for i in ids]


def main():
    rx = re.compile(sys.argv[1])
    passes = [load(d, rx) for d in sys.argv[2:]]
    n = max(len(p) for p in passes)
    names = []
    for p in passes:
        for _, c in p:
            for k in c:
                if k not in names:
                    names.append(k)
    print("%4s " % "#" + " ".join("%9s" % ("us.p%d" % i) for i in range(len(passes))) + " " +
          " ".join("%14s" % k[:14] for k in names))
    for k in range(n):
        durs, vals = [], {}
        for p in passes:
            if k < len(p):
                durs.append(p[k][0])
                vals.update(p[k][1])
            else:
                durs.append(None)
        print("%4d " % k + " ".join("%9.1f" % d if d is not None else "%9s" % "-" for d in durs) + " " +
              " ".join("%14.4g" % vals[m] if m in vals else "%14s" % "-" for m in names))


if __name__ == "__main__":
    main()

#!/bin/bash
# HBM traffic of the aggregation push kernels (FETCH_SIZE / WRITE_SIZE, separate passes),
# per dispatch, averaged over the steady-state pushes of bench.py --agg.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aggtraffic}
mkdir -p $OUT
K=${AGG_KEY:-5tuple}
N=${RECORDS:-100000000}
CMD="python3 bench.py --agg $K --steps 2 --warmup 1 --records $N"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $OUT/rd -o run -- $CMD > $OUT/rd.json 2> $OUT/rd.err || { tail -5 $OUT/rd.err; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE TCC_EA0_ATOMIC_sum TCC_MISS_sum --output-format csv -d $OUT/wr -o run -- $CMD > $OUT/wr.json 2> $OUT/wr.err || { tail -5 $OUT/wr.err; exit 2; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:40]
        if "k_agg" in k:
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(agg.items()):
    # the last two dispatches of each kernel are the timed steady-state pushes
    print(k, {m: "%.4g" % (sum(v[-2:]) / len(v[-2:])) for m, v in sorted(c.items())})
PY

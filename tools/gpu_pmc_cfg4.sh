#!/bin/bash
# HBM bytes per kernel of a config 4 step (FETCH_SIZE / WRITE_SIZE in separate passes): how much
# of the batch the framing reads besides the decode.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_cfg4}
mkdir -p $OUT
CMD="python3 bench.py --workload cfg4 --records ${RECORDS:-20000000} --steps 2 --warmup 1 --no-cpu-baseline"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o run -- $CMD > $OUT/$C.json 2> $OUT/$C.err || { tail -5 $OUT/$C.err; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob("%s/%s/*counter_collection.csv" % (d, c)):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[:30]
            per[(k, r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in per.items():
            res[k][c].append(v)
print("per dispatch, last dispatch of each kernel (KB; FETCH_SIZE x2 = bytes on gfx950 for wide streaming reads)")
for k in ("k_frame", "k_emit", "k_counts", "k_layout", "ngz_tpl"):
    if k in res:
        print(k, {c: "%.4g" % v[-1] for c, v in res[k].items()}, "dispatches", len(res[k]["FETCH_SIZE"]))
PY

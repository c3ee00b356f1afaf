#!/bin/bash
# PMC passes (one per run) over the aggregation bench: wave-cycle breakdown, HBM bytes,
# per record kernel (averaged over its dispatches).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aggpmc}
mkdir -p $OUT
K=${AGG_KEY:-5tuple}
N=${RECORDS:-20000000}
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 bench.py --agg $K --steps 2 --warmup 1 --records $N > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; exit 1; }
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES
run fetch FETCH_SIZE
run write WRITE_SIZE
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ("sq", "fetch", "write", "tcc"):
    for f in glob.glob("%s/%s/*counter_collection.csv" % (out, sub)):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
            if "k_agg" not in k:
                continue
            per[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, d, c), v in per.items():
            res[k][c].append(v)
for k in sorted(res):
    print(k, " ".join("%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(res[k].items())))
PY

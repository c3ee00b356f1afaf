#!/bin/bash
# SQ / TCC counters of the framing kernels on config 4 (separate passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_frame}
mkdir -p $OUT
CMD="python3 bench.py --workload cfg4 --records ${RECORDS:-4000000} --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o run -- $CMD > $OUT/sq.json 2> $OUT/sq.err || { tail -5 $OUT/sq.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/tcc -o run -- $CMD > $OUT/tcc.json 2> $OUT/tcc.err || { tail -5 $OUT/tcc.err; exit 2; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for f in glob.glob(d + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:30]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
for k, c in agg.items():
    if any(x in k for x in ("k_frame", "k_emit", "ngz_tpl", "k_counts")):
        print(k, {m: "%.3g" % (v / max(1, n[(k, m)])) for m, v in sorted(c.items())})
PY

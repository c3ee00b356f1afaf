#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each) over one bench.py command, summed per kernel
# matching KREGEX.  usage: KREGEX=k_agg_lc_part ARGS="--agg proto_dir --steps 1 --warmup 0" \
#   PASSES="SQ_WAVES SQ_WAVE_CYCLES;SQ_INSTS_VALU SQ_INSTS_LDS" bash tools/gpu_pmc_kernel.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmck}
mkdir -p $OUT
IFS=';' read -ra PS <<< "$PASSES"
i=0
for pc in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pc --kernel-include-regex "$KREGEX" --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS --no-cpu-baseline > $OUT/p$i.json 2> $OUT/p$i.err || { tail -5 $OUT/p$i.err; exit 3; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        tot[(r["Kernel_Name"][:40], r["Counter_Name"])] += float(r["Counter_Value"])
        n[(r["Kernel_Name"][:40], r["Counter_Name"])] += 1
for k in sorted(tot):
    print("%-40s %-24s %16.0f  (%d rows)" % (k[0], k[1], tot[k], n[k]))
PY

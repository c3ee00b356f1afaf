#!/bin/bash
# Round 6: config 3 with its template launches serialized on one stream (NGZ_DECODE_STREAMS=1) and the
# column stride padded or not (experiment build; drop ./tools/exp from .gpurunignore for this call).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6stride
mkdir -p $OUT
for rep in 1 2; do
  for pad in 0 85449; do
    NGZ_EXPERIMENTS=1 NGZ_DECODE_STREAMS=1 NGZ_CAP_PAD=$pad NGZ_PLACE_TRIALS=1 timeout -k 10 200 python bench.py --workload mixed8 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/cfg3s1_pad${pad}_$rep.json 2> $OUT/cfg3s1_pad${pad}_$rep.err || { echo FAIL $pad; tail -5 $OUT/cfg3s1_pad${pad}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], sys.argv[3], r['kernel_ms'], r['frac'], d['ms_per_step'])" $OUT/cfg3s1_pad${pad}_$rep.json $pad $rep
  done
done

#!/bin/bash
# A/B one env knob over workloads: VAR=NAME VALS="a b" WORKLOADS="t20 mixed8"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for w in ${WORKLOADS:-t20}; do
  for v in ${VALS}; do
    env $VAR=$v timeout -k 10 300 python bench.py --workload $w --records ${REC:-100000000} --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b_${w}_$v.json 2> $OUT/b_${w}_$v.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'ms_per_step %.3f' % d['ms_per_step'])" $OUT/b_${w}_$v.json "$w $VAR=$v"
  done
done

#!/bin/bash
# A/B arbitrary env settings: CASES="A:ENV=1,ENV2=2 B:ENV=3" WORKLOADS="t20 mixed8"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab3}
mkdir -p $OUT
for w in ${WORKLOADS:-t20}; do
  for c in ${CASES}; do
    name=${c%%:*}; envs=${c#*:}
    env $(echo $envs | tr ',' ' ') timeout -k 10 300 python bench.py --workload $w --records ${REC:-100000000} --steps 10 --warmup 3 --no-cpu-baseline > $OUT/b_${w}_$name.json 2> $OUT/b_${w}_$name.err || { tail -5 $OUT/b_${w}_$name.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'ms_per_step %.3f' % d['ms_per_step'])" $OUT/b_${w}_$name.json "$w $name"
  done
done

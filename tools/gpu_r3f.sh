#!/bin/bash
# r3 re-entry check at HEAD: every -m gpu test, smoke(), then one bench line per workload / aggregation key.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3f}
mkdir -p $OUT
bash tools/gpu_tests_all.sh || exit 1
cp gpurun_out/pytest_gpu.log $OUT/
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
for W in ${WLS:-t20 mixed8 cfg5 cfg4}; do
  A="--workload $W --steps 20 --warmup 5 --no-cpu-baseline"
  [ $W = cfg4 ] && A="$A --records 20000000"
  timeout -k 10 300 python bench.py $A > $OUT/$W.json 2> $OUT/$W.err || { tail -5 $OUT/$W.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/$W.json')); print('$W', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), 'step', round(d['ms_per_step'],4), d['value'])"
done
for K in ${AGGS:-proto_dir dport 5tuple}; do
  timeout -k 10 300 python bench.py --agg $K --steps 10 --warmup 2 > $OUT/agg_$K.json 2> $OUT/agg_$K.err || { tail -5 $OUT/agg_$K.err; exit 4; }
  python -c "import json; d=json.load(open('$OUT/agg_$K.json')); print('$K', d['path'], round(d['push_kernels_ms'],3), 'first', round(d['config']['first_push_ms'],3), 'groups', d['config']['groups'])"
done

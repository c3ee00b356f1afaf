#!/bin/bash
# r3: aggregation GPU tests (low-cardinality path), bench --agg x3, config 3 group A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3d
( while sleep 20; do date >> gpurun_out/r3d/ticks.txt; done ) &
TK=$!
timeout -k 10 900 python -u -m pytest ${R3D_TESTS:-tests/test_gpu_agg.py} ${R3D_K:+-k "$R3D_K"} -q -x --timeout 300 --timeout-method thread > gpurun_out/r3d/pytest.log 2>&1
rc=$?
kill $TK
tail -15 gpurun_out/r3d/pytest.log
[ $rc -eq 0 ] || exit $rc
for K in ${AGGS:-proto_dir dport 5tuple}; do
  timeout -k 10 300 python bench.py --agg $K --steps 10 --warmup 2 > gpurun_out/r3d/agg_$K.json 2> gpurun_out/r3d/agg_$K.err || { tail -5 gpurun_out/r3d/agg_$K.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/r3d/agg_$K.json')); print('$K', d['path'], round(d['push_kernels_ms'],3), 'first', round(d['config']['first_push_ms'],3), 'groups', d['config']['groups'])"
done
for G in ${GROUPS_AB:-1 0}; do
  NGZ_GROUP=$G timeout -k 10 300 python bench.py --workload mixed8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3d/mixed8_g$G.json 2> gpurun_out/r3d/mixed8_g$G.err || exit 4
  python -c "import json; d=json.load(open('gpurun_out/r3d/mixed8_g$G.json')); print('mixed8 group=$G', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['ms_per_step'],4))"
done

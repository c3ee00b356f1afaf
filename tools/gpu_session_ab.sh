#!/bin/bash
# Aggregation GPU tests, then per-kernel breakdowns of every bench key (first push included).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/pytest_agg.log 2>&1 || { grep -v "^    " gpurun_out/pytest_agg.log | tail -40; exit 1; }
tail -1 gpurun_out/pytest_agg.log
for K in ${KEYS:-dport proto_dir 5tuple}; do
  TAG=agg_$K AGG_KEY=$K CONFIGS="X=1" bash tools/gpu_agg_ab.sh || exit 2
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ms_per_step %.2f first_push_ms %.2f' % (d['ms_per_step'], d['config']['first_push_ms']))" gpurun_out/agg_$K/b1.json $K
done

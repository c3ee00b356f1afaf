#!/bin/bash
# Aggregation GPU tests, then an aggregation A/B (CONFIGS) through tools/gpu_agg_ab.sh.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_agg.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_agg.log
[ $rc = 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_agg.log | head -30; exit 1; }
bash tools/gpu_agg_ab.sh

#!/bin/bash
# GPU tests then a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu -x ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -v "^    " gpurun_out/pytest_gpu.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --records ${REC:-100000000} --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
exit $rc

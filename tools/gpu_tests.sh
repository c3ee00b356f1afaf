#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -v "^    " gpurun_out/pytest_gpu.log | tail -60
exit $rc

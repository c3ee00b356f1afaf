#!/bin/bash
# Every -m gpu test, verbose, no early stop, a ticker under gpurun_out so a slow run is not taken for a hang.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( while sleep 20; do date >> gpurun_out/ticks.txt; done ) &
TK=$!
timeout -k 10 1000 python -u -m pytest tests/ -v -m gpu --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
kill $TK
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | grep -v PASSED | head -20
tail -3 gpurun_out/pytest_gpu.log
exit $rc

#!/bin/bash
# first GPU contact: a few parity tests and a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "t20_small or framing or steady" > gpurun_out/pytest1.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --records 10000000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench1.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -20 gpurun_out/bench1.log
exit $rc

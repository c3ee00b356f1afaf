set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( while sleep 20; do date >> gpurun_out/ticks.txt; done ) &
TK=$!
timeout -k 10 500 python -u -m pytest tests/test_gpu_dist.py -v -m gpu -x -s --timeout 400 --timeout-method thread > gpurun_out/pytest_dist.log 2>&1
rc=$?
kill $TK
tail -60 gpurun_out/pytest_dist.log
exit $rc

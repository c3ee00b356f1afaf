#!/bin/bash
# Round 5 correctness pass on one GPU box: smoke(), every -m gpu test (a ticker keeps the
# run visibly alive), then the T20 and config-4 bench lines.  usage: TAG=r5a bash tools/gpu_r5_check.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r5}
mkdir -p $OUT
( while sleep 20; do date >> $OUT/ticks.txt; done ) &
TK=$!
trap "kill $TK" EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 2; }
timeout -k 10 1500 python -u -m pytest tests/ -v -m gpu --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -20
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/t20.json 2> $OUT/t20.err && cat $OUT/t20.json
timeout -k 10 300 python bench.py --workload cfg4 --records 20000000 --steps 20 --warmup 5 > $OUT/cfg4.json 2> $OUT/cfg4.err && cat $OUT/cfg4.json
exit $rc

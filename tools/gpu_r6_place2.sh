#!/bin/bash
# Round 6: the kept arena used without a re-decode -- the placement GPU test, then the T20 line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6place2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_placement.py tests/test_gpu_async.py > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" $OUT/tests.log | head -20; tail -20 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/t20.json 2> $OUT/t20.err && cat $OUT/t20.json

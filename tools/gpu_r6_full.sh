#!/bin/bash
# Round 6 end: every -m gpu test in one invocation, as the driver runs it (a ticker keeps the run visibly alive).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6full
mkdir -p $OUT
( while sleep 20; do date >> $OUT/ticks.txt; done ) &
TK=$!
trap "kill $TK" EXIT
timeout -k 10 1100 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
exit $rc

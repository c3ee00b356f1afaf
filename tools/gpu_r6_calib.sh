#!/bin/bash
# Round 6: FETCH_SIZE / WRITE_SIZE against known bytes for the aggregation's random
# row shapes (tools/fetch_calib, built on the CPU with hipcc), one --pmc pass per counter.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6calib
mkdir -p $OUT
timeout -k 10 120 ./tools/fetch_calib > $OUT/plain.txt 2>&1 || { echo FAIL plain; cat $OUT/plain.txt; exit 1; }
cat $OUT/plain.txt
i=0
for pc in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pc --kernel-trace --output-format csv -d $OUT/p$i -o run -- ./tools/fetch_calib > $OUT/p$i.txt 2>&1 || { echo FAIL pass $i; tail -5 $OUT/p$i.txt; exit 3; }
done
python3 tools/pmc_dispatch.py "stream_read|rand_" $OUT/p1 $OUT/p2 > $OUT/pmc.txt && cat $OUT/pmc.txt

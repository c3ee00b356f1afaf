#!/bin/bash
# Round 6 end, on one GPU box.  PART=a: smoke() and every -m gpu test but the fuzz corpus (a ticker keeps
# the run visibly alive).  PART=b: the fuzz corpus tests, then the T20 profile (tools/gpu_profile.sh);
# PART=p: the config 3 / config 5 profiles.  PART=c: the config-4 profile (tools/gpu_r5_cfg4.sh) and the default bench line.
# usage: TAG=r6f PART=a bash tools/gpu_r6_final.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r6f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
( while sleep 20; do date >> $OUT/ticks_${PART}.txt; done ) &
TK=$!
trap "kill $TK" EXIT
case "$PART" in
a)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 2; }
  tail -2 $OUT/smoke.log
  timeout -k 10 1000 python -u -m pytest tests/ -v -m gpu -k "not fuzz" --timeout 240 --timeout-method thread > $OUT/pytest_gpu_a.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" $OUT/pytest_gpu_a.log | head -20
  tail -3 $OUT/pytest_gpu_a.log
  exit $rc
  ;;
b)
  timeout -k 10 700 python -u -m pytest tests/ -v -s -m gpu -k "fuzz" --timeout 600 --timeout-method thread > $OUT/pytest_gpu_b.log 2>&1 || { echo FUZZ_FAILED; grep -E "FAILED|ERROR" $OUT/pytest_gpu_b.log | head; tail -5 $OUT/pytest_gpu_b.log; exit 1; }
  tail -3 $OUT/pytest_gpu_b.log
  TAG=$TAG WORKLOADS="t20" bash tools/gpu_profile.sh
  ;;
p)
  TAG=$TAG WORKLOADS="${WORKLOADS:-mixed8 cfg5}" bash tools/gpu_profile.sh
  ;;
c)
  TAG=$TAG/cfg4 bash tools/gpu_r5_cfg4.sh || exit $?
  timeout -k 10 300 python bench.py > $OUT/t20_default.json 2> $OUT/t20_default.err && cat $OUT/t20_default.json
  ;;
esac

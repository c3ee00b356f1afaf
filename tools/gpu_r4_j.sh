#!/bin/bash
# r4: XCD phase rotation (NGZ_WIN_ROT) on mid-size and full-size T20 and config 3, parity first.
# usage: TAG=r4j bash tools/gpu_r4_j.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4j}
mkdir -p $OUT
NGZ_WIN_ROT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --timeout 200 --timeout-method thread \
  -k "t20 or cfg3_mixed_templates_1e7 or cfg5_sixteen" > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
CASES="n4=--workload t20 --records 12500000;t20=--workload t20;mixed8=--workload mixed8" SETTINGS="r0=;r1=NGZ_WIN_ROT=1;r2=NGZ_WIN_ROT=2" \
  STEPS=20 TAG=${TAG:-r4j}/rot bash tools/gpu_sweep.sh || exit 3

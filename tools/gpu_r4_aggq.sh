#!/bin/bash
# r4: scatter with 4 consecutive records per thread (wide operand loads): parity, then the three
# aggregation profiles (traffic.json for this source)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r4q2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py tests/test_gpu_jsonl.py -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
TAG=r4q2 AGGS="dport proto_dir 5tuple" bash tools/gpu_profile_agg.sh || exit 3

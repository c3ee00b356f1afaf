#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r4red
mkdir -p $OUT
NGZ_AGG_RED_THREADS=1024 timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -v -m gpu --timeout 300 --timeout-method thread -k partitioned > $OUT/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for T in 256 512 1024; do
  NGZ_AGG_RED_THREADS=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t$T -o run -- \
    python3 bench.py --agg dport --steps 5 --warmup 1 > $OUT/t$T.json 2> $OUT/t$T.err || { tail -5 $OUT/t$T.err; exit 3; }
  python3 -c "import json; d=json.load(open('$OUT/t$T.json')); print('reduce threads $T: push %.3f ms' % d['push_kernels_ms'])"
  grep -h "k_agg_part_reduce" $OUT/t$T/run_kernel_stats.csv | cut -d, -f1-4
done

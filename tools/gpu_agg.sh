#!/bin/bash
# Aggregation evidence on one GPU box: parity tests, bench lines per key set, rocprofv3 stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-agg}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_agg.log 2>&1 || { tail -40 $OUT/pytest_agg.log; exit 1; }
tail -3 $OUT/pytest_agg.log
for K in ${AGG_KEYS:-proto_dir dport 5tuple}; do
  timeout -k 10 300 python bench.py --agg $K --steps 10 --warmup 2 > $OUT/bench_agg_$K.json 2> $OUT/bench_agg_$K.err || { tail -20 $OUT/bench_agg_$K.err; exit 2; }
  cat $OUT/bench_agg_$K.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --agg dport --steps 5 --warmup 1 > $OUT/trace_agg.json 2> $OUT/trace.err || exit 3
head -12 $OUT/trace/run_kernel_stats.csv | cut -c1-200

#!/bin/bash
# GPU parity suite (verbose, ticker), then the config 4 per-kernel breakdown at 2e7 records.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests_all.sh || exit 1
TAG=cfg4 BENCH_ARGS="--workload cfg4 --records 20000000 --steps 5 --warmup 2 --no-cpu-baseline" CONFIGS="X=1" bash tools/gpu_trace_ab.sh || exit 3

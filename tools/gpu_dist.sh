#!/bin/bash
# Multi-rank product path on the one-GPU box: the 2-rank GPU test, then a
# 2-rank bench rehearsal (ranks share the GPU, gloo carries the count exchange).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dist}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py -k "two_ranks or counts_device or wide" -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_dist.log 2>&1 || { tail -40 $OUT/pytest_dist.log; exit 1; }
tail -3 $OUT/pytest_dist.log
NGZ_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --records 20000000 > $OUT/bench_dist2_gloo.json 2> $OUT/bench_dist2.err || { tail -30 $OUT/bench_dist2.err; exit 2; }
cat $OUT/bench_dist2_gloo.json

#!/bin/bash
# Insert-kernel grid sweep (NGZ_AGG_GRID) over the three aggregation keys.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-agggrid}
mkdir -p $OUT
for G in 1024 2048 4096 16384 65536; do
  for K in proto_dir dport 5tuple; do
    NGZ_AGG_GRID=$G timeout -k 10 300 python bench.py --agg $K --steps 5 --warmup 1 > $OUT/g${G}_$K.json 2> $OUT/g${G}_$K.err || exit 1
    echo "grid $G $K $(grep -o '"push_kernels_ms": [0-9.]*' $OUT/g${G}_$K.json)"
  done
done | tee $OUT/grid.txt

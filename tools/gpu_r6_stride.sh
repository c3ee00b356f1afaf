#!/bin/bash
# Round 6: column stride of mid-size launches (tools/stride_size.py, experiment build: drop ./tools/exp
# from .gpurunignore for this call).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6stride
mkdir -p $OUT
NGZ_EXPERIMENTS=1 timeout -k 10 400 python tools/stride_size.py 4 6 > $OUT/stride.json 2> $OUT/stride.err || { echo FAIL; tail -20 $OUT/stride.err; exit 1; }
cat $OUT/stride.json

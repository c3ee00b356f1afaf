#!/bin/bash
# Round 6: the LDS walk probe (tools/walk_probe.py, experiment build) under a
# kernel trace, so k_frame / the V900 decode of the same batch sit beside the probe launches.
# Needs tools/exp/libngz_exp.so on the box (drop ./tools/exp from .gpurunignore for this call).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6walk
mkdir -p $OUT
NGZ_EXPERIMENTS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/walk_probe.py 20000000 5 > $OUT/probe.json 2> $OUT/probe.err || { echo FAIL; tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.json
grep -E "walk_probe|k_frame|ngz_tpl" $OUT/trace/run_kernel_stats.csv

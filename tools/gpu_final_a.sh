#!/bin/bash
# Round-end evidence, part A: every -m gpu test, smoke(), aggregation bench lines + 5-tuple kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests_all.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 2; }
tail -1 gpurun_out/smoke.log
TAG=${TAG:-r2f}/agg bash tools/gpu_agg_bench.sh || exit 3

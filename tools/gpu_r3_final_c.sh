#!/bin/bash
# r3 evidence after an aggregation-only change: every -m gpu test, smoke(), aggregation profiles.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3b}
mkdir -p gpurun_out/$TAG
bash tools/gpu_tests_all.sh || exit 1
cp gpurun_out/pytest_gpu.log gpurun_out/$TAG/
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 2; }
tail -1 gpurun_out/$TAG/smoke.log
TAG=$TAG AGGS="${AGGS:-proto_dir dport 5tuple}" bash tools/gpu_profile_agg.sh || exit 4

#!/bin/bash
# r4: nontemporal column stores by default -- decode parity, smoke, default bench, decode profiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r4nt}
mkdir -p gpurun_out/$TAG
PYTEST_K="not agg" bash tools/gpu_tests_all.sh || exit 1
cp gpurun_out/pytest_gpu.log gpurun_out/$TAG/
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 2; }
tail -1 gpurun_out/$TAG/smoke.log
TAG=$TAG WORKLOADS="t20 cfg4 mixed8 cfg5" RECORDS_cfg4=20000000 bash tools/gpu_profile.sh || exit 4

#!/bin/bash
# r3 round-end evidence, part A: every -m gpu test, smoke(), then the T20 and config-4 profiles
# (bench line, kernel stats, FETCH_SIZE / WRITE_SIZE passes, summary + traffic.json).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3}
mkdir -p gpurun_out/$TAG
bash tools/gpu_tests_all.sh || exit 1
cp gpurun_out/pytest_gpu.log gpurun_out/$TAG/
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 2; }
tail -1 gpurun_out/$TAG/smoke.log
TAG=$TAG WORKLOADS="${WORKLOADS:-t20 cfg4}" RECORDS_cfg4=20000000 bash tools/gpu_profile.sh || exit 3

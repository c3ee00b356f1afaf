#!/bin/bash
# r4 round-end evidence: every -m gpu test, smoke(), the bench default line, profiles (bench line,
# kernel stats, FETCH / WRITE passes, summary + traffic.json) of T20, configs 3 / 4 / 5 and the
# three aggregation keys, and the host-to-host bench.   usage: TAG=r4 [PART=a|b] bash tools/gpu_r4_final.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r4}
mkdir -p gpurun_out/$TAG
if [ "${PART:-a}" = a ]; then
  bash tools/gpu_tests_all.sh || exit 1
  cp gpurun_out/pytest_gpu.log gpurun_out/$TAG/
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 2; }
  tail -1 gpurun_out/$TAG/smoke.log
  timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err || { tail -20 gpurun_out/$TAG/bench_default.err; exit 3; }
  cat gpurun_out/$TAG/bench_default.json
  TAG=$TAG WORKLOADS="t20 cfg4" RECORDS_cfg4=20000000 bash tools/gpu_profile.sh || exit 4
else
  TAG=$TAG WORKLOADS="mixed8 cfg5" bash tools/gpu_profile.sh || exit 5
  TAG=$TAG AGGS="proto_dir dport 5tuple" bash tools/gpu_profile_agg.sh || exit 6
  NGZ_EXPERIMENTS=1 NGZ_AGG_RED_RPT=1 timeout -k 10 300 python bench.py --agg dport --steps 10 --warmup 2 > gpurun_out/$TAG/agg_dport_rpt1.json 2> gpurun_out/$TAG/agg_dport_rpt1.err || exit 8
  python3 -c "import json; d=json.load(open('gpurun_out/$TAG/agg_dport_rpt1.json')); print('dport reduce 1 payload/thread: push %.3f ms' % d['push_kernels_ms'])"
  timeout -k 10 300 python3 bench.py --e2e --records 10000000 --steps 5 --warmup 2 > gpurun_out/$TAG/e2e_1e7.json 2> gpurun_out/$TAG/e2e.err || { tail -5 gpurun_out/$TAG/e2e.err; exit 7; }
  cat gpurun_out/$TAG/e2e_1e7.json
fi

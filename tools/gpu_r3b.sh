#!/bin/bash
# r3: decode parity with multi-template launches, then config 3 / 5 with and without them
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3b
( while sleep 20; do date >> gpurun_out/r3b/ticks.txt; done ) &
TK=$!
timeout -k 10 700 python -u -m pytest ${R3B_TESTS:-tests/test_gpu_parity.py tests/test_gpu_packet_kats.py tests/test_gpu_rtc.py} ${R3B_K:+-k "$R3B_K"} -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/r3b/pytest.log 2>&1
rc=$?
kill $TK
tail -15 gpurun_out/r3b/pytest.log
[ $rc -eq 0 ] || exit $rc
for W in ${WLS:-mixed8 cfg5}; do
for G in ${GROUPS_AB:-1 0}; do
  NGZ_GROUP=$G timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3b/${W}_g$G.json 2> gpurun_out/r3b/${W}_g$G.err || { tail -5 gpurun_out/r3b/${W}_g$G.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/r3b/${W}_g$G.json')); print('$W group=$G', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['ms_per_step'],4))"
done; done

#!/bin/bash
# r3: aggregation / rtc / dist GPU tests, then the T20 kernel time against batch size
# (is a 1.25e7-record launch slower per byte than a 1e8 one?)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest ${R3A_TESTS:-tests/test_gpu_agg.py tests/test_gpu_rtc.py} tests/test_gpu_dist.py "tests/test_gpu_parity.py::test_cfg4_vlen_columns_full_size" "tests/test_gpu_parity.py::test_cfg3_mixed_templates_1e8" "tests/test_gpu_parity.py::test_cfg5_shard_full_size" -q -x \
  --timeout 200 --timeout-method thread > gpurun_out/r3a/pytest.log 2>&1
rc=$?
tail -25 gpurun_out/r3a/pytest.log
[ $rc -eq 0 ] || exit $rc
for N in 12500000 25000000 50000000 100000000; do
  timeout -k 10 300 python bench.py --records $N --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3a/t20_$N.json 2> gpurun_out/r3a/t20_$N.err || exit 3
  python -c "import json,sys; d=json.load(open('gpurun_out/r3a/t20_$N.json')); print($N, d['roofline']['kernel_ms'], d['roofline']['frac'], d['ms_per_step'])"
done

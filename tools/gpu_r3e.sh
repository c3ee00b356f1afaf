#!/bin/bash
# r3: vlen record lists + low-card aggregation: tests, then cfg4 A/B and bench --agg proto_dir
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3e
( while sleep 20; do date >> gpurun_out/r3e/ticks.txt; done ) &
TK=$!
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jsonl.py tests/test_gpu_agg.py tests/test_gpu_packet_kats.py \
  -k "${R3E_K:-vlen or cfg4 or variable or srv6 or golden or lowcard or kat}" -q -x --timeout 300 --timeout-method thread > gpurun_out/r3e/pytest.log 2>&1
rc=$?
kill $TK
tail -8 gpurun_out/r3e/pytest.log
[ $rc -eq 0 ] || exit $rc
for M in 2 1; do
  NGZ_RECMAP=$M timeout -k 10 300 python bench.py --workload cfg4 --records 20000000 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3e/cfg4_m$M.json 2> gpurun_out/r3e/cfg4_m$M.err || { tail -5 gpurun_out/r3e/cfg4_m$M.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/r3e/cfg4_m$M.json')); print('cfg4 recmap=$M', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), 'step', round(d['ms_per_step'],4))"
done
timeout -k 10 300 python bench.py --agg proto_dir --steps 10 --warmup 2 > gpurun_out/r3e/agg_proto_dir.json 2> gpurun_out/r3e/agg.err || { tail -5 gpurun_out/r3e/agg.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/r3e/agg_proto_dir.json')); print('proto_dir', d['path'], round(d['push_kernels_ms'],3), 'first', round(d['config']['first_push_ms'],3))"

#!/bin/bash
# r4: LDS-staged k_frame (decode parity, config-4 step and dispatches), then the aggregation parity
# and profiles.  usage: TAG=r4c2 bash tools/gpu_r4_combo.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4c2}
mkdir -p $OUT
( while sleep 20; do date >> $OUT/ticks.txt; done ) &
TK=$!
trap "kill $TK" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_packet_kats.py tests/test_gpu_agg.py tests/test_gpu_jsonl.py \
  -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_cfg4 -o run -- \
  python3 bench.py --workload cfg4 --records 20000000 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err || { tail -5 $OUT/cfg4.err; exit 3; }
python3 -c "import json; d=json.load(open('$OUT/cfg4.json')); print('cfg4 step %.4f ms decode %.4f ms' % (d['ms_per_step'], d['roofline']['kernel_ms']))"
python3 tools/dispatches.py $OUT/trace_cfg4 | tail -11
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/t20.json 2> $OUT/t20.err || { tail -5 $OUT/t20.err; exit 4; }
python3 -c "import json; d=json.load(open('$OUT/t20.json')); print('t20 step %.4f ms decode %.4f ms' % (d['ms_per_step'], d['roofline']['kernel_ms']))"
TAG=${TAG:-r4c2} AGGS="dport proto_dir 5tuple" bash tools/gpu_profile_agg.sh || exit 5

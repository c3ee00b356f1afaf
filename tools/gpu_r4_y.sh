#!/bin/bash
# r4: windowed record walk in k_frame (vlen parity + config-4 step, dispatches); reduce without
# redundant LDS atomics (partitioned parity + dport push); scatter without operand loads (timing)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r4y
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_agg.py tests/test_gpu_packet_kats.py -v -m gpu --timeout 300 --timeout-method thread \
  -k "cfg4 or variable or vlen or partitioned or capture or kat" > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_cfg4 -o run -- \
  python3 bench.py --workload cfg4 --records 20000000 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err \
  || { tail -5 $OUT/cfg4.err; exit 3; }
python3 -c "import json; d=json.load(open('$OUT/cfg4.json')); print('cfg4 step %.4f ms decode %.4f ms' % (d['ms_per_step'], d['roofline']['kernel_ms']))"
python3 tools/dispatches.py $OUT/trace_cfg4 | tail -12
for S in 0 2; do
  NGZ_AGG_SCATTER_DBG=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/agg_s$S -o run -- \
    python3 bench.py --agg dport --steps 5 --warmup 1 > $OUT/agg_s$S.json 2> $OUT/agg_s$S.err || { tail -5 $OUT/agg_s$S.err; exit 4; }
  python3 -c "import json; d=json.load(open('$OUT/agg_s$S.json')); print('scatter_dbg=$S push %.3f ms' % d['push_kernels_ms'])"
  python3 - $OUT/agg_s$S <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:4]:
    print("   %-60s %6s %12.0f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])))
PY
done

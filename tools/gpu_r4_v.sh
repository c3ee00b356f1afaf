#!/bin/bash
# r4: partition reduce through LDS (parity + time), scatter with record-order stores (timing only),
# then the config-4 dispatch / window traces (tools/gpu_r4_u.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r4v
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -v -m gpu --timeout 300 --timeout-method thread \
  -k "partitioned" > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for S in 0 1; do
  NGZ_AGG_SCATTER_DBG=$S timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/agg_s$S -o run -- \
    python3 bench.py --agg dport --steps 5 --warmup 1 > $OUT/agg_s$S.json 2> $OUT/agg_s$S.err || { tail -5 $OUT/agg_s$S.err; exit 3; }
  python3 -c "import json; d=json.load(open('$OUT/agg_s$S.json')); print('scatter_dbg=$S push %.3f ms' % d['push_kernels_ms'])"
  python3 - $OUT/agg_s$S <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:5]:
    print("   %-60s %6s %12.0f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])))
PY
done
TAG=r4u bash tools/gpu_r4_u.sh

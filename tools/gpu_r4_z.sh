#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4z}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -v -m gpu --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for K in dport proto_dir 5tuple; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/agg_$K -o run -- \
    python3 bench.py --agg $K --steps 5 --warmup 1 > $OUT/agg_$K.json 2> $OUT/agg_$K.err || { tail -5 $OUT/agg_$K.err; exit 4; }
  python3 -c "import json; d=json.load(open('$OUT/agg_$K.json')); print('$K push %.3f ms path %s' % (d['push_kernels_ms'], d['path']))"
  python3 - $OUT/agg_$K <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:5]:
    print("   %-60s %6s %12.0f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])))
PY
done

#!/bin/bash
# r4: compact partition payloads -- partitioned-reduction parity, the dport push (kernel stats),
# per-kernel FETCH / WRITE of the push.  usage: TAG=r4s bash tools/gpu_r4_s.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4s}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_agg.py -v -m gpu --timeout 300 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/agg_dport -o run -- \
  python3 bench.py --agg dport --steps 5 --warmup 1 > $OUT/agg_dport.json 2> $OUT/agg_dport.err || { tail -5 $OUT/agg_dport.err; exit 3; }
python3 -c "import json; d=json.load(open('$OUT/agg_dport.json')); print('agg dport push %.3f ms first %.3f ms path %s' % (d['push_kernels_ms'], d['config']['first_push_ms'], d['path']))"
python3 - $OUT/agg_dport <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print("%-60s %6s %12.0f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])))
PY
KREGEX="k_agg" ARGS="--agg dport --steps 1 --warmup 0" PASSES="FETCH_SIZE;WRITE_SIZE" TAG=${TAG:-r4s}/pmc bash tools/gpu_pmc_kernel.sh

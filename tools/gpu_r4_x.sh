#!/bin/bash
# r4: two-level partitioning parity + push A/B; k_frame counters, split and not
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r4x
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -v -m gpu --timeout 300 --timeout-method thread \
  -k "partitioned" > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for T in 0 1; do
  NGZ_AGG_PART2=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/agg$T -o run -- \
    python3 bench.py --agg dport --steps 5 --warmup 1 > $OUT/agg$T.json 2> $OUT/agg$T.err || { tail -5 $OUT/agg$T.err; exit 3; }
  python3 -c "import json; d=json.load(open('$OUT/agg$T.json')); print('PART2=$T push %.3f ms' % d['push_kernels_ms'])"
  python3 - $OUT/agg$T <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:7]:
    print("   %-60s %6s %12.0f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"])))
PY
done
for S in 0 1; do
  echo "== k_frame counters, NGZ_SPLIT=$S"
  NGZ_SPLIT=$S KREGEX="k_frame" ARGS="--workload cfg4 --records 20000000 --steps 1 --warmup 0" \
    PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
    TAG=r4x/frame$S bash tools/gpu_pmc_kernel.sh || exit 4
done

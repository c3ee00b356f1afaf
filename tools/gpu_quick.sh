#!/bin/bash
# Quick iteration on one GPU box: a subset of the GPU tests (PYTEST_K), then
# one bench line (BENCH_ARGS) and its kernel-trace stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "$PYTEST_K" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -2 $OUT/pytest.log
fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
  cat $OUT/bench.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $BENCH_ARGS --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 3; }
  python3 - $OUT <<'PY'
import csv, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(d + "/trace/run_kernel_trace.csv")))
last = rows[-16:]
for r in last:
    print("%-40s %10.1f us grid %s wg %s lds %s vgpr %s" % (r["Kernel_Name"].replace("(anonymous namespace)::", "")[:40],
          (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Grid_Size_X"], r["Workgroup_Size_X"],
          r["LDS_Block_Size"], r["VGPR_Count"]))
PY
fi

#!/bin/bash
# Aggregation push throughput per key (bench.py --agg), one line each, plus a kernel trace of the 5-tuple.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-agg_bench}
mkdir -p $OUT
N=${RECORDS:-100000000}
for K in proto_dir dport 5tuple; do
  timeout -k 10 400 python bench.py --agg $K --records $N --steps ${STEPS:-5} --warmup 2 > $OUT/bench_$K.json 2> $OUT/bench_$K.err || { tail -20 $OUT/bench_$K.err; exit 1; }
  cat $OUT/bench_$K.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --agg 5tuple --records $N --steps 3 --warmup 1 > $OUT/trace_bench.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 2; }
python3 - $OUT <<'PY'
import csv, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(d + "/trace/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-60s %6s %12.1f us" % (r["Name"].replace("(anonymous namespace)::", "")[:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY

#!/bin/bash
# rocprofv3 kernel trace of one bench workload: WORKLOAD, REC, TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tr}
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${WORKLOAD:-t20} -o run -- python3 bench.py --no-cpu-baseline --workload ${WORKLOAD:-t20} --records ${REC:-100000000} --steps 5 --warmup 1 > $OUT/${WORKLOAD:-t20}.json 2> $OUT/${WORKLOAD:-t20}.err || exit 1
python3 - $OUT/trace_${WORKLOAD:-t20} <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/*kernel_stats.csv"):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print("%-60s %6s %12.0f %14.0f" % (r["Name"].replace("(anonymous namespace)::", "")[:60], r["Calls"], float(r["AverageNs"]), float(r["TotalDurationNs"])))
PY

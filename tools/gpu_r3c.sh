#!/bin/bash
# r3: config 3 multi-template launch A/B: workgroups per CU, and per-kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r3c
for G in 1 0; do for B in 2 8; do
  NGZ_GROUP=$G NGZ_LDS_BLOCKS_PER_CU=$B timeout -k 10 300 python bench.py --workload mixed8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3c/g${G}_b$B.json 2> gpurun_out/r3c/g${G}_b$B.err || exit 3
  python -c "import json; d=json.load(open('gpurun_out/r3c/g${G}_b$B.json')); print('group=$G bpc=$B', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['ms_per_step'],4))"
done; done
NGZ_GROUP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c/trace -o run -- python3 bench.py --workload mixed8 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r3c/trace.json 2> gpurun_out/r3c/trace.err || exit 4
python3 - <<'PY'
import csv, glob
rows = []
for f in glob.glob("gpurun_out/r3c/trace/*kernel_stats.csv"):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%-40s %6s %12.0f" % (r["Name"][:40], r["Calls"], float(r["AverageNs"])))
PY

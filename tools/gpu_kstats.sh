#!/bin/bash
# Per-kernel times (rocprofv3 kernel trace + stats) of bench.py command lines.
# usage: RUNS="name1=--agg proto_dir;name2=--workload mixed8" [ENV_name1="NGZ_GROUP=1"] bash tools/gpu_kstats.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-kstats}
mkdir -p $OUT
IFS=';' read -ra R <<< "$RUNS"
for run in "${R[@]}"; do
  N=${run%%=*}; A=${run#*=}
  EV=ENV_$N
  ( [ -n "${!EV}" ] && export ${!EV}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$N -o run -- python3 bench.py $A --no-cpu-baseline > $OUT/$N.json 2> $OUT/$N.err ) || { tail -5 $OUT/$N.err; exit 3; }
  echo "== $N: $A ${!EV}"
  python3 - $OUT/$N <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-48s %6s %12.0f %12.0f" % (r["Name"][:48], r["Calls"], float(r["AverageNs"]), float(r["TotalDurationNs"])))
PY
done

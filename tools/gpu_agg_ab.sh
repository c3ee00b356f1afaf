#!/bin/bash
# A/B of aggregation push variants: per-kernel durations of the steady-state pushes of
# bench.py --agg (kernel trace), one run per env setting in CONFIGS (";"-separated).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export NGZ_EXPERIMENTS=1  # env knobs are read only by the experiment build (tools/build_experiments.sh)
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-agg_ab}
mkdir -p $OUT
K=${AGG_KEY:-5tuple}
N=${RECORDS:-100000000}
IFS=';' read -ra CS <<< "${CONFIGS:-X=1}"
i=0
for c in "${CS[@]}"; do
  i=$((i+1))
  env $c timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$i -o run -- python3 bench.py --agg $K --records $N --steps 3 --warmup 1 > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 - $OUT/t$i "$c" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
per = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if "agg" in k:
        per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
tot = 0
out = []
for k, v in per.items():
    last = v[-3:]
    m = sum(last) / len(last)
    tot += m
    out.append("%s %.2f" % (k.replace("void ", "")[:22], m))
print("[%s] push kernels %.2f ms: %s" % (sys.argv[2], tot, ", ".join(out)))
PY
done

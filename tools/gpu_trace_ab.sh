#!/bin/bash
# A/B of env settings (CONFIGS, ";"-separated) on one bench command (BENCH_ARGS): per-kernel
# mean durations over the timed steps from a rocprofv3 kernel trace, plus the bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-trace_ab}
mkdir -p $OUT
ARGS=${BENCH_ARGS:---workload cfg4 --steps 5 --warmup 2 --no-cpu-baseline}
IFS=';' read -ra CS <<< "${CONFIGS:-X=1}"
i=0
for c in "${CS[@]}"; do
  i=$((i+1))
  env $c timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$i -o run -- python3 bench.py $ARGS > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 - $OUT/t$i "$c" $OUT/b$i.json <<'PY'
import csv, sys, collections, json
rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
per = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
b = json.load(open(sys.argv[3]))
out = ["%s %d x %.1f us" % (k[:40], len(v), sum(v[-5:]) / len(v[-5:])) for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:8]]
print("[%s] ms_per_step %.3f value %.3g | %s" % (sys.argv[2], b["ms_per_step"], b["value"], "; ".join(out)))
PY
done

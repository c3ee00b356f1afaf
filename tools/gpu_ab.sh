#!/bin/bash
# A/B of experiment-knob settings (CONFIGS, ";"-separated NGZ_<knob>=value lists) on one bench
# command (BENCH_ARGS), run on the experiment build (libngz_exp.so, NGZ_EXPERIMENTS=1): per kernel
# (name, workgroup, LDS, VGPRs) the mean duration over the last dispatches, and the bench line.
# usage: TAG=r5/ab CONFIGS="X=1;NGZ_LDS_BUDGET=40960" BENCH_ARGS="--workload cfg4" bash tools/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
ARGS="${BENCH_ARGS:---workload cfg4} --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline"
IFS=';' read -ra CS <<< "${CONFIGS:-X=1}"
i=0
for c in "${CS[@]}"; do
  i=$((i+1))
  env NGZ_EXPERIMENTS=1 $c timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$i -o run -- python3 bench.py $ARGS > $OUT/b$i.json 2> $OUT/b$i.err || { tail -5 $OUT/b$i.err; exit 1; }
  python3 - $OUT/t$i "$c" $OUT/b$i.json ${STEPS:-5} <<'PY'
import csv, sys, collections, json
rows = list(csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")))
steps = int(sys.argv[4])
per = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    key = "%s[wg%s lds%s v%s g%s]" % (k[:24], r["Workgroup_Size_X"], r["LDS_Block_Size"], r["VGPR_Count"], r["Grid_Size_X"])
    per[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
b = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
out = ["%s %dx %.1fus" % (k, len(v), sum(v[-steps:]) / len(v[-steps:])) for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1][-steps:]))[:7]]
print("[%s] ms_per_step %.3f kernel_ms %.3f | %s" % (sys.argv[2], b["ms_per_step"], b["roofline"]["kernel_ms"], "; ".join(out)), flush=True)
PY
done

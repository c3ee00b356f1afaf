#!/bin/bash
# r4: the partitioned scatter (bench --agg dport + per-kernel times), the LDS-staged decode grid
# on config 3 and small T20 batches, and the arena placement experiment.  usage: TAG=r4e bash tools/gpu_r4_e.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4e}
mkdir -p $OUT
timeout -k 10 120 tools/pcie_kernel_probe 640 5 > $OUT/pcie_kernel.json 2> $OUT/pcie_kernel.err || { tail -5 $OUT/pcie_kernel.err; exit 5; }
cat $OUT/pcie_kernel.json
for PK in "3 12" "4 24" "6 24" "8 48"; do set -- $PK
  timeout -k 10 300 python3 bench.py --e2e --records 10000000 --steps 5 --warmup 2 --e2e-contexts $1 --e2e-ranges $2 \
    > $OUT/e2e_p$1_k$2.json 2> $OUT/e2e_p$1_k$2.err || { tail -5 $OUT/e2e_p$1_k$2.err; exit 6; }
  python3 -c "import json; d=json.load(open('$OUT/e2e_p$1_k$2.json')); print('e2e P=$1 K=$2 duplex %.2f threads %.2f ms' % (d['ms_per_step'], d['threads']['ms_per_step']))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/agg_dport -o run -- \
  python3 bench.py --agg dport --steps 5 --warmup 1 > $OUT/agg_dport.json 2> $OUT/agg_dport.err || { tail -5 $OUT/agg_dport.err; exit 2; }
python3 -c "import json; d=json.load(open('$OUT/agg_dport.json')); print('agg dport push %.3f ms first %.3f ms path %s' % (d['push_kernels_ms'], d['config']['first_push_ms'], d['path']))"
python3 - $OUT/agg_dport <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("%-48s %6s %12.0f" % (r["Name"][:48], r["Calls"], float(r["AverageNs"])))
PY
CASES="t20s=--workload t20 --records 12500000;mixed8=--workload mixed8" SETTINGS="b2=NGZ_LDS_BLOCKS_PER_CU=2;b8=NGZ_LDS_BLOCKS_PER_CU=8" \
  STEPS=10 TAG=${TAG:-r4e}/sweep bash tools/gpu_sweep.sh || exit 3
RUNS=3 TAG=${TAG:-r4e}/arena bash tools/gpu_arena.sh || exit 4

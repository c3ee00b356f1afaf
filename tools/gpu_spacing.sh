#!/bin/bash
# column-spacing probe sweeps.  usage: TAG=r4q bash tools/gpu_spacing.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export NGZ_EXPERIMENTS=1  # env knobs are read only by the experiment build (tools/build_experiments.sh)
OUT=gpurun_out/${TAG:-spacing}
mkdir -p $OUT
P=tools/spacing_probe
timeout -k 10 120 $P 12500000 0 150000 5000 5 > $OUT/n4_coarse.txt || exit 2
timeout -k 10 120 $P 12500000 36990 37010 1 5 > $OUT/n4_fine.txt || exit 3
timeout -k 10 120 $P 12500000 0 20 1 5 > $OUT/n4_fine0.txt || exit 4
timeout -k 10 200 $P 100000000 0 100000 10000 3 > $OUT/t20_coarse.txt || exit 5
timeout -k 10 120 $P 12500000 0 150000 5000 5 > $OUT/n4_coarse_again.txt || exit 6
python3 - $OUT <<'PY'
import json, sys
for f in ["n4_coarse", "n4_fine", "n4_fine0", "t20_coarse", "n4_coarse_again"]:
    rows = [json.loads(l) for l in open(sys.argv[1] + "/" + f + ".txt")]
    print(f, " ".join("%d:%.2f" % (r["pad"], r["tbs"]) for r in rows))
PY

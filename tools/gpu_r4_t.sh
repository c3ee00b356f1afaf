#!/bin/bash
# r4: HBM placement map, then the compact-payload aggregation measurements (tools/gpu_r4_s.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4r
timeout -k 10 200 tools/hbm_map_probe 256 512 > gpurun_out/r4r/map.txt || exit 2
python3 - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/r4r/map.txt")]
print(" ".join("%d:%.2f/%.2f/%.2f" % (r["chunk"], r["read_tbs"], r["write_tbs"], r["window_tbs"]) for r in rows))
PY
TAG=r4s bash tools/gpu_r4_s.sh

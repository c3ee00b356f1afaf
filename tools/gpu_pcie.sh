#!/bin/bash
# PCIe: the probe with SDMA copies and with blit-kernel copies (HSA_ENABLE_SDMA=0), and the
# host-to-host bench under each.  usage: TAG=r4d bash tools/gpu_pcie.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pcie}
mkdir -p $OUT
for S in 1 0; do
  HSA_ENABLE_SDMA=$S timeout -k 10 120 python3 tools/pcie_probe.py > $OUT/probe_sdma$S.json 2> $OUT/probe_sdma$S.err \
    || { tail -5 $OUT/probe_sdma$S.err; exit 3; }
  cat $OUT/probe_sdma$S.json
  HSA_ENABLE_SDMA=$S timeout -k 10 300 python3 bench.py --e2e --records 10000000 --steps 5 --warmup 2 > $OUT/e2e_sdma$S.json 2> $OUT/e2e_sdma$S.err \
    || { tail -5 $OUT/e2e_sdma$S.err; exit 4; }
  python3 -c "import json; d=json.load(open('$OUT/e2e_sdma$S.json')); print('sdma=$S duplex %.2f ms threads %.2f ms serial %.2f ms' % (d['ms_per_step'], d['threads']['ms_per_step'], d['serial']['ms_per_step']))"
done

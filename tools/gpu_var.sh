#!/bin/bash
# Run-to-run variance on one box: HBM probe and bench alternately.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-var}
mkdir -p $OUT
hipcc -O3 --offload-arch=gfx950 tools/hbm_probe.hip -o /tmp/hbm_probe 2>/dev/null || exit 4
for rep in 1 2 3 4 5; do
  timeout -k 5 200 /tmp/hbm_probe > $OUT/hbm_$rep.txt || exit 4
  grep "grid  1024 | copy16 " $OUT/hbm_$rep.txt | cut -c1-60
  timeout -k 10 300 python bench.py --records ${REC:-100000000} --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_$rep.json 2> $OUT/b_$rep.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench kernel_ms %.4f' % d['roofline']['kernel_ms'], 'ms_per_step %.4f' % d['ms_per_step'])" $OUT/b_$rep.json
done

#!/bin/bash
# A/B an env knob on one box with the HBM probe as box calibration:
# VAR=NAME VALS="a b" [REC=...] [WORKLOAD=t20]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab2}
mkdir -p $OUT
hipcc -O3 --offload-arch=gfx950 tools/hbm_probe.hip -o /tmp/hbm_probe 2>/dev/null && timeout -k 5 200 /tmp/hbm_probe > $OUT/hbm_probe.txt || exit 4
grep "grid  1024" $OUT/hbm_probe.txt
for rep in 1 2; do
for v in ${VALS}; do
  env $VAR=$v timeout -k 10 300 python bench.py --workload ${WORKLOAD:-t20} --records ${REC:-100000000} --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel_ms %.4f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'ms_per_step %.4f' % d['ms_per_step'], 'overhead_us %.1f' % (1e3*(d['ms_per_step']-d['roofline']['kernel_ms'])))" $OUT/b_${v}_$rep.json "$VAR=$v"
done
done

#!/bin/bash
# A/B the run-time kernel generator's knobs on the bench workload (VARS="NAME=v1,v2 ...").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-var}
mkdir -p $OUT
# same-box ceiling reference (copy / naive column shape)
hipcc -O3 --offload-arch=gfx950 tools/hbm_probe.hip -o /tmp/hbm_probe 2>/dev/null && timeout -k 5 200 /tmp/hbm_probe > $OUT/hbm_probe.txt && grep "grid  1024" $OUT/hbm_probe.txt | cut -c1-200
for spec in ${VARS:-NGZ_RTC_RPL=1,2,4}; do
  name=${spec%%=*}; vals=${spec#*=}
  for v in ${vals//,/ }; do
    env $name=$v timeout -k 10 300 python bench.py --records ${REC:-100000000} --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b_${name}_$v.json 2> $OUT/b_${name}_$v.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'ms_per_step %.3f' % d['ms_per_step'])" $OUT/b_${name}_$v.json "$name=$v"
  done
done

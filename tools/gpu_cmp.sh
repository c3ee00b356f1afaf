#!/bin/bash
# Same-box comparison: the HBM probe (copy ceiling, realigned LDS-staged T20
# shape) followed by bench runs under each env setting in CONFIGS
# (";"-separated, e.g. CONFIGS="NGZ_LDS=0;NGZ_LDS=1").
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-cmp}
mkdir -p $OUT
hipcc -O3 --offload-arch=gfx950 tools/hbm_probe2.hip -o /tmp/p2 2>/dev/null || exit 1
timeout -k 5 120 /tmp/p2 > $OUT/probe2.txt || exit 2
grep -E "grid|copy16|al5 mis4|lds1024 buf mis4|read" $OUT/probe2.txt
IFS=';' read -ra CS <<< "${CONFIGS:-NGZ_LDS=1}"
i=0
for w in ${WORKLOADS:-t20}; do
  for c in "${CS[@]}"; do
    i=$((i+1))
    env $c timeout -k 10 300 python bench.py --workload $w --records ${REC:-100000000} --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b_$i.json 2> $OUT/b_$i.err || { tail -5 $OUT/b_$i.err; exit 3; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'frac %.3f' % d['roofline']['frac'], 'ms_per_step %.3f' % d['ms_per_step'])" $OUT/b_$i.json "$w [$c]"
  done
done

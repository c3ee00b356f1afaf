#!/bin/bash
# Decode time of config 3 / T20 at 1.25e7 against workgroups per CU and decode streams
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/grid
for W in ${WLS:-mixed8}; do
for S in ${STREAMS:-1 4}; do
for B in ${BPC:-0 8 48}; do
  if [ "$B" = 0 ]; then unset NGZ_LDS_BLOCKS_PER_CU; else export NGZ_LDS_BLOCKS_PER_CU=$B; fi
  export NGZ_DECODE_STREAMS=$S
  timeout -k 10 300 python bench.py --workload $W ${RECS:+--records $RECS} --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/grid/${W}_s${S}_b${B}.json 2> gpurun_out/grid/${W}_s${S}_b${B}.err || exit 3
  python -c "import json; d=json.load(open('gpurun_out/grid/${W}_s${S}_b${B}.json')); print('$W streams=$S bpc=$B', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['ms_per_step'],4))"
done; done; done

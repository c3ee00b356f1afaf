#!/bin/bash
# r3: count-matrix rows per active slot: every -m gpu test, then config 4 / T20 bench lines and the
# config 4 per-kernel HBM bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3c}
mkdir -p gpurun_out/$TAG
bash tools/gpu_tests_all.sh || exit 1
cp gpurun_out/pytest_gpu.log gpurun_out/$TAG/
for W in cfg4 t20; do
  A="--workload $W --steps 20 --warmup 5 --no-cpu-baseline"
  [ $W = cfg4 ] && A="$A --records 20000000"
  timeout -k 10 300 python bench.py $A > gpurun_out/$TAG/$W.json 2> gpurun_out/$TAG/$W.err || { tail -5 gpurun_out/$TAG/$W.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/$TAG/$W.json')); print('$W', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), 'step', round(d['ms_per_step'],4), '%.3g' % d['value'])"
done
TAG=$TAG/cfg4_pmc bash tools/gpu_pmc_cfg4.sh || exit 4

#!/bin/bash
# aggregation A/B: key x env settings (CONFIGS="NAME=ENV;...")
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/aggab
IFS=';' read -ra CS <<< "${CONFIGS:-base=}"
for K in ${AGGS:-proto_dir dport}; do
for C in "${CS[@]}"; do
  NAME=${C%%=*}; ENVS=${C#*=}
  env $ENVS timeout -k 10 300 python bench.py --agg $K --steps 10 --warmup 2 ${BARGS} > gpurun_out/aggab/${K}_$NAME.json 2> gpurun_out/aggab/${K}_$NAME.err || { tail -5 gpurun_out/aggab/${K}_$NAME.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/aggab/${K}_$NAME.json')); print('$K $NAME', d['path'], round(d['push_kernels_ms'],3), 'first', round(d['config']['first_push_ms'],3))"
done; done

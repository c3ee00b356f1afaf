#!/bin/bash
# One aggregation key's evidence: bench line, rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE passes,
# and tools/summarize_agg_profile.py's summary + traffic.json.
# usage: TAG=r3x AGGS="proto_dir dport 5tuple" bash tools/gpu_profile_agg.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-prof}
for K in ${AGGS:-proto_dir}; do
  OUT=gpurun_out/$TAG/agg_$K
  mkdir -p $OUT
  ARGS="--agg $K --steps 10 --warmup 2"
  timeout -k 10 300 python bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
  cat $OUT/bench.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 3; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- python3 bench.py --agg $K --steps 2 --warmup 0 > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err || { tail -20 $OUT/pmc_$C.err; exit 4; }
  done
  python3 tools/summarize_agg_profile.py $OUT > $OUT/summary.txt
  cat $OUT/summary.txt | tail -25
done

#!/bin/bash
# One workload's evidence on one GPU box: the bench line, rocprofv3
# --kernel-trace --stats of the same command, FETCH_SIZE / WRITE_SIZE in
# separate PMC passes, and tools/summarize_profile.py's summary + traffic.json.
# usage: TAG=r2b WORKLOADS="t20 cfg4" [RECORDS_cfg4=20000000] bash tools/gpu_profile.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-prof}
for W in ${WORKLOADS:-t20}; do
  OUT=gpurun_out/$TAG/$W
  mkdir -p $OUT
  RV=RECORDS_$W
  ARGS="--workload $W ${!RV:+--records ${!RV}} --steps 20 --warmup 5"
  echo "== $W: bench.py $ARGS"
  timeout -k 10 600 python bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
  cat $OUT/bench.json
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || { tail -20 $OUT/trace.err; exit 3; }
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- python3 bench.py $ARGS --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err || { tail -20 $OUT/pmc_$C.err; exit 4; }
  done
  python3 tools/summarize_profile.py $OUT > $OUT/summary.txt
  cat $OUT/summary.txt
done

#!/bin/bash
# Round evidence: full bench line (with cpu_baseline), rocprofv3 kernel stats
# of the same command, and separate PMC passes for HBM traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || exit 2
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err || exit 3
done
python3 tools/summarize_profile.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt

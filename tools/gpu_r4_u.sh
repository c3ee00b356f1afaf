#!/bin/bash
# r4: config 4 per-dispatch kernel times and per-slot window traces; NFv9-only and vlen-only halves
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4u}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_cfg4 -o run -- \
  python3 bench.py --workload cfg4 --records 20000000 --steps 5 --warmup 3 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err \
  || { tail -5 $OUT/cfg4.err; exit 2; }
python3 tools/dispatches.py $OUT/trace_cfg4 | tail -16
NGZ_TRACE=1 timeout -k 10 300 python3 bench.py --workload cfg4 --records 20000000 --steps 3 --warmup 2 --no-cpu-baseline \
  > $OUT/cfg4_trace.json 2> $OUT/cfg4_trace.err || { tail -5 $OUT/cfg4_trace.err; exit 3; }
grep "trace slot" $OUT/cfg4_trace.err | tail -4
NGZ_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_cfg4_split -o run -- \
  python3 bench.py --workload cfg4 --records 20000000 --steps 5 --warmup 3 --no-cpu-baseline > $OUT/cfg4_split.json 2> $OUT/cfg4_split.err \
  || { tail -5 $OUT/cfg4_split.err; exit 4; }
python3 tools/dispatches.py $OUT/trace_cfg4_split | tail -18

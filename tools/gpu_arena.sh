#!/bin/bash
# Arena placement root cause: fresh-process T20 bench lines without placement trials
# (NGZ_PLACE_TRIALS=1), the column arena from hipMalloc vs physically contiguous memory
# (NGZ_ARENA_CONTIG=1), and the counter list of this rocprofv3 (for translation counters).
# usage: TAG=r4c [RUNS=5] bash tools/gpu_arena.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export NGZ_EXPERIMENTS=1  # env knobs are read only by the experiment build (tools/build_experiments.sh)
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-arena}
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
grep -iE "UTCL|TLB|TRANSLATION" $OUT/counters_avail.txt | head -40
for MODE in malloc contig; do
  for i in $(seq 1 ${RUNS:-5}); do
    ( export NGZ_PLACE_TRIALS=1; [ $MODE == contig ] && export NGZ_ARENA_CONTIG=1
      timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/$MODE.$i.json 2> $OUT/$MODE.$i.err ) \
      || { echo "FAILED $MODE $i"; tail -5 $OUT/$MODE.$i.err; exit 3; }
    python3 -c "import json; d=json.load(open('$OUT/$MODE.$i.json')); print('$MODE run $i: kernel %.4f ms step %.4f ms' % (d['roofline']['kernel_ms'], d['ms_per_step']))"
  done
done

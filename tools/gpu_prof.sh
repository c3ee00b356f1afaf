#!/bin/bash
# kernel trace + stats, then PMC passes (each its own run), for the bench workload
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG:-r1}
mkdir -p $OUT
REC=${REC:-100000000}
timeout -k 10 400 python bench.py --records $REC --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
echo "bench rc=$?"; cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --records $REC --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1
echo "trace rc=$?"
find $OUT/trace -name "*kernel_stats.csv" -exec cat {} \;
for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  N=$(echo $C | tr ' ' '_')
  timeout -k 10 400 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$N -o run -- python3 bench.py --records $REC --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_$N.log 2>&1
  echo "pmc $C rc=$?"
done
exit 0

#!/bin/bash
# Config-4 evidence for one tree (round 5): the bench line, rocprofv3 kernel stats of the same
# command, and per-dispatch counter passes (each its own --pmc run, with --kernel-trace so every
# dispatch's duration sits beside its counters) over the decode, framing and emit kernels.
# usage: TAG=r5/cfg4 [RECORDS=20000000] bash tools/gpu_r5_cfg4.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5cfg4}
mkdir -p $OUT
ARGS="--workload cfg4 --records ${RECORDS:-20000000}"
timeout -k 10 300 python bench.py $ARGS --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 2; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS --steps 20 --warmup 5 --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 3; }
RX="ngz_tpl|k_frame|k_emit|k_decode_generic"
i=0
for pc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU" \
          "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pc --kernel-trace --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc$i.json 2> $OUT/pmc$i.err || { tail -5 $OUT/pmc$i.err; exit 4; }
done
python3 tools/pmc_dispatch.py "$RX" $OUT/pmc1 $OUT/pmc2 $OUT/pmc3 $OUT/pmc4 > $OUT/pmc_dispatch.txt
tail -30 $OUT/pmc_dispatch.txt

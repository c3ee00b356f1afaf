#!/bin/bash
# Round 6: configs 3 / 5 experiment -- tools/decode_size.py plain, then two rocprofv3 --pmc passes
# (TCC DRAM credit stalls; SQ waits), per dispatch of the decode kernel with its duration.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r6ds
mkdir -p $OUT
timeout -k 10 300 python tools/decode_size.py 3 8 > $OUT/plain.json 2> $OUT/plain.err || { echo FAIL plain; tail $OUT/plain.err; exit 1; }
cat $OUT/plain.json
i=0
for pc in "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum" \
          "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $pc --kernel-trace --kernel-include-regex ngz_tpl --output-format csv -d $OUT/p$i -o run -- python3 tools/decode_size.py 2 6 > $OUT/p$i.json 2> $OUT/p$i.err || { echo FAIL pass $i; tail -5 $OUT/p$i.err; exit 3; }
  cat $OUT/p$i.json
done
python3 tools/pmc_dispatch.py ngz_tpl $OUT/p1 > $OUT/tcc.txt && python3 tools/pmc_dispatch.py ngz_tpl $OUT/p2 > $OUT/sq.txt
cat $OUT/tcc.txt $OUT/sq.txt

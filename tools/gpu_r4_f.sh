#!/bin/bash
# r4: async / kernel D2H (test + host-to-host bench), arena placement under translation and
# DRAM-credit counters (per dispatch, every placement trial), SQ counters of small vs large
# launches, and the cache-policy knobs.  usage: TAG=r4f bash tools/gpu_r4_f.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4f}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -m gpu --timeout 120 --timeout-method thread \
  -k "columns_to_host or t20_small" > $OUT/pytest.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for PK in "4 24" "6 24" "6 48"; do set -- $PK
  timeout -k 10 300 python3 bench.py --e2e --records 10000000 --steps 5 --warmup 2 --e2e-contexts $1 --e2e-ranges $2 \
    > $OUT/e2e_p$1_k$2.json 2> $OUT/e2e_p$1_k$2.err || { tail -5 $OUT/e2e_p$1_k$2.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$OUT/e2e_p$1_k$2.json'))
print('e2e P=$1 K=$2', ' '.join('%s %.2f ms %.1f GB/s' % (m, v['ms_per_step'], v['pcie_gbps']) for m, v in d['modes'].items()))"
done
# arena placement: per-dispatch counters of every trial (NGZ_DEBUG prints the trial times)
i=0
for pc in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum" \
          "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  NGZ_DEBUG=1 timeout -s KILL 180 rocprofv3 --pmc $pc --kernel-trace --kernel-include-regex ngz_tpl --output-format csv \
    -d $OUT/arena_p$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/arena_p$i.json 2> $OUT/arena_p$i.err \
    || { tail -5 $OUT/arena_p$i.err; exit 4; }
  grep "arena placement" $OUT/arena_p$i.err
done
python3 tools/pmc_dispatch.py ngz_tpl $OUT/arena_p1 $OUT/arena_p2
# SQ counters: T20 at 1.25e7 (one template launch) and at 1e8, config 3
for W in "t20s:--workload t20 --records 12500000" "t20:--workload t20" "mixed8:--workload mixed8"; do
  WN=${W%%:*}; WA=${W#*:}
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU \
    --kernel-trace --kernel-include-regex ngz_tpl --output-format csv -d $OUT/sq_$WN -o run -- \
    python3 bench.py $WA --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq_$WN.json 2> $OUT/sq_$WN.err || { tail -5 $OUT/sq_$WN.err; exit 5; }
  echo "== $WN"; python3 tools/pmc_dispatch.py ngz_tpl $OUT/sq_$WN | tail -9
done
CASES="t20=--workload t20;mixed8=--workload mixed8" SETTINGS="base=;ld=NGZ_LD_AUX=2;st=NGZ_ST_AUX=2" \
  STEPS=10 TAG=${TAG:-r4f}/nt bash tools/gpu_sweep.sh || exit 6

#!/bin/bash
# r4: mid-size launches (T20 at 1.25e7 records): column spacing (NGZ_CAP_PAD) and DRAM credit
# stalls per record against the 1e8 launch.  usage: TAG=r4i bash tools/gpu_r4_i.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4i}
mkdir -p $OUT
CASES="n4=--workload t20 --records 12500000" SETTINGS="p0=NGZ_CAP_PAD=0;p1=NGZ_CAP_PAD=1;p5=NGZ_CAP_PAD=5;p17=NGZ_CAP_PAD=17;p64=NGZ_CAP_PAD=64;p500=NGZ_CAP_PAD=500" \
  STEPS=20 TAG=${TAG:-r4i}/pad bash tools/gpu_sweep.sh || exit 3
for W in "n4:--workload t20 --records 12500000" "n7:--workload t20"; do
  WN=${W%%:*}; WA=${W#*:}
  timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
    --kernel-trace --kernel-include-regex ngz_tpl --output-format csv -d $OUT/ea_$WN -o run -- \
    python3 bench.py $WA --steps 2 --warmup 1 --no-cpu-baseline > $OUT/ea_$WN.json 2> $OUT/ea_$WN.err || { tail -5 $OUT/ea_$WN.err; exit 5; }
  echo "== $WN"; python3 tools/pmc_dispatch.py ngz_tpl $OUT/ea_$WN | tail -4
done

#!/bin/bash
# Bench-line sweep over environment settings: one bench.py run per (case, setting), each line's
# decode kernel time, fraction and step time summarised.  Optional per-dispatch kernel trace of
# chosen cases (rocprofv3 --kernel-trace; the per-launch durations of a multi-template step).
# usage: CASES="t20s=--workload t20 --records 12500000;mixed8=--workload mixed8" \
#        SETTINGS="b2=NGZ_LDS_BLOCKS_PER_CU=2;b8=NGZ_LDS_BLOCKS_PER_CU=8" [TRACE="mixed8:b8 mixed8:b2"] \
#        [STEPS=10] TAG=r4a bash tools/gpu_sweep.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export NGZ_EXPERIMENTS=1  # env knobs are read only by the experiment build (tools/build_experiments.sh)
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
IFS=';' read -ra CS <<< "$CASES"
IFS=';' read -ra SS <<< "${SETTINGS:-default=}"
for c in "${CS[@]}"; do
  CN=${c%%=*}; CA=${c#*=}
  for s in "${SS[@]}"; do
    SN=${s%%=*}; SE=${s#*=}
    ( [ -n "$SE" ] && export $SE
      timeout -k 10 300 python3 bench.py $CA --no-cpu-baseline --steps ${STEPS:-10} --warmup 3 > $OUT/$CN.$SN.json 2> $OUT/$CN.$SN.err ) \
      || { echo "FAILED $CN $SN"; tail -5 $OUT/$CN.$SN.err; exit 3; }
    python3 - $OUT/$CN.$SN.json "$CN" "$SN" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("%-10s %-12s kernel %.4f ms  frac %.4f  step %.4f ms  %.3e rec/s" % (sys.argv[2], sys.argv[3], r["kernel_ms"], r["frac"], d["ms_per_step"], d["value"]))
PY
  done
done
for t in ${TRACE}; do
  CN=${t%%:*}; SN=${t#*:}
  CA=""; SE=""
  for c in "${CS[@]}"; do [ "${c%%=*}" == "$CN" ] && CA=${c#*=}; done
  for s in "${SS[@]}"; do [ "${s%%=*}" == "$SN" ] && SE=${s#*=}; done
  ( [ -n "$SE" ] && export $SE
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$CN.$SN -o run -- python3 bench.py $CA --no-cpu-baseline --steps 3 --warmup 2 > $OUT/trace_$CN.$SN.json 2> $OUT/trace_$CN.$SN.err ) \
    || { echo "TRACE FAILED $CN $SN"; tail -5 $OUT/trace_$CN.$SN.err; exit 4; }
  echo "== per-dispatch ngz_tpl, last step: $CN $SN"
  python3 tools/dispatches.py $OUT/trace_$CN.$SN 2>&1 | tail -40
done

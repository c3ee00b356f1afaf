#!/bin/bash
# r3: selected -m gpu tests (default: dist + rtc), smoke(), bench lines per workload (NGZ_GROUP A/B for
# the multi-template ones) and per aggregation key.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r3g}
mkdir -p $OUT
( while sleep 20; do date >> $OUT/ticks.txt; done ) &
TK=$!
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_dist.py tests/test_gpu_rtc.py} ${K:+-k "$K"} -v -x \
  --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
kill $TK
grep -E "PASSED|FAILED|ERROR" $OUT/pytest.log | tail -12
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 2; }
tail -1 $OUT/smoke.log
for WG in ${WLS:-t20:0 mixed8:0 mixed8:1 cfg5:0 cfg5:1 cfg4:0}; do
  W=${WG%%:*}; G=${WG##*:}
  A="--workload $W --steps 20 --warmup 5 --no-cpu-baseline"
  [ $W = cfg4 ] && A="$A --records 20000000"
  NGZ_GROUP=$G timeout -k 10 300 python bench.py $A > $OUT/${W}_g$G.json 2> $OUT/${W}_g$G.err || { tail -5 $OUT/${W}_g$G.err; exit 3; }
  python -c "import json; d=json.load(open('$OUT/${W}_g$G.json')); print('$W group=$G', round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), 'step', round(d['ms_per_step'],4), '%.3g' % d['value'])"
done
for K in ${AGGS:-proto_dir dport 5tuple}; do
  timeout -k 10 300 python bench.py --agg $K --steps 10 --warmup 2 > $OUT/agg_$K.json 2> $OUT/agg_$K.err || { tail -5 $OUT/agg_$K.err; exit 4; }
  python -c "import json; d=json.load(open('$OUT/agg_$K.json')); print('$K', d['path'], round(d['push_kernels_ms'],3), 'first', round(d['config']['first_push_ms'],3), 'groups', d['config']['groups'])"
done

#!/bin/bash
# Round 6: the arena placement probe against the decode trials (NGZ_OPT_PLACE_PROBE 2: every trial
# arena gets the probe and the batch's decode; the decodes decide), then the probe deciding (1).
set -o pipefail
OUT=gpurun_out/r6p
mkdir -p $OUT
for i in 1 2 3 4; do
  timeout -k 10 240 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --place-probe 2 > $OUT/t20_diag_$i.json 2> $OUT/t20_diag_$i.err || { echo FAIL t20 $i; tail $OUT/t20_diag_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/t20_diag_$i.json'))['roofline'];print('t20', [round(x,3) for x in d['placement_trials_ms']], [round(x,3) for x in d['placement_probe_ms']], d['frac'])"
done
for w in mixed8 cfg4; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline --place-probe 2 > $OUT/${w}_diag.json 2> $OUT/${w}_diag.err || { echo FAIL $w; tail $OUT/${w}_diag.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/${w}_diag.json'))['roofline'];print('$w', [round(x,3) for x in d['placement_trials_ms']], [round(x,3) for x in d['placement_probe_ms']], d['frac'])"
done
for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --place-probe 1 > $OUT/t20_probe_$i.json 2> $OUT/t20_probe_$i.err || { echo FAIL probe $i; tail $OUT/t20_probe_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/t20_probe_$i.json'))['roofline'];print('t20 probe-decides', [round(x,3) for x in d['placement_probe_ms']], d['placement_kept'], d['kernel_ms'], d['frac'])"
done

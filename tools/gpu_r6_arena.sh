#!/bin/bash
# Round 6: arena placement -- per-step decode times without trials (fresh allocation transient vs
# lifetime mode), then bench with probe-decided and decode-decided placement, 3 runs each.
set -o pipefail
OUT=gpurun_out/r6a
mkdir -p $OUT
timeout -k 10 300 python tools/arena_steps.py 4 > $OUT/steps.json 2> $OUT/steps.err || { echo FAIL steps; tail $OUT/steps.err; exit 1; }
cat $OUT/steps.json
for mode in 1 0; do for i in 1 2 3; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --place-probe $mode > $OUT/t20_m${mode}_$i.json 2> $OUT/t20_m${mode}_$i.err || { echo FAIL $mode $i; tail $OUT/t20_m${mode}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/t20_m${mode}_$i.json'))['roofline'];print('mode $mode', [round(x,3) for x in d.get('placement_trials_ms',[])], [round(x,3) for x in d.get('placement_probe_ms',[])], d['placement_kept'], round(d['kernel_ms'],3), round(d['frac'],4))"
done; done

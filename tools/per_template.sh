#!/bin/bash
# Per-template decode kernel times of a multi-template bench run, for env cases:
# CASES="a:ENV=1 b:ENV=2" [WORKLOAD=mixed8]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for c in ${CASES}; do
  name=${c%%:*}; envs=${c#*:}
  OUT=gpurun_out/pt_$name
  mkdir -p $OUT
  env $(echo $envs | tr ',' ' ') NGZ_DECODE_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --workload ${WORKLOAD:-mixed8} --steps 3 --warmup 2 --no-cpu-baseline > $OUT/b.json 2>&1 || exit 1
  python3 - $OUT ${WORKLOAD:-mixed8} $name <<'PY'
import csv, sys
sys.path.insert(0, '.')
from netgauze_amd import synth
out, wl, name = sys.argv[1:]
tpl = synth.CFG3_TEMPLATES if wl == "mixed8" else synth.CFG5_TEMPLATES
rows = sorted([r for r in csv.DictReader(open(out + '/run_kernel_trace.csv')) if 'ngz_tpl' in r['Kernel_Name']],
              key=lambda r: int(r['Start_Timestamp']))[-len(tpl):]
n = 100_000_000 // len(tpl)
line, tot = [], 0
for (tid, f), r in zip(tpl, rows):
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    tot += d
    line.append('%d:%.3f(v%s,l%s)' % (tid, d, r['VGPR_Count'], r['LDS_Block_Size']))
print(name, 'sum %.3f' % tot, ' '.join(line))
PY
done

#!/bin/bash
# Copy the judged pieces of a gpu_round.sh output dir into profiles/<tag>/
set -e
SRC=gpurun_out/$1
DST=profiles/$1
mkdir -p $DST
for f in bench.json e2e_1e7.json e2e_1e8.json hbm_probe.txt summary.txt traffic.json trace_bench.json pytest_gpu.log; do
  [ -f $SRC/$f ] && cp $SRC/$f $DST/
done
cp $SRC/trace/run_kernel_stats.csv $DST/kernel_stats.csv
for C in FETCH_SIZE WRITE_SIZE; do
  python3 - $SRC $DST $C <<'PY'
import csv, sys
src, dst, c = sys.argv[1:]
rows = [r for r in csv.DictReader(open(f'{src}/pmc_{c}/run_counter_collection.csv'))
        if 'ngz_tpl' in r['Kernel_Name'] or 'k_decode' in r['Kernel_Name']]
if rows:
    with open(f'{dst}/pmc_{c}_decode.csv', 'w') as f:
        w = csv.DictWriter(f, fieldnames=rows[0].keys()); w.writeheader(); w.writerows(rows)
PY
done
ls $DST

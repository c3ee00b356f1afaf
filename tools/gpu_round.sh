#!/bin/bash
# Round evidence on one GPU box: parity tests (both kernel paths), the
# default bench line (with cpu_baseline), host-to-host rate, HBM ceiling
# probe, rocprofv3 kernel stats of the bench command, PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 2
cat $OUT/bench.json
timeout -k 10 300 python bench.py --e2e --records 10000000 --steps 5 --warmup 1 > $OUT/e2e_1e7.json 2> $OUT/e2e.err || exit 3
cat $OUT/e2e_1e7.json
hipcc -O3 --offload-arch=gfx950 tools/hbm_probe.hip -o /tmp/hbm_probe && timeout -k 5 200 /tmp/hbm_probe > $OUT/hbm_probe.txt || exit 4
cat $OUT/hbm_probe.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace.err || exit 5
cat $OUT/trace_bench.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$C -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/pmc_$C.json 2> $OUT/pmc_$C.err || exit 6
done
python3 tools/summarize_profile.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt

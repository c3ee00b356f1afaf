#!/bin/bash
# Iteration loop on the GPU box: parity tests, a short bench, kernel-trace stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-iter}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/ -q -m gpu -x ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -v "^    " $OUT/pytest_gpu.log | tail -25
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --records ${REC:-100000000} --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 2
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --records ${REC:-100000000} --steps 5 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1 || exit 3
python3 tools/summarize_profile.py $OUT

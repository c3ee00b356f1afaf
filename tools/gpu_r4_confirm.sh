#!/bin/bash
# r4: the final tree -- every -m gpu test, smoke(), the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r4end}
mkdir -p gpurun_out/$TAG
bash tools/gpu_tests_all.sh || exit 1
cp gpurun_out/pytest_gpu.log gpurun_out/$TAG/
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 2; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/$TAG/bench_default.json 2> gpurun_out/$TAG/bench_default.err || { tail -20 gpurun_out/$TAG/bench_default.err; exit 3; }
cat gpurun_out/$TAG/bench_default.json

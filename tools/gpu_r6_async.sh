#!/bin/bash
# Round 6: ngz_decode_batch_submit / _wait -- the GPU test, then config 4 with 1 / 2 / 3 contexts driven
# by threads and by one thread submitting.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r6async
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_async.py tests/test_gpu_rtc.py > $OUT/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for args in "--contexts 1" "--contexts 2" "--contexts 2 --submit" "--contexts 3" "--contexts 3 --submit"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 200 python bench.py --workload cfg4 --records 20000000 --steps 30 --warmup 5 --no-cpu-baseline $args > $OUT/cfg4_$tag.json 2> $OUT/cfg4_$tag.err || { echo FAIL $args; tail -5 $OUT/cfg4_$tag.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'])" $OUT/cfg4_$tag.json "$args"
done

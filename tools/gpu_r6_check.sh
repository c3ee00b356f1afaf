set -o pipefail
mkdir -p gpurun_out/r6v
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py::test_fuzz_regressions tests/test_gpu_records.py tests/test_gpu_dist.py tests/test_gpu_rtc.py tests/test_gpu_knobs.py > gpurun_out/r6v/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6v/tests.log; exit 1; }
tail -3 gpurun_out/r6v/tests.log
NGZ_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --records 20000000 > gpurun_out/r6v/dist2.json 2> gpurun_out/r6v/dist2.err || { echo DIST_FAILED; tail -20 gpurun_out/r6v/dist2.err; exit 1; }
cat gpurun_out/r6v/dist2.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r6v/t20.json 2> gpurun_out/r6v/t20.err || { echo BENCH_FAILED; tail -20 gpurun_out/r6v/t20.err; exit 1; }
cat gpurun_out/r6v/t20.json

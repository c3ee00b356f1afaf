#!/bin/bash
# Round 6: the NFv9 staged-row kernel with register-staged cells and 16-byte image stores -- the
# fuzz corpus, the NFv9 / config-4 parity tests and the config-4 profile (tools/gpu_r5_cfg4.sh).
set -o pipefail
mkdir -p gpurun_out/r6nf
timeout -k 10 1000 python -u -m pytest -q -s -x --timeout 600 --timeout-method thread tests/test_gpu_fuzz.py tests/test_gpu_parity.py -k "netflow or cfg4 or v9 or nfv9 or fuzz or variable or record" tests/test_gpu_records.py > gpurun_out/r6nf/tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r6nf/tests.log; exit 1; }
tail -2 gpurun_out/r6nf/tests.log
TAG=r6nf/cfg4 bash tools/gpu_r5_cfg4.sh

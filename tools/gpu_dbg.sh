#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NGZ_DEBUG=1 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "failing_record" 2>&1 | grep -v "^    " | tail -30

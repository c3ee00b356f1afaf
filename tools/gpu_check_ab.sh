#!/bin/bash
# GPU parity suite, then an aggregation A/B (CONFIGS) through tools/gpu_agg_ab.sh.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests.sh || exit 1
bash tools/gpu_agg_ab.sh

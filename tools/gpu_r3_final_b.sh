#!/bin/bash
# r3 round-end evidence, part B: config 3 / 5 profiles, aggregation profiles per key.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3}
TAG=$TAG WORKLOADS="${WORKLOADS:-mixed8 cfg5}" bash tools/gpu_profile.sh || exit 3
TAG=$TAG AGGS="${AGGS:-proto_dir dport 5tuple}" bash tools/gpu_profile_agg.sh || exit 4

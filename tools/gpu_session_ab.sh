set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_tests.sh || exit 1
TAG=cfg4_ab CONFIGS="NGZ_FRAME_STAGE=0;NGZ_FRAME_STAGE=16;NGZ_FRAME_STAGE=24;NGZ_FRAME_STAGE=32" bash tools/gpu_trace_ab.sh || exit 2
CONFIGS="NGZ_AGG_OWN_SPLIT=1;X=1" bash tools/gpu_agg_ab.sh

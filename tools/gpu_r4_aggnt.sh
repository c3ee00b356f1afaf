#!/bin/bash
# r4: nontemporal partition payload stores -- dport push A/B against the committed profile, parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/r4aggnt
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -v -m gpu --timeout 300 --timeout-method thread -k "partitioned" > $OUT/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $OUT/pytest.log | head -20; tail -5 $OUT/pytest.log; exit 2; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --agg dport --steps 10 --warmup 2 > $OUT/dport$i.json 2> $OUT/dport$i.err || { tail -5 $OUT/dport$i.err; exit 3; }
  python3 -c "import json; d=json.load(open('$OUT/dport$i.json')); print('dport push %.3f ms' % d['push_kernels_ms'])"
done

#!/bin/bash
# Same-box ceiling and host-to-host rate: HBM probe (copy / read / write shapes), the default
# bench line, and bench.py --e2e (pinned host datagrams -> H2D -> decode -> D2H of every column).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ceiling}
mkdir -p $OUT
hipcc -O3 --offload-arch=gfx950 tools/hbm_probe.hip -o /tmp/hbm_probe && timeout -k 5 200 /tmp/hbm_probe > $OUT/hbm_probe.txt || exit 1
grep "grid  1024" $OUT/hbm_probe.txt | cut -c1-160
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 2
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('t20 kernel_ms %.3f frac %.3f step %.3f' % (d['roofline']['kernel_ms'], d['roofline']['frac'], d['ms_per_step']))" $OUT/bench.json
timeout -k 10 300 python bench.py --e2e --records 10000000 --steps 5 --warmup 1 > $OUT/e2e_1e7.json 2> $OUT/e2e.err || exit 3
cut -c1-400 $OUT/e2e_1e7.json

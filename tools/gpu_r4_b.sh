#!/bin/bash
# r4: GPU tests of the new paths (byte-valued aggregation, split framing), config 4 split vs not,
# the PCIe probe and the host-to-host bench.  usage: TAG=r4b bash tools/gpu_r4_b.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4b}
mkdir -p $OUT
( while sleep 20; do date >> $OUT/ticks.txt; done ) &
TK=$!
trap "kill $TK" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_agg.py tests/test_gpu_parity.py \
  -v -m gpu --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $OUT/pytest.log | head -20
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for S in 1 0; do
  NGZ_SPLIT=$S timeout -k 10 300 python3 bench.py --workload cfg4 --records 20000000 --steps 20 --warmup 5 --no-cpu-baseline \
    > $OUT/cfg4_split$S.json 2> $OUT/cfg4_split$S.err || { tail -5 $OUT/cfg4_split$S.err; exit 3; }
  python3 -c "import json,sys; d=json.load(open('$OUT/cfg4_split$S.json')); print('cfg4 split=$S step %.4f ms kernel %.4f ms' % (d['ms_per_step'], d['roofline']['kernel_ms']))"
done
NGZ_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_cfg4 -o run -- \
  python3 bench.py --workload cfg4 --records 20000000 --steps 5 --warmup 3 --no-cpu-baseline > $OUT/trace_cfg4.json 2> $OUT/trace_cfg4.err \
  || { tail -5 $OUT/trace_cfg4.err; exit 4; }
python3 tools/dispatches.py $OUT/trace_cfg4 | tail -20
timeout -k 10 120 python3 tools/pcie_probe.py > $OUT/pcie_probe.json 2> $OUT/pcie_probe.err || { tail -5 $OUT/pcie_probe.err; exit 5; }
cat $OUT/pcie_probe.json
timeout -k 10 300 python3 bench.py --e2e --records 10000000 --steps 5 --warmup 2 > $OUT/e2e.json 2> $OUT/e2e.err || { tail -5 $OUT/e2e.err; exit 6; }
cat $OUT/e2e.json

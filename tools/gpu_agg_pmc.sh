#!/bin/bash
# PMC passes (one per run) over the aggregation bench: wave-cycle breakdown and atomic traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aggpmc}
mkdir -p $OUT
K=${AGG_KEY:-proto_dir}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv -d $OUT/sq -o run -- python3 bench.py --agg $K --steps 2 --warmup 1 --records 20000000 > $OUT/sq.json 2> $OUT/sq.err || { tail -5 $OUT/sq.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/tcc -o run -- python3 bench.py --agg $K --steps 2 --warmup 1 --records 20000000 > $OUT/tcc.json 2> $OUT/tcc.err || { tail -5 $OUT/tcc.err; exit 2; }
python3 - <<'PY'
import csv, glob, os, collections
out = os.environ.get("TAG", "aggpmc")
for sub in ("sq", "tcc"):
    for f in glob.glob("gpurun_out/%s/%s/*counter_collection.csv" % (out, sub)):
        agg = collections.defaultdict(float)
        n = collections.Counter()
        for r in csv.DictReader(open(f)):
            if "k_agg_insert" in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
        for k, v in sorted(agg.items()):
            print(sub, k, v / max(1, n[k]) * 1.0, "(per dispatch-row avg over %d rows)" % n[k])
PY

"""The product library takes no tuning from the environment (ngz_knobs.cpp).

Rounds 1-4 read about 45 experiment knobs (NGZ_LDS, NGZ_CAP_PAD, NGZ_LD_AUX, NGZ_AGG_PART, ...)
from the environment inside libngz, so a collector's environment could change which kernels ran.
They are now ngz_ctx_set_option / ngz_agg_set_option options or exist only in the
-DNGZ_EXPERIMENTS build.  Here a child process decodes the same T20 and config-4 batches with
every old knob set to a value that used to change kernels or layout, and its column bytes,
datagram headers and per-template counts hash equal to a clean child's."""
import hashlib
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# values that changed kernels / layout / paths before (see git history of ngz_host.cpp, ngz_rtc.cpp)
OLD_KNOBS = {
    "NGZ_LDS": "0", "NGZ_LDS_BUDGET": "32768", "NGZ_LDS_MAXW": "1", "NGZ_LDS_DIRECT_MIN": "4", "NGZ_RECMAP": "1",
    "NGZ_SPLIT": "1", "NGZ_GROUP": "1", "NGZ_ARENA_MIN_MB": "4096", "NGZ_DSUM": "0", "NGZ_DECODE_STREAMS": "1",
    "NGZ_SPECIALIZE": "0", "NGZ_SPIN": "0", "NGZ_ARENA_CONTIG": "1", "NGZ_PLACE_TRIALS": "1", "NGZ_CAP_PAD": "7",
    "NGZ_BLOCKS_PER_CU": "1", "NGZ_LDS_BLOCKS_PER_CU": "1", "NGZ_LD_AUX": "3", "NGZ_ST_AUX": "0", "NGZ_WIN_ROT": "3",
    "NGZ_RTC_LAYOUT": "c2", "NGZ_RTC_LDS_LAYOUT": "c4", "NGZ_RTC_LONG": "c2", "NGZ_RTC_EXP": "1", "NGZ_TRACE": "1",
    "NGZ_AGG_ROW_PACK": "1", "NGZ_AGG_NO_PACK": "1", "NGZ_AGG_NO_KW": "1", "NGZ_AGG_NO_OWN": "1",
    "NGZ_AGG_HASH_BITS": "3", "NGZ_AGG_GRID": "1", "NGZ_AGG_LC": "0", "NGZ_AGG_OWN_SPLIT": "1", "NGZ_AGG_PART": "1",
    "NGZ_AGG_RED_RPT": "1", "NGZ_AGG_RED_THREADS": "64",
}

CHILD = r"""
import hashlib, json, sys
sys.path.insert(0, ROOT)
import numpy as np, torch
from netgauze_amd import synth, _lib
from netgauze_amd.flow import FlowInfoCodec
from netgauze_amd.aggregate import FlowAggregator
out = {"path": _lib.LIB_PATH}
dev = torch.device("cuda:0")
codec = FlowInfoCodec(0, rtc_sync=True)
codec.decode_datagrams([synth.template_message()])
rec = synth.t20_records(2_000_000, device=dev)
buf, offs, lens = synth.ipfix_data_stream(rec, 64)
for step in range(2):  # the second batch runs the steady-state (predicted) launches
    batch = codec.decode_batch(buf, offs, lens)
h = hashlib.sha256()
for s in batch.slots:
    for f in range(len(s.fields)):
        h.update(s.column_bytes(f).tobytes())
h.update(batch.dgram_headers().tobytes())
out["t20"] = h.hexdigest()
agg = FlowAggregator([(0, 8, 0, 0), (0, 12, 0, 0), (0, 7, 0, 0), (0, 11, 0, 0), (0, 4, 0, 0), (0, 1, 0, 1),
                      (0, 2, 0, 1)], capacity=1 << 22, lateness_s=60)
agg.push(batch, 4739, 0)
rows = agg.flush()
out["agg"] = hashlib.sha256(json.dumps(sorted(repr(sorted(r.items())) for r in rows)).encode()).hexdigest()
c4 = FlowInfoCodec(0, rtc_sync=True)
dg = synth.cfg4_datagrams(40_000)
for part in (dg[: len(dg) // 2], dg[len(dg) // 2:]):
    b4 = c4.decode_datagrams(part)
h = hashlib.sha256()
for s in b4.slots:
    for f in range(len(s.fields)):
        h.update(s.column_bytes(f).tobytes())
h.update(b4.dgram_headers().tobytes())
out["cfg4"] = h.hexdigest()
out["counts"] = [sorted(c4.template_counts(9).items()), sorted(c4.template_counts(10).items())]
print(json.dumps(out))
"""


def run_child(extra_env):
    env = {k: v for k, v in os.environ.items() if not k.startswith("NGZ_")}
    env.update(extra_env)
    p = subprocess.run([sys.executable, "-c", CHILD.replace("ROOT", repr(ROOT), 1)], env=env, capture_output=True,
                       text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_old_environment_knobs_change_nothing():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    clean = run_child({})
    knobbed = run_child(OLD_KNOBS)
    assert clean["path"].endswith("libngz.so") and knobbed["path"] == clean["path"]
    assert knobbed == clean


def test_product_library_reads_no_knobs():
    """Only ngz_knobs.cpp reads the environment: one getenv behind -DNGZ_EXPERIMENTS and
    NGZ_DEBUG; the built product library is not an experiments build."""
    import ctypes
    import glob
    import re
    srcs = glob.glob(os.path.join(ROOT, "netgauze_amd", "csrc", "*"))
    hits = {os.path.basename(f): len(re.findall(r"\bgetenv\s*\(", open(f, errors="replace").read()))
            for f in srcs if os.path.isfile(f) and not f.endswith(".inc")}
    hits = {k: v for k, v in hits.items() if v}
    assert hits == {"ngz_knobs.cpp": 2}, hits
    from netgauze_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    assert _lib.LIB_PATH.endswith("libngz.so")
    assert lib.ngz_experiments_build() == 0

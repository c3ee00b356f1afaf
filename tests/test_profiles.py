"""The committed profile evidence is self-consistent (CPU): every traffic.json's decode time per
timed step fits inside the step it was measured in (the config-3/5 summaries of r4
reported more decode time per step than the step took)."""
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _step_ms(d):
    for name in ("trace_bench.json", "bench.json"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            lines = [l for l in open(p).read().splitlines() if l.strip().startswith("{")]
            if lines:
                return json.loads(lines[-1]).get("ms_per_step")
    return None


def test_timed_decode_fits_in_the_step():
    checked = 0
    for f in glob.glob(os.path.join(ROOT, "profiles", "**", "traffic.json"), recursive=True):
        t = json.load(open(f))
        timed = t.get("timed_kernel_ms_trace") or t.get("timed_kernel_ms_stats")
        step = t.get("ms_per_step_trace_run") or _step_ms(os.path.dirname(f))
        if timed is None or step is None:
            continue
        assert timed <= step, (os.path.relpath(f, ROOT), timed, step)
        checked += 1
    assert checked >= 5

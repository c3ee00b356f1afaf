"""Run-time kernel compiles are off the decode path (ngz_rtc.cpp): a template
with a new layout compiles on a background thread while its context decodes
it with the generic kernel (bit-exact either way), and another context's
batches are not delayed by that compile."""
import os
import struct
import time

import pytest

import parity
from netgauze_amd import _lib as L

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _msg(sets, seq=1):
    body = b"".join(sets)
    return struct.pack(">HHIII", 10, 16 + len(body), 1_700_000_000, seq, 7) + body


def _set(sid, payload):
    return struct.pack(">HH", sid, 4 + len(payload)) + payload


def _fresh_layout(tid):
    """A template layout no earlier test compiled (random octet-array widths)."""
    w = os.urandom(3)
    fields = [(8, 4), (210, 1 + w[0] % 61), (7, 2), (1, 8), (210, 1 + w[1] % 29), (4, 1), (210, 1 + w[2] % 13)]
    body = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, ln) for i, ln in fields)
    rl = sum(ln for _, ln in fields)
    return _msg([_set(2, body)]), rl


def _data(tid, rl, n_msgs, per, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    return [_msg([_set(tid, rng.integers(0, 256, size=rl * per, dtype=np.uint8).tobytes())], seq=m)
            for m in range(n_msgs)]


def test_compile_is_off_the_decode_path():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.flow import FlowInfoCodec
    # the compile time of a fresh layout, waited for (NGZ_OPT_RTC_SYNC 1)
    s = FlowInfoCodec(0, rtc_sync=True)
    tm, rl = _fresh_layout(700)
    t0 = time.perf_counter()
    b = s.decode_datagrams([tm])
    t_compile = time.perf_counter() - t0
    assert t_compile > 0.02, t_compile  # a hiprtc compile, not a cache hit
    # context B: its template's kernel is ready
    B = FlowInfoCodec(0, rtc_sync=True)
    tmB, rlB = _fresh_layout(701)
    B.decode_datagrams([tmB])
    dataB = _data(701, rlB, 20, 30, 1)
    B.decode_datagrams(dataB)
    # context A (background compiles): a new layout and its data in one batch
    A = FlowInfoCodec(0)
    tmA, rlA = _fresh_layout(702)
    dataA = _data(702, rlA, 20, 30, 2)
    t0 = time.perf_counter()
    bA = A.decode_datagrams([tmA] + dataA)
    t_a = time.perf_counter() - t0
    slot = [i for i, sl in enumerate(bA.slots) if sl.template_id == 702][0]
    assert bA.slot_kernel(slot) == 2            # decoded by the generic kernel while its own compiles
    oracle, _ = parity.oracle_datagrams([tmA] + dataA)
    assert parity.check_batch(bA, oracle)["records"] == 20 * 30
    # B's batch while A's compile may still run
    t0 = time.perf_counter()
    bB = B.decode_datagrams(dataB)
    t_b = time.perf_counter() - t0
    assert bB.slot_kernel([i for i, sl in enumerate(bB.slots) if sl.template_id == 701][0]) == 1
    assert t_a < 0.5 * t_compile and t_b < 0.5 * t_compile, (t_a, t_b, t_compile)
    # A switches to its specialised kernel once the compile is done, results unchanged
    oc = parity.O.FlowInfoCodec()
    oc.decode(bytearray(tmA))
    deadline = time.time() + 30
    while True:
        b2 = A.decode_datagrams(dataA)
        k = b2.slot_kernel([i for i, sl in enumerate(b2.slots) if sl.template_id == 702][0])
        if k == 1 or time.time() > deadline:
            break
        time.sleep(0.05)
    assert k == 1
    o2, _ = parity.oracle_datagrams(dataA, oc)
    assert parity.check_batch(b2, o2)["records"] == 20 * 30
    assert int((b2.dgram_headers()["status"] == L.NGZ_DG_OK).sum()) == 20


_EXIT_CHILD = r"""
import os, struct, sys
sys.path.insert(0, os.environ["NGZ_ROOT"])
sys.path.insert(0, os.path.join(os.environ["NGZ_ROOT"], "tests"))
import test_gpu_rtc as T
from netgauze_amd import _lib as L
from netgauze_amd.flow import FlowInfoCodec
c = FlowInfoCodec(0)  # library default: per-template kernels compiled in the background
dg = []
for k in range(4):    # four fresh layouts: four compiles in flight
    tm, rl = T._fresh_layout(900 + k)
    dg += [tm] + T._data(900 + k, rl, 2, 20, k)
b = c.decode_datagrams(dg)
assert b.n_records == 4 * 2 * 20, b.n_records
ready = [b.slot_kernel(s.index) for s in b.slots]
print("EXITING", ready, flush=True)
sys.exit(0)       # while the background compiles run
"""


def test_exit_with_background_compiles_in_flight():
    """A process that exits right after a decode started background compiles exits cleanly
    (r2: a rank hung at exit with one in flight; root cause in ngz_rtc.cpp prime_rtc_runtime)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NGZ_ROOT=root)
    p = subprocess.run([sys.executable, "-c", _EXIT_CHILD], env=env, capture_output=True, text=True, timeout=90)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    assert "EXITING" in p.stdout


def test_c_host_exits_after_destroy_with_compiles_in_flight():
    """A plain C host (tests/native/exit_after_compile.c) that starts four background compiles,
    destroys its context and returns from main -- without ngz_rtc_drain -- exits 0:
    ngz_ctx_destroy joins the compiles its context started or waits on (synchronous drop,
    codec.rs:68-82).  The compiles were still running when the batch returned (slot kernel 2)."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "netgauze_amd", "bin", "ngz-exit-check")
    assert os.path.exists(exe), "built by __graft_entry__.build()"
    env = {k: v for k, v in os.environ.items() if not k.startswith("NGZ_")}
    p = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=90)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-2000:])
    fields = dict(kv.split("=") for kv in p.stdout.split())
    assert int(fields["records"]) == 4 * 2 * 200
    assert int(fields["compiling"]) >= 1, p.stdout

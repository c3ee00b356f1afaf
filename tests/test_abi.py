"""CPU checks of the C-ABI library: it is built, it loads, and it exports
every function include/ngz/flow_decode.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", "ngz", h) for h in ("flow_decode.h", "flow_ingest.h",
                                                                        "flow_aggregate.h")]


def declared_functions(headers=HEADERS):
    names = set()
    for h in headers:
        text = open(h).read()
        names |= set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(ngz_[a-z_0-9]+)\s*\(", text, re.M))
    return sorted(names)


def test_header_declares_abi():
    from netgauze_amd import _lib
    assert declared_functions(HEADERS[:1]) == sorted(_lib.ABI_FUNCTIONS)
    assert declared_functions(HEADERS[1:2]) == sorted(_lib.INGEST_FUNCTIONS)
    assert declared_functions(HEADERS[2:]) == sorted(_lib.AGG_FUNCTIONS)


def test_agg_config_validation_without_device():
    """AggregationConfig::validate / validate_operation_compatibility are checked before any
    device call (config.rs:107-119, 212-250): zero window, lateness > window, Add on a
    non-numeric IE, Min on a float all fail; the row layout matches ngz_agg_row."""
    from netgauze_amd import _lib
    lib = _lib.load()
    A = _lib.AggField

    def create(fields, window=60000, lateness=10000):
        arr = (A * max(len(fields), 1))(*[A(p, i, x, o) for p, i, x, o in fields])
        h = ctypes.c_void_p()
        return lib.ngz_agg_create(0, arr, len(fields), window, lateness, 1024, ctypes.byref(h))
    ok = [(0, 8, 0, _lib.NGZ_AGG_KEY), (0, 1, 0, _lib.NGZ_AGG_ADD)]
    assert create(ok, window=0) == -1
    assert create(ok, window=1000, lateness=2000) == -1
    assert create([(0, 8, 0, _lib.NGZ_AGG_ADD)]) == -1        # sourceIPv4Address: not arithmetic
    assert create([(0, 4, 0, _lib.NGZ_AGG_ADD)]) == -1        # protocolIdentifier: sub-registry
    assert create([(0, 6, 0, _lib.NGZ_AGG_OR)]) in (-2, -3)   # tcpControlBits OR: valid, needs the device
    assert create([(0, 56, 0, _lib.NGZ_AGG_ADD)]) == -1       # sourceMacAddress
    assert create([(0, 1, 0, 9)]) == -1                       # unknown op


def test_library_exports_every_declared_symbol():
    from netgauze_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libngz.so not built: run __graft_entry__.build()")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    _lib.load()


def test_ctx_create_without_device_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from netgauze_amd import _lib
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.ngz_ctx_create(0, ctypes.byref(ctx)) != 0
    assert not ctx.value


def test_product_does_not_import_oracle():
    """The product path never routes through the CPU oracle."""
    pkg = os.path.join(ROOT, "netgauze_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "ngz_oracle" not in text and "oracle/" not in text, f


@pytest.mark.parametrize("tid", [t for t, _ in __import__("netgauze_amd.synth", fromlist=["x"]).CFG5_TEMPLATES])
def test_template_kernels_compile_for_gfx950(tid):
    """The per-template decode kernel of every config-5 template (config 3 and
    its width permutations) is generated
    and compiled for gfx950 by hiprtc (no device needed): LDS-staged where the
    rows fit the workgroup budget, direct column stores otherwise."""
    import struct
    from netgauze_amd import _lib, synth
    fields = dict(synth.CFG5_TEMPLATES)[tid]
    rec = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, ln) for i, ln in fields)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    buf = ctypes.create_string_buffer(1 << 20)
    rc = lib.ngz_template_kernel(rec, len(rec), 1, buf, len(buf))
    src = buf.value.decode()
    assert rc == 0, src[-2000:]
    assert "ngz_tpl" in src
    assert ("run_lds" in src) == ("NGZ_LDS_WAVES" in src)

"""CPU ORACLE / BASELINE loader (test infrastructure): ctypes binding of
oracle/cpu/libngz_cpu.so (built by oracle/Makefile)."""
import ctypes
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpu", "libngz_cpu.so")


def load():
    lib = ctypes.CDLL(_PATH)
    P = ctypes.c_void_p
    lib.ngz_cpu_decode.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, ctypes.c_int, P, ctypes.c_int, P]
    lib.ngz_cpu_decode.restype = ctypes.c_uint64
    return lib


def decode(bytes_np, offs_np, lens_np, template_msg, threads=1, nsums=0):
    lib = load()
    b = np.ascontiguousarray(bytes_np, dtype=np.uint8)
    o = np.ascontiguousarray(offs_np, dtype=np.uint64)
    ln = np.ascontiguousarray(lens_np, dtype=np.uint32)
    t = np.frombuffer(template_msg, dtype=np.uint8).copy() if template_msg else None
    sums = np.zeros(max(nsums, 1), dtype=np.uint64)
    err = ctypes.c_uint64()
    n = lib.ngz_cpu_decode(b.ctypes.data, o.ctypes.data, ln.ctypes.data, len(ln),
                           t.ctypes.data if t is not None else None, len(t) if t is not None else 0,
                           threads, sums.ctypes.data, nsums, ctypes.byref(err))
    return int(n), sums[:nsums], int(err.value)

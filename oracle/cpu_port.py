"""CPU ORACLE / BASELINE loader (test infrastructure): ctypes binding of
oracle/cpu/libngz_cpu.so (built by oracle/Makefile)."""
import ctypes
import os

import numpy as np

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpu", "libngz_cpu.so")


def load():
    lib = ctypes.CDLL(_PATH)
    P = ctypes.c_void_p
    lib.ngz_cpu_decode.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, P, ctypes.c_int, P]
    lib.ngz_cpu_decode.restype = ctypes.c_uint64
    return lib


def stream(template_msgs, bytes_np, offs_np, lens_np):
    """One message stream: the template messages, then the data messages."""
    t = b"".join(template_msgs)
    b = np.concatenate([np.frombuffer(t, dtype=np.uint8), np.ascontiguousarray(bytes_np, dtype=np.uint8)])
    tl = np.array([len(m) for m in template_msgs], dtype=np.uint64)
    to = np.concatenate([[0], np.cumsum(tl)[:-1]]).astype(np.uint64) if len(tl) else tl
    o = np.concatenate([to, np.asarray(offs_np, dtype=np.uint64) + np.uint64(len(t))])
    ln = np.concatenate([tl.astype(np.uint32), np.asarray(lens_np, dtype=np.uint32)])
    return b, o, ln, len(template_msgs)


def decode(bytes_np, offs_np, lens_np, template_msgs, threads=1, nsums=0):
    """template_msgs: bytes of one template message, or a list of them; every
    thread decodes them before its contiguous range of the data messages."""
    if isinstance(template_msgs, (bytes, bytearray)):
        template_msgs = [bytes(template_msgs)]
    b, o, ln, n_pre = stream(template_msgs or [], bytes_np, offs_np, lens_np)
    return decode_stream(b, o, ln, n_pre, threads, nsums)


def decode_stream(b, o, ln, n_pre, threads=1, nsums=0):
    lib = load()
    sums = np.zeros(max(nsums, 1), dtype=np.uint64)
    err = ctypes.c_uint64()
    n = lib.ngz_cpu_decode(b.ctypes.data, o.ctypes.data, ln.ctypes.data, len(ln), n_pre, threads, sums.ctypes.data,
                           nsums, ctypes.byref(err))
    return int(n), sums[:nsums], int(err.value)

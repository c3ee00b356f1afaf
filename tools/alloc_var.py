#!/usr/bin/env python3
"""Does decode time depend on where the arena / input land in HBM?  New
context (new arena hipMalloc) per trial, input re-created every other
trial, pad allocations in between to move the next allocations."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes
import torch
from netgauze_amd import synth
from netgauze_amd.flow import FlowInfoCodec

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
pads = []


def make_input():
    rec = synth.t20_records(n, seed=synth.SEED_CFG2, device=dev, first=0)
    b, o, l = synth.ipfix_data_stream(rec, 64)
    del rec
    return b, o, l


buf, offs, lens = make_input()
for trial in range(10):
    if trial % 3 == 2:
        del buf, offs, lens
        torch.cuda.empty_cache()
        pads.append(torch.empty((trial * 37 + 5) << 20, dtype=torch.uint8, device=dev))
        buf, offs, lens = make_input()
    codec = FlowInfoCodec(0)
    codec.decode_datagrams([synth.template_message()])
    ts = []
    for _ in range(4):
        codec.decode_batch(buf, offs, lens)
        ts.append(codec.last_timing()[0])
    b = codec.decode_batch(buf, offs, lens)
    sl = [x for x in b.slots if x.n_records][0]
    import time
    from netgauze_amd import _lib
    hip = _lib.hip()
    hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    hip.hipDeviceSynchronize()
    mt = []
    for _ in range(3):
        t0 = time.perf_counter()
        hip.hipMemset(sl.columns_ptr, 0, sl.block_bytes())
        hip.hipDeviceSynchronize()
        mt.append((time.perf_counter() - t0) * 1e3)
    print("trial %d input 0x%x arena 0x%x kernel ms %s | memset %.1f GB: %s ms" % (
        trial, buf.data_ptr(), sl.columns_ptr, " ".join("%.3f" % t for t in ts), sl.block_bytes() / 1e9,
        " ".join("%.3f" % t for t in mt)), flush=True)
    del codec
    pads.append(torch.empty((trial * 13 + 3) << 20, dtype=torch.uint8, device=dev))

#!/usr/bin/env python3
"""Round 6: can the variable-length record walk run next to the data it decodes?

Decodes config 4 (2*10^7 records, the bench's batch) once with the experiment build
(NGZ_EXPERIMENTS=1, tools/build_experiments.sh), then times k_walk_probe (ngz_kernels.hip) over the
batch's variable-length sets: mode 0 one lane per set walking from HBM; mode 1 each wave staging up
to 64 consecutive sets in LDS with coalesced 16-byte loads and one lane per set walking there; mode 2
the staging alone -- at several LDS stage sizes (waves per CU).  Every walked set's record count is
checked against the framing's.  One JSON line."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from netgauze_amd import synth
    from netgauze_amd.flow import FlowInfoCodec, lib as ngz_lib
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    lib = ngz_lib()
    f = lib.ngz_exp_walk_probe
    f.restype = ctypes.c_float
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.POINTER(ctypes.c_uint32)]
    dev = torch.device("cuda", 0)
    codec = FlowInfoCodec(0, rtc_sync=True)
    dg = synth.cfg4_datagrams(n, seed=synth.SEED_CFG4)
    codec.decode_datagrams(dg[:2])
    buf, offs, lens = synth.host_batch(dg[2:], device=dev)
    torch.cuda.synchronize()
    for _ in range(3):
        codec.decode_batch(buf, offs, lens)
    decode_ms = [round(codec.last_timing()[0], 4) for _ in range(1)]
    out = {"records": n, "decode_kernel_ms": decode_ms, "probe": []}
    o = (ctypes.c_uint32 * 2)()
    for mode in (0, 1, 2):
        for kb, bpc in ((8, 5), (12, 3), (16, 2), (36, 1)) if mode else ((16, 8),):
            ms = f(codec._ctx, mode, kb, bpc, reps, o)
            out["probe"].append({"mode": mode, "lds_kb_per_wave": kb if mode else 0, "blocks_per_cu": bpc,
                                 "us": round(1000 * ms, 1), "records": o[0], "mismatched_sets": o[1]})
            print(json.dumps(out["probe"][-1]), file=sys.stderr, flush=True)
    codec.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

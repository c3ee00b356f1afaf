#!/usr/bin/env python3
"""Round 6, configs 3 / 5 follow-up: does a 1.25*10^7-record launch reach the 10^8 launch's rate when its
columns get the 10^8 launch's stride?  tools/decode_size.py showed the mid-size deficit follows the launch,
not the allocation, with the column stride (1.25e7 rows) shared by both of its arenas.  Here T20 at 1.25e7
records is decoded on fresh contexts whose slot capacity is padded (NGZ_CAP_PAD windows of 1024 rows,
experiment build) so the column stride is 1.25e7, 2.5e7, 5e7 or 1e8 rows; placement trials off, so each
context shows its allocation's mode.  `reps` fresh contexts per stride, `steps` decodes each: HIP-event
decode ms.  One JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from netgauze_amd import synth
    from netgauze_amd.flow import FlowInfoCodec, OPT_PLACE_TRIALS
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    dev = torch.device("cuda", 0)
    ns = 12_500_000
    small = synth.stream_range(ns, 0, len(synth.stream_index(ns)[2]), None, device=dev)[:3]
    tm = [synth.template_message()]
    base_w = (ns + 1023) // 1024
    out = {}
    for stride in (12_500_000, 25_000_000, 50_000_000, 100_000_000):
        pad = max(0, (stride + 1023) // 1024 - base_w)
        os.environ["NGZ_CAP_PAD"] = str(pad)
        runs = []
        for _ in range(reps):
            c = FlowInfoCodec(0, rtc_sync=True, options={OPT_PLACE_TRIALS: 1})
            c.decode_datagrams(tm)
            ms = []
            for _ in range(steps):
                c.decode_batch(*small)
                ms.append(round(c.last_timing()[0], 4))
            runs.append(ms)
            c.close()
            torch.cuda.synchronize()
            print(json.dumps({"stride_rows": stride, "pad_windows": pad, "ms": ms}), file=sys.stderr, flush=True)
        out[str(stride)] = runs
    print(json.dumps({"steps_ms": out, "alg_bytes": 127 * ns}))


if __name__ == "__main__":
    main()

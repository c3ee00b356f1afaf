#!/usr/bin/env python3
"""Round 6, configs 3 / 5 experiment: is the mid-size launch deficit the launch size
or the allocation?  T20 at 1.25*10^7 records (one config-3 / config-5 template's share) decoded
  fresh:  on a fresh context (arena sized for 1.25e7 rows), and
  sub:    on a context that first decoded 10^8 records (the same batch then sits in the first
          eighth of that 10^8-row arena; column stride 1.25e7 rows either way),
plus the 10^8 batch itself on that context.  Placement trials off (NGZ_OPT_PLACE_TRIALS 1), so each
context shows the mode its allocation got.  Per step: the decode kernel ms (HIP events).  Repeated
over `pairs` context pairs.  One JSON line; the launch order is printed with it so rocprofv3
per-dispatch counters (tools/gpu_r6_decode_size.sh) map to (pair, phase, step)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from netgauze_amd import synth
    from netgauze_amd.flow import FlowInfoCodec, OPT_PLACE_TRIALS
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    nb, ns = 100_000_000, 12_500_000
    big = synth.stream_range(nb, 0, len(synth.stream_index(nb)[2]), None, device=dev)[:3]
    small = synth.stream_range(ns, 0, len(synth.stream_index(ns)[2]), None, device=dev)[:3]
    tm = [synth.template_message()]
    out, order = {}, []

    def run(codec, batch, tag):
        ms = []
        for _ in range(steps):
            codec.decode_batch(*batch)
            ms.append(round(codec.last_timing()[0], 4))
        out[tag] = ms
        order.append((tag, steps))

    for p in range(pairs):
        a = FlowInfoCodec(0, rtc_sync=True, options={OPT_PLACE_TRIALS: 1})
        a.decode_datagrams(tm)
        run(a, small, "p%d_fresh_1.25e7" % p)
        b = FlowInfoCodec(0, rtc_sync=True, options={OPT_PLACE_TRIALS: 1})
        b.decode_datagrams(tm)
        run(b, big, "p%d_big_1e8" % p)
        run(b, small, "p%d_sub_1.25e7" % p)
        a.close()
        b.close()
        torch.cuda.synchronize()
    print(json.dumps({"steps_ms": out, "launch_order": order,
                      "alg_bytes": {"1e8": 127 * nb, "1.25e7": 127 * ns}}))


if __name__ == "__main__":
    main()

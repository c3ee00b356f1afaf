#!/usr/bin/env python3
"""Round 6 arena experiment: per-step decode time of 10^8 T20 records on one context without
placement trials (NGZ_OPT_PLACE_TRIALS 1), to tell a fresh allocation's transient (the first steps
slow, later ones fast) from an allocation-lifetime mode (every step slow).  Optionally reallocates
the arena mid-run (a second context) to see a fresh allocation again.  Prints one JSON line."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from netgauze_amd import synth
    from netgauze_amd.flow import FlowInfoCodec, OPT_PLACE_TRIALS
    dev = torch.device("cuda", 0)
    n = 100_000_000
    buf, offs, lens, _ = synth.stream_range(n, 0, len(synth.stream_index(n)[2]), None, device=dev)
    out = {}
    for run in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        codec = FlowInfoCodec(0, rtc_sync=True, options={OPT_PLACE_TRIALS: 1})
        codec.decode_datagrams([synth.template_message()])
        ms = []
        for _ in range(30):
            codec.decode_batch(buf, offs, lens)
            ms.append(round(codec.last_timing()[0], 3))
        out["ctx%d" % run] = ms
        codec.close()
        del codec
        torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Decode time vs column spacing (NGZ_OPT_CAP_PAD windows of 1024 rows) on
one arena, for a few contexts (arenas)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netgauze_amd import synth
from netgauze_amd.flow import FlowInfoCodec

dev = torch.device("cuda", 0)
n = 50_000_000
rec = synth.t20_records(n, seed=synth.SEED_CFG2, device=dev, first=0)
buf, offs, lens = synth.ipfix_data_stream(rec, 64)
del rec
keep = []
pads = [int(x) for x in os.environ.get("PADS", "0 1 2 3 4 5 7 8 16 31 32 64").split()]
for c in range(4):
    codec = FlowInfoCodec(0)
    codec.decode_datagrams([synth.template_message()])
    codec.set_option(4, max(pads))  # grow the arena once, for the largest spacing
    codec.decode_batch(buf, offs, lens)
    line = []
    for pad in pads:
        codec.set_option(4, pad)
        ts = []
        for _ in range(3):
            codec.decode_batch(buf, offs, lens)
            ts.append(codec.last_timing()[0])
        line.append("%d:%.3f" % (pad, min(ts)))
    print("ctx %d: %s" % (c, " ".join(line)), flush=True)
    keep.append(codec)

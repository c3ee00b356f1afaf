#!/usr/bin/env python3
"""Decode time vs the arena offset of the column blocks (same context, same input)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netgauze_amd import synth
from netgauze_amd.flow import FlowInfoCodec

dev = torch.device("cuda", 0)
n = 100_000_000
rec = synth.t20_records(n, seed=synth.SEED_CFG2, device=dev, first=0)
buf, offs, lens = synth.ipfix_data_stream(rec, 64)
del rec
for ctxi in range(3):
    codec = FlowInfoCodec(0)
    codec.decode_datagrams([synth.template_message()])
    line = []
    for k in list(range(12)) + [0]:
        shift = int(sys.argv[1]) * k if len(sys.argv) > 1 else (2 << 20) * k
        codec.set_option(3, shift)
        ts = []
        for _ in range(3):
            codec.decode_batch(buf, offs, lens)
            ts.append(codec.last_timing()[0])
        line.append("%.3f" % min(ts))
    print("ctx %d: %s" % (ctxi, " ".join(line)), flush=True)
    del codec

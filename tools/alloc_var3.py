#!/usr/bin/env python3
"""Which allocation decides the slow mode?  For 4 input placements, decode
with 6 fresh contexts each (earlier contexts kept alive, so every arena lands
on new memory): per input, the good/bad pattern over arenas."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netgauze_amd import synth
from netgauze_amd.flow import FlowInfoCodec

dev = torch.device("cuda", 0)
n = 50_000_000
keep = []
for place in range(int(os.environ.get("PLACES", "4"))):
    rec = synth.t20_records(n, seed=synth.SEED_CFG2, device=dev, first=0)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64)
    del rec
    line = []
    for k in range(6):
        codec = FlowInfoCodec(0)
        codec.decode_datagrams([synth.template_message()])
        ts = []
        for _ in range(3):
            codec.decode_batch(buf, offs, lens)
            ts.append(codec.last_timing()[0])
        line.append("%.3f" % min(ts))
        keep.append(codec)
    print("input %d: %s" % (place, " ".join(line)), flush=True)
    keep.append(buf)

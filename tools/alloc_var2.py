#!/usr/bin/env python3
"""Placement sensitivity vs decode grid: for several input placements, the
decode kernel time at NGZ_LDS_BLOCKS_PER_CU = 1, 2, 4, 8 (fresh context each)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from netgauze_amd import synth
from netgauze_amd.flow import FlowInfoCodec

dev = torch.device("cuda", 0)
n = 100_000_000
pads = []
for place in range(4):
    rec = synth.t20_records(n, seed=synth.SEED_CFG2, device=dev, first=0)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64)
    del rec
    line = []
    for bpc in (1, 2, 4, 8, 16):
        os.environ["NGZ_LDS_BLOCKS_PER_CU"] = str(bpc)
        codec = FlowInfoCodec(0)
        codec.decode_datagrams([synth.template_message()])
        ts = []
        for _ in range(3):
            codec.decode_batch(buf, offs, lens)
            ts.append(codec.last_timing()[0])
        line.append("bpc %d: %.3f" % (bpc, min(ts)))
        del codec
    print("input 0x%x | %s" % (buf.data_ptr(), " | ".join(line)), flush=True)
    del buf, offs, lens
    torch.cuda.empty_cache()
    pads.append(torch.empty((place * 97 + 11) << 20, dtype=torch.uint8, device=dev))

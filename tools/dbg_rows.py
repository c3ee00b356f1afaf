"""Debug helper (GPU box): decode a T20 stream and list mismatching rows per column."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from netgauze_amd import synth
from netgauze_amd.flow import FlowInfoCodec

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
rpm = int(sys.argv[2]) if len(sys.argv) > 2 else 1023
rec = synth.t20_records(n, seed=synth.SEED_CFG2)
buf, offs, lens = synth.ipfix_data_stream(rec, 64, rec_per_msg=rpm)
b = bytes(buf.numpy())
dg = [synth.template_message()] + [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]
codec = FlowInfoCodec(0)
batch = codec.decode_datagrams(dg)
slot = batch.slots[0]
raw = rec.numpy().reshape(n, 64)
for f, fi in enumerate(slot.fields):
    col = np.asarray(slot.column_bytes(f))[:n]
    off, ln = fi.wire_offset, fi.wire_length
    exp = raw[:, off:off + ln][:, ::-1]
    w = col.shape[1]
    e = np.zeros((n, w), np.uint8)
    e[:, :min(w, ln)] = exp[:, :min(w, ln)]
    bad = np.nonzero((col != e).any(axis=1))[0]
    if len(bad):
        print("field", f, "off", off, "len", ln, "bad rows", len(bad), bad[:20], "...", bad[-5:])
print("done")

"""Config-4 framing split by protocol (not product code): the config-4 batch of bench.py, and its
NetFlow v9 datagrams alone and its IPFIX (variable-length template 900) datagrams alone, each decoded
STEPS times on one context.  Run under `rocprofv3 --kernel-trace` to see what k_frame / k_emit /
the decode kernels cost per protocol.  usage: python tools/frame_probe.py [records] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from netgauze_amd import synth  # noqa: E402
from netgauze_amd.flow import FlowInfoCodec  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    dg = synth.cfg4_datagrams(n, seed=synth.SEED_CFG4)
    data = dg[2:]
    parts = {"all": data, "nfv9": [d for d in data if d[1] == 9], "ipfix": [d for d in data if d[1] == 10]}
    for name, part in parts.items():
        codec = FlowInfoCodec(0, rtc_sync=True)
        codec.decode_datagrams(dg[:2])
        buf, offs, lens = synth.host_batch(part, device=dev)
        torch.cuda.synchronize()
        ms = []
        for _ in range(steps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            b = codec.decode_batch(buf, offs, lens)
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        print("%-6s datagrams %8d records %9d  step %.3f ms (min of %d)" % (name, len(part), b.n_records,
                                                                           min(ms[1:]), steps), flush=True)
        codec.close()
        del buf, offs, lens


if __name__ == "__main__":
    main()

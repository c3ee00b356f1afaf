#!/usr/bin/env python3
"""PCIe probe on one GPU: pinned host -> device, device -> pinned host, and both at once on two
streams (duplex), for the host-to-host decode path (bench.py --e2e).  Prints one JSON line.
usage: python tools/pcie_probe.py [--mb 640] [--reps 5]"""
import argparse
import json
import os
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=640)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    n = a.mb << 20
    dev = torch.device("cuda", 0)
    h_src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(n, dtype=torch.uint8, device=dev)
    d_b = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return best

    def h2d():
        with torch.cuda.stream(s1):
            d_a.copy_(h_src, non_blocking=True)

    def d2h():
        with torch.cuda.stream(s2):
            h_dst.copy_(d_b, non_blocking=True)

    def both():
        h2d()
        d2h()

    def h2d_split(k=4):
        # the same bytes as k copies on alternating streams (do several engines take one direction?)
        c = n // k
        for i in range(k):
            with torch.cuda.stream(s1 if i % 2 == 0 else s2):
                d_a[i * c:(i + 1) * c].copy_(h_src[i * c:(i + 1) * c], non_blocking=True)

    ss = [torch.cuda.Stream(dev) for _ in range(4)]

    def both_four(k=8):
        # both directions cut in k pieces over four streams (does the runtime spread them over engines?)
        c = n // k
        for i in range(k):
            with torch.cuda.stream(ss[i % 4]):
                if i % 2 == 0:
                    d_a[i * c:(i + 1) * c].copy_(h_src[i * c:(i + 1) * c], non_blocking=True)
                    d_a[(i + 1) * c:(i + 2) * c].copy_(h_src[(i + 1) * c:(i + 2) * c], non_blocking=True)
                else:
                    h_dst[(i - 1) * c:i * c].copy_(d_b[(i - 1) * c:i * c], non_blocking=True)
                    h_dst[i * c:(i + 1) * c].copy_(d_b[i * c:(i + 1) * c], non_blocking=True)

    t1, t2, t3, t4, t5 = timed(h2d), timed(d2h), timed(both), timed(h2d_split), timed(both_four)
    gb = n / 1e9
    print(json.dumps({"bytes": n, "h2d_gbps": gb / t1, "d2h_gbps": gb / t2, "duplex_gbps": 2 * gb / t3,
                      "duplex_ms": t3 * 1e3, "h2d_ms": t1 * 1e3, "d2h_ms": t2 * 1e3,
                      "h2d_two_streams_gbps": gb / t4, "duplex_four_streams_gbps": 2 * gb / t5,
                      "HSA_ENABLE_SDMA": os.environ.get("HSA_ENABLE_SDMA")}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Table of the configs 3 / 5 experiment (tools/gpu_r6_decode_size.sh output dir): per (pair, phase)
the decode kernel's traced duration, fraction of the 8 TB/s peak for 127 B per record, DRAM read /
write credit stalls per microsecond (TCC pass) and the share of wave cycles waiting on memory / on
issue (SQ pass).  Dispatch order is the launch order printed by tools/decode_size.py.
usage: decode_size_table.py DIR"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_dispatch  # noqa: E402


def phases(order):
    out, i = [], 0
    for tag, n in order:
        out.append((tag, list(range(i, i + n))))
        i += n
    return out


def main():
    d = sys.argv[1]
    import re
    rx = re.compile("ngz_tpl")
    plain = json.load(open(os.path.join(d, "plain.json")))
    tcc = pmc_dispatch.load(os.path.join(d, "p1"), rx)
    sq = pmc_dispatch.load(os.path.join(d, "p2"), rx)
    order = json.load(open(os.path.join(d, "p1.json")))["launch_order"]
    print("configs 3 / 5 experiment: T20 decode at 1.25e7 records on a fresh 1.25e7-row arena ('fresh') and")
    print("into the first eighth of a 1e8-row arena that just decoded 1e8 ('sub'; column stride 1.25e7 rows")
    print("either way), and the 1e8 decode itself ('big').  Placement trials off: each arena shows its mode.")
    print()
    print("1. HIP-event decode ms per step, no profiler (plain.json):")
    for tag, ms in plain["steps_ms"].items():
        n = 1e8 if "1e8" in tag else 1.25e7
        med = statistics.median(ms)
        print("   %-18s median %.4f ms  frac %.3f   %s" % (tag, med, 127 * n / med / 1e6 / 8000, ms))
    print()
    print("2. Per dispatch, profiled runs (kernel-trace duration beside counters; TCC and SQ are two runs,")
    print("   each with its own arenas, so a phase's mode can differ between them):")
    print("   %-18s %9s %6s %12s %12s | %9s %6s %7s %7s" % ("phase", "us(TCC)", "frac", "rd_stall/us", "wr_stall/us",
                                                          "us(SQ)", "frac", "wait%", "winst%"))
    for tag, ids in phases(order):
        n = 1e8 if "1e8" in tag else 1.25e7
        t_us = statistics.median(tcc[i][0] for i in ids)
        rd = statistics.median(tcc[i][1].get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", 0) / tcc[i][0] for i in ids)
        wr = statistics.median(tcc[i][1].get("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", 0) / tcc[i][0] for i in ids)
        s_us = statistics.median(sq[i][0] for i in ids)
        wa = statistics.median(sq[i][1]["SQ_WAIT_ANY"] / sq[i][1]["SQ_WAVE_CYCLES"] for i in ids)
        wi = statistics.median(sq[i][1]["SQ_WAIT_INST_ANY"] / sq[i][1]["SQ_WAVE_CYCLES"] for i in ids)
        f = lambda us: 127 * n / (us / 1e3) / 1e6 / 8000  # noqa: E731
        print("   %-18s %9.1f %6.3f %12.0f %12.0f | %9.1f %6.3f %7.1f %7.1f" % (tag, t_us, f(t_us), rd, wr, s_us, f(s_us),
                                                                         100 * wa, 100 * wi))


if __name__ == "__main__":
    main()

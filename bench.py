#!/usr/bin/env python3
"""Benchmark: device-resident IPFIX T20 data-record decode on MI355X.

One step = one ngz_decode_batch over a batch of synthetic IPFIX datagrams
already resident in HBM (1023 x 64-byte T20 records per 65,492-byte message;
the T20 template was learnt by the context before timing, like a running
collector): framing, record counting/layout and the LDS-staged columnar
decode kernel, ending with the library's own stream sync.  Multi-GPU: one
process per GPU, each decodes its own shard (weak scaling) and the
per-template processed counts are all-gathered over RCCL after every step.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BYTES_PER_RECORD_IN = 64
BYTES_PER_RECORD_OUT = 63  # T20 canonical columns
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec


def cpu_threads():
    """Threads for the CPU baseline: the CPUs this process may run on
    (sched_getaffinity), capped by OMP_NUM_THREADS when set (the GPU box sets
    it to the box's CPU share, 16 per GPU, while nproc shows the whole
    machine)."""
    affinity = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(affinity, cap) if cap > 0 else affinity), affinity


def cpu_sample(workload, n):
    """Host sample of the workload's stream: (template messages, bytes, offsets, lengths, description)."""
    import numpy as np
    from netgauze_amd import synth
    if workload == "t20":
        rec = synth.t20_records(n, seed=synth.SEED_CFG2)
        buf, offs, lens = synth.ipfix_data_stream(rec, 64)
        return [synth.template_message()], buf.numpy(), offs.numpy(), lens.numpy(), "T20"
    if workload in ("mixed8", "cfg5"):
        tpls = synth.CFG3_TEMPLATES if workload == "mixed8" else synth.CFG5_TEMPLATES
        seed = synth.SEED_CFG3 if workload == "mixed8" else synth.SEED_CFG5
        buf, offs, lens, _ = synth.mixed_stream(n, templates=tpls, seed=seed)
        return [synth.templates_message(tpls)], buf.numpy(), offs.numpy(), lens.numpy(), \
            "%d templates, interleaved" % len(tpls)
    dg = synth.cfg4_datagrams(n, seed=synth.SEED_CFG4)
    lens = np.array([len(d) for d in dg[2:]], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1], dtype=np.uint64)]).astype(np.uint64)
    return dg[:2], np.frombuffer(b"".join(dg[2:]), dtype=np.uint8), offs, lens, "NFv9 313 + IPFIX vlen 900, MTU packets"


def cpu_baseline(workload="t20", seconds_budget=10.0, single_budget=4.0):
    """The reference algorithm's restatement (oracle/cpu/ngz_cpu.c: record at
    a time, one heap-allocated field array per record, per-field dispatch;
    IPFIX and NetFlow v9) timed on this host's cores, one independent codec per
    thread over a contiguous message range (one exporter peer per thread), plus
    the same on one core.  A bounded sample of the workload, repeated for about
    seconds_budget (all cores) + single_budget (one core)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_port
    threads, affinity = cpu_threads()
    sample = {"t20": 4_000_000, "mixed8": 2_000_000, "cfg5": 2_000_000, "cfg4": 1_000_000}[workload]
    tm, b, o, ln, desc = cpu_sample(workload, sample)
    sb, so, sl, n_pre = cpu_port.stream(tm, b, o, ln)

    def timed(th, budget):
        n = reps = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget:
            got, _, err = cpu_port.decode_stream(sb, so, sl, n_pre, threads=th)
            assert err == 0 and got == sample, (got, err)
            n += got
            reps += 1
        dt = time.perf_counter() - t0
        return n / dt, reps, dt

    v, reps, dt = timed(threads, seconds_budget)
    v1, reps1, dt1 = timed(1, single_budget)
    return {"value": v, "unit": "records/s", "cores": threads, "kind": "port",
            "single_core": v1, "nproc": os.cpu_count(), "affinity": affinity,
            "sample": "%d x %d records (%s; %d messages) through oracle/cpu/ngz_cpu.c, a C restatement of the "
                      "reference decode (Rust reference not buildable here): %d threads (CPUs in this process's "
                      "affinity: %d, capped by OMP_NUM_THREADS; nproc %d) for %.1f s, then 1 thread %d x for %.1f s"
                      % (reps, sample, desc, len(o), threads, affinity, os.cpu_count(), dt, reps1, dt1)}


def committed_traffic(records, workload):
    """Per-launch HBM bytes of the decode kernel from a committed rocprofv3 PMC
    profile of this same workload (profiles/**/traffic.json at any depth, written
    by tools/summarize_profile.py) taken of THIS build's decode sources (their
    hash, netgauze_amd/buildinfo.decode_source_hash), or None: a profile of an
    older decode build is never reported as this build's traffic.  The newest
    matching profile (by path: profiles/<round><letter>/...) wins."""
    import glob
    from netgauze_amd import buildinfo
    want, whole = buildinfo.decode_source_hash(), buildinfo.source_hash()
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "traffic.json"), recursive=True)):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if t.get("records") == records and t.get("workload") == workload and \
                (t.get("decode_source_hash") == want or t.get("source_hash") == whole):
            best = (t["traffic_bytes"], os.path.relpath(f, ROOT))
    return best


def committed_agg_traffic(key, workload):
    """Per-push HBM bytes of one aggregation key from a committed profile
    (profiles/**/agg_KEY/traffic.json, tools/summarize_agg_profile.py) of THIS
    tree's aggregation sources (buildinfo.agg_source_hash), or None."""
    import glob
    from netgauze_amd import buildinfo
    want = buildinfo.agg_source_hash()
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "agg_%s" % key, "traffic.json"), recursive=True)):
        try:
            t = json.load(open(f))
        except (OSError, ValueError):
            continue
        if t.get("workload") == workload and t.get("agg_source_hash") == want:
            best = (t["traffic_bytes"], os.path.relpath(f, ROOT))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--records", type=int, default=None,
                    help="records per GPU (default 10^8; cfg5: 1.25*10^8, i.e. 10^9 over 8 GPUs)")
    ap.add_argument("--workload", choices=["t20", "mixed8", "cfg4", "cfg5"], default="t20",
                    help="t20 (headline): one 20-field 64-B template; mixed8: config 3, 8 reference-shaped "
                         "templates (40-153 B) in interleaved messages; cfg4: config 4, NetFlow v9 + IPFIX "
                         "variable-length/enterprise IEs; cfg5: config 5, 16 templates (config 3 + 8 width "
                         "permutations), one shard per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--split", action="store_true",
                    help="split framing (NGZ_OPT_SPLIT: variable-length record walks on a second stream)")
    ap.add_argument("--place-probe", type=int, choices=[0, 1, 2], default=0,
                    help="NGZ_OPT_PLACE_PROBE: arena placement trials timed by the batch's decode (0), by a probe "
                         "of the decode's memory streams (1), or both with the decodes deciding (2)")
    ap.add_argument("--contexts", type=int, default=1,
                    help="decode contexts in flight (one host thread and HIP stream each, the steps dealt round "
                         "robin): batch k+1's framing overlaps batch k's decode")
    ap.add_argument("--submit", action="store_true",
                    help="with --contexts P: one host thread keeps the P contexts' batches in flight through "
                         "ngz_decode_batch_submit / ngz_decode_batch_wait instead of a thread per context")
    ap.add_argument("--e2e-contexts", type=int, default=3, help="--e2e: contexts (host threads) in flight")
    ap.add_argument("--e2e-ranges", type=int, default=12, help="--e2e: message ranges per batch")
    ap.add_argument("--e2e-duplex-contexts", type=int, default=6, help="--e2e duplex modes: contexts")
    ap.add_argument("--e2e-duplex-ranges", type=int, default=24, help="--e2e duplex modes: message ranges")
    ap.add_argument("--e2e", action="store_true",
                    help="host-to-host rate instead: pinned host datagrams -> H2D -> decode -> D2H of all columns")
    ap.add_argument("--agg", choices=["proto_dir", "dport", "5tuple"], default=None,
                    help="device flow aggregation of decoded T20 columns instead (include/ngz/flow_aggregate.h): "
                         "key protocol+flowDirection (6 groups/window), protocol+dport (~2e5) or the 5-tuple "
                         "(~1 group per record); 7 aggregated fields")
    ap.add_argument("--agg-max-peers", type=int, default=256, help="--agg: the aggregator's max_peers")
    args = ap.parse_args()
    if args.agg:
        return main_agg(args)
    if args.records is None:
        args.records = 125_000_000 if args.workload == "cfg5" else 100_000_000
    if args.e2e:
        return main_e2e(args)

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; on a box with fewer GPUs than ranks (a rehearsal of
    # the multi-rank path) ranks share devices round robin
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # "nccl" is RCCL on ROCm (over xGMI between the GPUs of a node); NGZ_DIST_BACKEND=gloo
        # rehearses the multi-rank path where ranks share one GPU
        dist.init_process_group(os.environ.get("NGZ_DIST_BACKEND", "nccl"), init_method="env://")

    from netgauze_amd import synth
    from netgauze_amd.flow import FlowInfoCodec

    dev = torch.device("cuda", local)
    cdev = dev if dist is None or dist.get_backend() == "nccl" else torch.device("cpu")  # collective tensors
    from netgauze_amd.flow import OPT_PLACE_PROBE, OPT_SPLIT
    copts = {OPT_SPLIT: 1} if args.split else {}
    popts = dict(copts)
    if args.place_probe:
        popts[OPT_PLACE_PROBE] = args.place_probe
    codec = FlowInfoCodec(local, rtc_sync=True, options=popts)  # template kernels compiled when learnt
    n = args.records
    learnt = []  # the template messages every context learns before timing
    from netgauze_amd import dist as ndist
    n_rank = n  # records this rank decodes per step
    if args.workload in ("t20", "mixed8", "cfg5"):
        # one stream of n * world records: its message index (records per message, no
        # bytes) is cut into contiguous ranges balanced by records, and each rank builds only its
        # range -- byte for byte the messages the whole stream has there
        tpls = None if args.workload == "t20" else \
            synth.CFG3_TEMPLATES if args.workload == "mixed8" else synth.CFG5_TEMPLATES
        seed = {"t20": synth.SEED_CFG2, "mixed8": synth.SEED_CFG3, "cfg5": synth.SEED_CFG5}[args.workload]
        learnt = [synth.template_message() if tpls is None else synth.templates_message(tpls)]
        codec.decode_datagrams(learnt)  # the exporter's templates, learnt before timing
        _, _, per_msg = synth.stream_index(n * world, tpls)
        m0, m1 = ndist.shard_by_records(per_msg, rank, world)
        buf, offs, lens, n_rank = synth.stream_range(n * world, m0, m1, tpls, seed=seed, device=dev)
        if os.environ.get("NGZ_BENCH_INPUT_MB"):  # experiment: the batch at the start of a larger allocation
            big = torch.empty(max(buf.numel(), int(os.environ["NGZ_BENCH_INPUT_MB"]) << 20), dtype=torch.uint8, device=dev)
            big[:buf.numel()].copy_(buf)
            buf = big[:buf.numel()]
        rec_bytes = {256: 64} if tpls is None else {tid: synth.field_offsets(f)[1] for tid, f in tpls}
    else:
        dg = synth.cfg4_datagrams(n, seed=synth.SEED_CFG4 + 16 * rank)
        learnt = dg[:2]
        codec.decode_datagrams(learnt)  # the NFv9 and IPFIX templates
        buf, offs, lens = synth.host_batch(dg[2:], device=dev)
        rec_bytes = None  # variable: the data bytes of the batch stand in for record bytes
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev).cuda_stream

    # templates.usage: per step, both protocols' processed counts -> one device table
    # (ngz_template_counts_device, stream-ordered) -> one RCCL all-gather; no host sync
    exchange = ndist.CountExchange(codec, stream=stream) if dist is not None else None

    def step():
        batch = codec.decode_batch(buf, offs, lens, stream=stream)
        if exchange is not None:
            exchange.step(reset=True)
        return batch

    # --contexts P > 1: P codecs (contexts) on P streams, each driven by its own host thread (the
    # decode call blocks its thread until its batch is framed and decoded; ctypes releases the GIL)
    P = max(1, args.contexts)
    assert P == 1 or exchange is None, "--contexts > 1 is a single-rank measurement"
    extra = []
    for _ in range(P - 1):
        c = FlowInfoCodec(local, rtc_sync=True, options=copts)
        c.decode_datagrams(learnt)
        extra.append((c, torch.cuda.Stream(dev).cuda_stream))
    ctxs = [(codec, stream)] + extra

    for _ in range(max(1, args.warmup)):  # (one untimed step even at --warmup 0: it sizes the roofline bytes)
        b = step()
        for c, st in extra:
            c.decode_batch(buf, offs, lens, stream=st)
    # (experiment builds may be timing-attribution variants whose output is wrong by design)
    assert b.n_records == n_rank or os.environ.get("NGZ_EXPERIMENTS", "0") not in ("", "0", "1"), (b.n_records, n_rank)
    # algorithmic bytes per launch: wire bytes read + canonical column bytes written, per template
    if rec_bytes is not None:
        read_bytes = sum(s.n_records * rec_bytes[s.template_id] for s in b.slots if s.n_records)
    else:
        read_bytes = int(lens.sum())  # every datagram byte (headers are < 1 %)
    alg_bytes = read_bytes + sum(s.n_records * sum(f.width for f in s.fields) for s in b.slots if s.n_records)
    dec_ms = []
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if P == 1:
        for _ in range(args.steps):
            step()
            dec_ms.append(codec.last_timing()[0])
    elif args.submit:
        # one host thread: step k goes to context k % P once that context's previous batch is collected
        pending = [False] * P
        for k in range(args.steps):
            c, st = ctxs[k % P]
            if pending[k % P]:
                c.decode_batch_wait()
                dec_ms.append(c.last_timing()[0])
            c.decode_batch_submit(buf, offs, lens, stream=st)
            pending[k % P] = True
        for i, (c, st) in enumerate(ctxs):
            if pending[i]:
                c.decode_batch_wait()
                dec_ms.append(c.last_timing()[0])
    else:
        import threading

        def drive(i):
            c, st = ctxs[i]
            for _ in range(i, args.steps, P):
                c.decode_batch(buf, offs, lens, stream=st)
                dec_ms.append(c.last_timing()[0])

        th = [threading.Thread(target=drive, args=(i,)) for i in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    usage = None
    if exchange is not None:
        # the last step's node-wide counts: every record of every rank, once (one data set per message
        # for the fixed-template workloads: +1 per IPFIX set, ipfix.rs:223; +1 per NFv9 record, netflow.rs:218)
        tot, fitted = exchange.totals()
        usage = {"templates": len(tot), "fitted": fitted, "total_count": sum(tot.values())}
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    # t20 / mixed8 / cfg5: the ranks' ranges partition one stream of n * world records; cfg4: a
    # stream of n records per rank
    total_records = n * world * args.steps
    value = total_records / elapsed
    dec_avg = sum(dec_ms) / len(dec_ms)
    achieved = alg_bytes / (dec_avg * 1e-3) / 1e9
    workload_desc = {"t20": "T20 x %d records/GPU, 1023 records per 65,492-byte IPFIX message" % n,
                     "mixed8": "config 3: %d records/GPU over templates %s, interleaved messages"
                     % (n, ",".join(str(t) for t, _ in synth.CFG3_TEMPLATES)),
                     "cfg5": "config 5: %d records/GPU (10^9 at 8 GPUs) over 16 templates %s"
                     % (n, ",".join(str(t) for t, _ in synth.CFG5_TEMPLATES)),
                     "cfg4": "config 4: %d records/GPU, NFv9 template 313 (130 B, 10/packet) + IPFIX "
                             "template 900 (vlen strings/octets, VMware/Huawei IEs)" % n}[args.workload]
    traffic = committed_traffic(n, workload_desc)
    # the arena placement lottery of the first large batch (ngz_placement_trials): every trial's
    # decode time, the kept one, and the fraction the median trial would have reached
    trials, kept, probes = codec.placement_trials(probes=True)
    placement = None
    if trials:
        med = sorted(trials)[len(trials) // 2]
        placement = {"placement_trials_ms": trials, "placement_kept": kept,
                     "placement_median_frac": alg_bytes / (med * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "placement_best_frac": alg_bytes / (min(trials) * 1e-3) / 1e9 / HBM_PEAK_GBS}
    if any(probes):
        placement = dict(placement or {}, placement_probe_ms=probes, placement_kept=kept)
    out = {
        "metric": {"t20": "IPFIX flow records/sec + GB/s (device-resident), 20-field fixed template",
                   "mixed8": "IPFIX flow records/sec (device-resident), config 3: 8 templates",
                   "cfg5": "IPFIX flow records/sec (device-resident), config 5: 16 templates, sharded per GPU",
                   "cfg4": "flow records/sec (device-resident), config 4: NetFlow v9 + IPFIX variable-length"}
                  [args.workload],
        "value": value,
        "unit": "records/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic (splitmix64 records, seed 0x4E475A4500000004+16*rank, a stream per rank)"
                 if args.workload == "cfg4" else
                 "synthetic (splitmix64 records, seed 0x4E475A450000000%d): one stream of %d records, each rank "
                 "decodes its record-balanced message range (this rank: %d)"
                 % ({"t20": 2, "mixed8": 3, "cfg5": 5}[args.workload], n * world, n_rank)),
        "config": {"workload": workload_desc,
                   "records_per_gpu": n, "messages_per_gpu": int(offs.numel()),
                   "parallelism": ("record-balanced message ranges of one stream, one per GPU"
                                   if args.workload != "cfg4" else "a stream per GPU") if world > 1 else "single",
                   **({"contexts": P} if P > 1 else {}), **({"one_thread_submit": True} if P > 1 and args.submit else {}), **({"split_framing": True} if args.split else {})},
        "gbps_step": alg_bytes * world * args.steps / elapsed / 1e9,
        "templates_usage_exchange": usage,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic[0] if traffic else None,
                     "traffic_src": traffic[1] if traffic else None,
                     "kernel": "ngz_tpl (per-template decode kernels)", "kernel_ms": dec_avg,
                     "alg_bytes_per_launch": alg_bytes,
                     "read_gbps": read_bytes / (dec_avg * 1e-3) / 1e9, **(placement or {})},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.workload)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main_agg(args):
    """Aggregation throughput: T20 records decoded once into HBM, then pushed through the
    device FlowAggregator every step (explode + reduce of every record into the HBM group
    table); export times restamped so the batch spans two minute windows."""
    import torch
    from netgauze_amd import synth
    from netgauze_amd.aggregate import FlowAggregator
    from netgauze_amd.flow import FlowInfoCodec
    n = args.records or 100_000_000
    dev = torch.device("cuda", 0)
    codec = FlowInfoCodec(0, rtc_sync=True)
    codec.decode_datagrams([synth.template_message()])
    rec = synth.t20_records(n, device=dev)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64)
    del rec
    m = torch.arange(offs.numel(), device=dev, dtype=torch.int64)
    t = 1_700_000_010 + (m * 60) // offs.numel()  # export times 1_700_000_010 .. +59: windows ..1_699_999_980 and ..040
    for b in range(4):
        buf[offs + 4 + b] = ((t >> (8 * (3 - b))) & 0xFF).to(torch.uint8)
    keys = {"proto_dir": [(0, 4, 0, 0), (0, 61, 0, 0)], "dport": [(0, 4, 0, 0), (0, 11, 0, 0)],
            "5tuple": [(0, 8, 0, 0), (0, 12, 0, 0), (0, 7, 0, 0), (0, 11, 0, 0), (0, 4, 0, 0)]}[args.agg]
    vals = [(0, 1, 0, 1), (0, 2, 0, 1), (0, 6, 0, 4), (0, 22, 0, 2), (0, 21, 0, 3), (0, 16, 0, 3), (0, 10, 0, 2)]
    col_bytes = {4: 1, 61: 1, 11: 2, 7: 2, 8: 4, 12: 4, 1: 8, 2: 8, 6: 1, 22: 4, 21: 4, 16: 4, 10: 4}
    per_rec = sum(col_bytes[f[1]] for f in keys + vals)
    cap = {"proto_dir": 1 << 10, "dport": 1 << 20, "5tuple": n}[args.agg]
    # lateness = the window: the same batch pushed again is not late (its export times are
    # within 60 s of the event time), so every step aggregates every record
    agg = FlowAggregator(keys + vals, capacity=cap, lateness_s=60, max_peers=args.agg_max_peers)
    batch = codec.decode_batch(buf, offs, lens)
    assert batch.n_records == n
    # the first push creates every group (slot claims, key writes); the timed steps then
    # reduce into the existing groups: steady state, as a collector's windows see it
    assert agg.push(batch, 4739, 0) == 0
    first_push_ms = agg.push_ms()
    for _ in range(args.warmup):
        assert agg.push(batch, 4739, 0) == 0
    groups = agg.n_groups()
    torch.cuda.synchronize()
    push_ms = []
    t0 = time.perf_counter()
    late = 0
    for _ in range(args.steps):
        late += agg.push(batch, 4739, 0)
        push_ms.append(agg.push_ms())
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    avg = sum(push_ms) / len(push_ms)
    alg = per_rec * n
    workload = "aggregate %d T20 records, %d key fields + %d aggregated fields, 2 minute windows" % (
        n, len(keys), len(vals))
    traffic = committed_agg_traffic(args.agg, workload)
    print(json.dumps({
        "metric": "flow records aggregated/sec (device-resident decoded columns), T20, key %s" % args.agg,
        "value": n * args.steps / elapsed, "unit": "records/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic T20 (seed 0x4E475A4500000002)",
        "config": {"workload": workload, "records": n, "groups": groups, "table_capacity": cap,
                   "late_records": late, "first_push_ms": first_push_ms},
        "push_kernels_ms": avg, "push_records_per_s": n / (avg * 1e-3), "path": agg.last_path(),
        "roofline": {"bound": "hbm (atomic-throughput limited)", "achieved": alg / (avg * 1e-3) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": traffic[0] if traffic else None, "traffic_src": traffic[1] if traffic else None,
                     "alg_bytes_per_launch": alg, "alg_bytes_per_record": per_rec}}), flush=True)


def main_e2e(args):
    """Host-resident path (north star: UDP/PCAP -> decoded record arrays in host
    memory): the batch sits in pinned host memory, ngz_decode_batch_host copies
    it H2D, decodes, and every column block is copied back D2H
    (ngz_columns_to_host).  Three rates: one context doing whole batches in turn
    (serial: H2D, decode, D2H never overlap); the batch cut into message ranges
    decoded by --e2e-contexts contexts (one per exporter peer, as the collector
    runs them) from their own host threads and HIP streams ("threads"); and the
    same ranges from one host thread with the H2D of the next range and the D2H
    of the previous one queued on two streams around each decode, so PCIe
    carries both directions at once ("duplex"), and the same with the D2H
    stored by a kernel ("duplex_kernel").  The line's value is the fastest
    mode, named in config.mode.  Reported in DESIGN.md; never the headline
    value."""
    import threading

    import torch
    from netgauze_amd import synth
    from netgauze_amd.flow import FlowInfoCodec
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    n = args.records
    rec = synth.t20_records(n, seed=synth.SEED_CFG2, device=dev, first=0)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64)
    del rec
    hb = torch.empty(buf.numel(), dtype=torch.uint8, pin_memory=True)
    hb.copy_(buf)
    ho = torch.empty(offs.numel(), dtype=torch.int64, pin_memory=True)
    ho.copy_(offs)
    hl = torch.empty(lens.numel(), dtype=torch.int32, pin_memory=True)
    hl.copy_(lens)
    del buf, offs, lens
    torch.cuda.synchronize()
    tm = synth.template_message()

    def timed(step):
        for _ in range(args.warmup):
            step()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            moved = step()
        return (time.perf_counter() - t0) / args.steps, moved

    # serial: one context, the whole batch per step
    codec = FlowInfoCodec(0, rtc_sync=True)
    codec.decode_datagrams([tm])
    out = torch.empty(n * BYTES_PER_RECORD_OUT + (4 << 20), dtype=torch.uint8, pin_memory=True)

    def serial():
        b = codec.decode_host_buffers(hb.data_ptr(), hb.numel(), ho.data_ptr(), hl.data_ptr(), ho.numel())
        assert b.n_records == n
        return codec.columns_to_host(out.data_ptr(), out.numel())

    t_serial, moved = timed(serial)
    del codec

    # pipelined: message ranges over P contexts in P host threads
    P, K = args.e2e_contexts, args.e2e_ranges
    nmsg = ho.numel()
    cuts = [nmsg * k // K for k in range(K + 1)]
    ranges = []
    for k in range(K):
        m0, m1 = cuts[k], cuts[k + 1]
        b0 = int(ho[m0])
        b1 = int(ho[m1 - 1]) + int(hl[m1 - 1])
        o = torch.empty(m1 - m0, dtype=torch.int64, pin_memory=True)
        o.copy_(ho[m0:m1] - b0)
        ranges.append((hb.data_ptr() + b0, b1 - b0, o, hl[m0:m1].clone().pin_memory(), m1 - m0))
    codecs = []
    for _ in range(P):
        c = FlowInfoCodec(0, rtc_sync=True)
        c.decode_datagrams([tm])
        codecs.append(c)
    per_out = (n // K + 1024) * BYTES_PER_RECORD_OUT + (4 << 20)
    outs = [torch.empty(per_out, dtype=torch.uint8, pin_memory=True) for _ in range(P)]
    got = [0] * P

    def worker(i):
        c, o = codecs[i], outs[i]
        moved = 0
        for k in range(i, K, P):
            ptr, size, ro, rl, m = ranges[k]
            c.decode_host_buffers(ptr, size, ro.data_ptr(), rl.data_ptr(), m)
            moved += c.columns_to_host(o.data_ptr(), o.numel())
        got[i] = moved

    def pipelined():
        th = [threading.Thread(target=worker, args=(i,)) for i in range(P)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return sum(got)

    t_pipe, moved_pipe = timed(pipelined)
    for c in codecs:
        c.close()

    # duplex: one host thread; the H2D of range k+1 (stream h) and the D2H of range k-1's columns
    # (stream d) are queued before the decode of range k, so PCIe carries both directions at once
    # while the GPU decodes.  Contexts round robin (a context's columns stay valid until its next
    # decode: the D2H that reads them is waited for first), device inputs double buffered.
    KD = args.e2e_duplex_ranges
    cuts = [nmsg * k // KD for k in range(KD + 1)]
    dranges = []
    for k in range(KD):
        m0, m1 = cuts[k], cuts[k + 1]
        b0 = int(ho[m0])
        b1 = int(ho[m1 - 1]) + int(hl[m1 - 1])
        meta = torch.empty(12 * (m1 - m0), dtype=torch.uint8, pin_memory=True)  # offsets (int64) + lengths (int32)
        meta[:8 * (m1 - m0)].view(torch.int64).copy_(ho[m0:m1] - b0)
        meta[8 * (m1 - m0):].view(torch.int32).copy_(hl[m0:m1])
        dranges.append((b0, b1 - b0, meta, m1 - m0))
    max_b = max(r[1] for r in dranges) + 16
    max_m = max(r[3] for r in dranges)
    dbuf = [torch.empty(max_b, dtype=torch.uint8, device=dev) for _ in range(2)]
    dmeta = [torch.empty(12 * max_m, dtype=torch.uint8, device=dev) for _ in range(2)]
    PD = max(2, args.e2e_duplex_contexts)
    dcodecs = []
    for _ in range(PD):
        c = FlowInfoCodec(0, rtc_sync=True)
        c.decode_datagrams([tm])
        dcodecs.append(c)
    sh, sd = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    out_d = torch.empty(n * BYTES_PER_RECORD_OUT + KD * (4 << 20), dtype=torch.uint8, pin_memory=True)

    def h2d(k):
        b0, nb, meta, m = dranges[k]
        with torch.cuda.stream(sh):
            dbuf[k % 2][:nb].copy_(hb[b0:b0 + nb], non_blocking=True)
            dmeta[k % 2][:12 * m].copy_(meta, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(sh)
        return ev

    def duplex(kernel):
        moved = 0
        ev_h = h2d(0)
        at = 0
        for k in range(KD):
            ev_h.synchronize()
            if k + 1 < KD:
                ev_h = h2d(k + 1)  # overlaps this decode and the previous range's D2H
            c = dcodecs[k % PD]  # its next decode waits for its last column copy (library side)
            _, nb, _, m = dranges[k]
            offs_k = dmeta[k % 2][:8 * m].view(torch.int64)
            lens_k = dmeta[k % 2][8 * m:12 * m].view(torch.int32)
            c.decode_batch(dbuf[k % 2][:nb], offs_k, lens_k)
            at = (at + 255) & ~255
            at += c.columns_to_host_async(out_d.data_ptr() + at, out_d.numel() - at, stream=sd.cuda_stream,
                                          kernel=kernel)
        torch.cuda.synchronize()
        return at

    t_dup, moved_dup = timed(lambda: duplex(False))
    t_dupk, moved_dupk = timed(lambda: duplex(True))
    modes = {
        "serial": (t_serial, moved, "one context, whole batch: H2D, decode, D2H in turn"),
        "threads": (t_pipe, moved_pipe, "%d message ranges over %d contexts in %d host threads" % (K, P, P)),
        "duplex": (t_dup, moved_dup, "one host thread: H2D of range k+1 and copy-engine D2H of range k-1 "
                                     "queued on two streams around range k's decode, %d contexts" % PD),
        "duplex_kernel": (t_dupk, moved_dupk, "as duplex, the D2H stored to pinned host memory by a kernel "
                                              "(ngz_columns_to_host_async NGZ_D2H_KERNEL), the copy engines "
                                              "left to the H2D"),
    }
    best = min(modes, key=lambda m: modes[m][0])
    t_best, moved_best, _ = modes[best]
    print(json.dumps({
        "metric": "IPFIX flow records/sec host-to-host (pinned H2D + decode + D2H of all columns), T20",
        "value": n / t_best, "unit": "records/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": t_best * 1e3, "higher_is_better": True,
        "dtype": "u8", "data": "synthetic T20, pinned host memory",
        "config": {"workload": "T20 x %d records, 1023 per message" % n, "h2d_bytes": int(hb.numel()),
                   "d2h_bytes": int(moved_best), "contexts": PD, "ranges": KD, "mode": best},
        "pcie_gbps": (hb.numel() + moved_best) / t_best / 1e9,
        "modes": {m: {"value": n / t, "ms_per_step": t * 1e3, "d2h_bytes": int(mv),
                      "pcie_gbps": (hb.numel() + mv) / t / 1e9, "how": how}
                  for m, (t, mv, how) in modes.items()}}), flush=True)


if __name__ == "__main__":
    main()

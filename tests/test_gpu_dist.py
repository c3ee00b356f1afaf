"""The multi-rank product path on the GPU: two processes share the one GPU of
the test box (gloo carries the collective, as RCCL needs one GPU per rank),
each cuts its contiguous message range of the one shared stream balanced by
records (ngz_message_records under its codec's templates, then
dist.shard_by_records: SURVEY §8(e)), decodes it with libngz on cuda:0, and the
per-template processed counts of both protocols (NetFlow v9 and IPFIX) are
exchanged with netgauze_amd.dist.CountExchange.  The node-wide totals must
equal a single oracle codec's over the whole stream, and every record must be
decoded exactly once.  (The 8-GPU RCCL run is the driver's; not measured
here.)"""
import os
import socket
import sys

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream(n):
    sys.path.insert(0, ROOT)
    from netgauze_amd import synth
    dg = synth.cfg4_datagrams(n, seed=synth.SEED_CFG4 + 5)
    t20 = synth.t20_records(3 * n, seed=synth.SEED_CFG2 + 5)
    buf, offs, lens = synth.ipfix_data_stream(t20, 64, rec_per_msg=97)
    b = bytes(buf.numpy())
    data = dg[2:] + [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]
    return dg[:2] + [synth.template_message()], data


def _threads(pid):
    """Threads of a process that did not exit: name, state, kernel wait channel, syscall."""
    out = []
    base = "/proc/%d/task" % pid
    try:
        tids = sorted(os.listdir(base))
    except OSError:
        return ["(gone)"]
    for t in tids:
        info = [t]
        for f in ("comm", "wchan", "syscall"):
            try:
                info.append(open(os.path.join(base, t, f)).read().strip()[:80])
            except OSError:
                info.append("?")
        out.append(" | ".join(info))
    return out


def _join_all(procs, timeout=120):
    """Join the ranks; a rank still running after the timeout is described and killed, so a
    hang fails the test with its threads instead of holding the test runner at exit."""
    hung = {}
    for p in procs:
        p.join(timeout=timeout)
        if p.exitcode is None:
            hung[p.pid] = _threads(p.pid)
            p.kill()
            p.join(timeout=10)
    return hung


def _worker(rank, world, port, n, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from netgauze_amd import dist as ndist
        from netgauze_amd.flow import FlowInfoCodec
        templates, data = _stream(n)
        # library default: template kernels compiled in the background; a rank may exit with a
        # compile in flight (ngz_rtc.cpp: the exit join runs before hiprtc's / comgr's teardown)
        codec = FlowInfoCodec(0)
        codec.decode_datagrams(templates)
        # the shard plan: every rank computes the same per-message records of the shared stream
        # and cuts its own range (no data-path collective)
        lens = [len(d) for d in data]
        offs = [0]
        for ln in lens[:-1]:
            offs.append(offs[-1] + ln)
        counts = ndist.message_records(b"".join(data), offs, lens, codec=codec)
        first, last = ndist.shard_by_records(counts, rank, world)
        batch = codec.decode_datagrams(data[first:last])
        ok = int((batch.dgram_headers()["status"] == 0).sum())
        ex = ndist.CountExchange(codec)
        ex.step(reset=True)
        total, fitted = ex.totals()
        q.put((rank, int(batch.n_records), ok, last - first, total, fitted, codec.template_counts(10),
               codec.template_counts(9), int(counts[first:last].sum()), int(counts.max())))
        import faulthandler  # a rank that does not exit: where it waits
        faulthandler.dump_traceback_later(45, repeat=False)
    except Exception as e:  # surface the failure instead of hanging the parent
        q.put((rank, "error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_two_ranks_decode_shards_and_exchange_counts():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import parity
    n = 3000
    templates, data = _stream(n)
    oracle, oc = parity.oracle_datagrams(templates + data)
    exp = {(10, t): v.processed_count for t, v in oc.ipfix_templates.items()}
    exp.update({(9, t): v.processed_count for t, v in oc.netflow_templates.items()})
    exp_records = sum(1 for kind, m in oracle if kind == "ok" for _ in m.data_records())
    world = 2
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in range(world)), key=lambda r: r[0])
    hung = _join_all(procs)
    assert not hung, hung
    assert all(r[1] != "error" for r in res), res
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert sum(r[3] for r in res) == len(data)              # every message in exactly one shard
    assert sum(r[1] for r in res) == exp_records            # every record decoded exactly once
    assert sum(r[2] for r in res) == len(data)              # every data message Ok
    # balanced by records: each rank decoded what the plan counted, and the two ranks are within
    # two of the largest messages of each other (shard_by_records' bound) although the stream
    # mixes 10-record NFv9 packets, ~15-record IPFIX MTU packets and 97-record T20 messages
    assert all(r[1] == r[8] for r in res), [(r[1], r[8]) for r in res]
    assert abs(res[0][1] - res[1][1]) <= 2 * res[0][9], [(r[1], r[9]) for r in res]
    for r in res:
        total, fitted = r[4], r[5]
        assert fitted and total == exp, (total, exp)        # node-wide templates.usage, protocols 10 and 9
        assert r[6] == {t: 0 for t in oc.ipfix_templates}   # reset after the exchange
        assert r[7] == {t: 0 for t in oc.netflow_templates}
    assert {k[0] for k in exp} == {9, 10}


def _nccl_worker(port, n_steps, q):
    """World-size-1 RCCL ("nccl") group: CountExchange(codec) with its default arguments (stream =
    torch's current stream), the device count table (ngz_template_counts_device) and the RCCL
    all_gather.  17 IPFIX templates + 1 NetFlow v9 template outgrow the 16-row default table:
    the first exchange does not fit (its counts carry over), the next grows the table."""
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from netgauze_amd import dist as ndist
        from netgauze_amd import synth
        from netgauze_amd.flow import FlowInfoCodec
        codec = FlowInfoCodec(0, specialize=True)
        ex = ndist.CountExchange(codec)
        assert ex.on_device and ex.stream == torch.cuda.current_stream().cuda_stream
        dg = synth.cfg4_datagrams(2000, seed=synth.SEED_CFG4 + 9)
        buf, offs, lens, _ = synth.mixed_stream(4000, templates=synth.CFG5_TEMPLATES, seed=synth.SEED_CFG5 + 9)
        b = bytes(buf.numpy())
        mixed = [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]
        codec.decode_datagrams(dg[:2] + [synth.templates_message(synth.CFG5_TEMPLATES)])
        steps = []
        for s in range(n_steps):
            data = dg[2:] if s % 2 == 0 else mixed
            codec.decode_datagrams(data)
            ex.step(reset=True)
            total, fitted = ex.totals()
            steps.append((s, fitted, ex.cap, total))
        q.put(("ok", steps))
    except Exception as e:
        q.put(("error", repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_count_exchange_rccl_defaults_and_growth():
    """the NCCL (RCCL) path of CountExchange with default arguments, against the
    oracle's processed counts, across a table growth."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import parity
    from netgauze_amd import synth
    dg = synth.cfg4_datagrams(2000, seed=synth.SEED_CFG4 + 9)
    buf, offs, lens, _ = synth.mixed_stream(4000, templates=synth.CFG5_TEMPLATES, seed=synth.SEED_CFG5 + 9)
    b = bytes(buf.numpy())
    mixed = [b[o:o + ln] for o, ln in zip(offs.tolist(), lens.tolist())]
    templates = dg[:2] + [synth.templates_message(synth.CFG5_TEMPLATES)]

    def oracle_counts(data):
        _, oc = parity.oracle_datagrams(templates + data)
        c = {(10, t): v.processed_count for t, v in oc.ipfix_templates.items()}
        c.update({(9, t): v.processed_count for t, v in oc.netflow_templates.items()})
        return c

    c_cfg4, c_mixed = oracle_counts(dg[2:]), oracle_counts(mixed)
    keys = set(c_cfg4) | set(c_mixed)
    assert len([k for k in keys if k[0] == 10]) > 16  # the 16-row default table must grow
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), 3, q))
    p.start()
    status, steps = q.get(timeout=240)
    hung = _join_all([p])
    assert not hung, hung
    assert status == "ok", steps
    assert p.exitcode == 0
    # step 0 (config-4 stream): 17 IPFIX templates > 16 rows -> not fitted, nothing reset
    s0, fit0, cap0, _ = steps[0]
    assert not fit0 and cap0 == 16
    # step 1 (config-5 stream): the table grew; the carried config-4 counts go out with this step's
    s1, fit1, cap1, tot1 = steps[1]
    assert fit1 and cap1 >= 17
    exp1 = {k: c_cfg4.get(k, 0) + c_mixed.get(k, 0) for k in keys}
    assert tot1 == exp1, (tot1, exp1)
    # step 2 (config-4 again): reset after step 1, so exactly this step's counts
    s2, fit2, _, tot2 = steps[2]
    assert fit2 and tot2 == {k: c_cfg4.get(k, 0) for k in keys}

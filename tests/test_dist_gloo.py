"""Multi-rank path on CPU (gloo, world_size 2): message sharding and the
per-template count all-gather, checked against a single-process oracle run."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_records, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ngz_oracle as O
    from netgauze_amd import dist as ndist, synth
    rec = synth.t20_records(n_records)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64, rec_per_msg=100)
    b = bytes(buf.numpy())
    first, last = ndist.shard_range(offs.numel(), rank, world)
    codec = O.FlowInfoCodec()
    codec.decode(bytearray(synth.template_message()))
    nrec = 0
    for o, ln in zip(offs.tolist()[first:last], lens.tolist()[first:last]):
        nrec += sum(1 for _ in codec.decode(bytearray(b[o:o + ln])).data_records())
    counts = {tid: t.processed_count for tid, t in codec.ipfix_templates.items()}
    total, tables = ndist.gather_template_counts(counts)
    q.put((rank, nrec, total, last - first))
    dist.destroy_process_group()


def test_sharded_counts_allgather_gloo():
    world, n = 2, 1234
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert sum(r[1] for r in res) == n                     # every record decoded exactly once
    n_msgs = (n + 99) // 100
    assert sum(r[3] for r in res) == n_msgs
    for r in res:                                          # every rank sees the node-wide count
        assert r[2] == {256: n_msgs}                       # +1 per data set (ipfix.rs:223)


def test_shard_range_partitions():
    from netgauze_amd.dist import shard_range
    for n in (0, 1, 7, 97752):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))


def _worker_many(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from netgauze_amd import dist as ndist
    # rank 0 sees 20 templates (more than the default table), rank 1 three of them
    counts = {256 + t: 10 * t + 1 for t in range(20)} if rank == 0 else {256: 5, 260: 7, 5000: 9}
    total, tables = ndist.gather_template_counts(counts)
    q.put((rank, total, [tuple(t.shape) for t in tables]))
    dist.destroy_process_group()


def test_count_allgather_more_templates_than_default_table():
    """Config 5 has 16 templates per rank; a rank with more must not have any
    dropped: ranks agree on the table size before the all-gather."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_many, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = {256 + t: 10 * t + 1 for t in range(20)}
    exp[256] += 5
    exp[260] += 7
    exp[5000] = 9
    for _, total, shapes in res:
        assert total == exp
        assert shapes == [(20, 2), (20, 2)]


def _skewed_stream():
    """MTU-sized NetFlow v9 datagrams (template 313, 10 records each, as Cisco exporters send)
    followed by 64 KB IPFIX T20 messages (1023 records each): the template messages, then the
    data messages."""
    from netgauze_amd import synth
    _, rl = synth.field_offsets(synth.NF313)
    nf = synth.template_records(synth.NF313, 20_000, 7, "cpu").numpy()
    nf_msgs = synth._pack_nfv9(nf, rl, synth.NF313_ID)
    rec = synth.t20_records(20 * 1023)
    buf, offs, lens = synth.ipfix_data_stream(rec, 64)
    b = bytes(buf.numpy())
    t20 = [b[o:o + n] for o, n in zip(offs.tolist(), lens.tolist())]
    return [synth.nfv9_template_message(), synth.template_message()], nf_msgs + t20, {
        (9, synth.NF313_ID): rl, (10, synth.T20_ID): 64}


def _worker_skewed(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "oracle"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import numpy as np
    import ngz_oracle as O
    from netgauze_amd import dist as ndist
    tmpl, data, rl = _skewed_stream()
    blob = b"".join(data)
    offs = np.cumsum([0] + [len(d) for d in data[:-1]])
    counts = ndist.message_records(blob, offs, [len(d) for d in data], rl)
    first, last = ndist.shard_by_records(counts, rank, world)
    codec = O.FlowInfoCodec()
    for t in tmpl:
        codec.decode(bytearray(t))
    nrec = 0
    for d in data[first:last]:
        nrec += sum(1 for _ in codec.decode(bytearray(d)).data_records())
    mine = {(10, t): v.processed_count for t, v in codec.ipfix_templates.items()}
    mine.update({(9, t): v.processed_count for t, v in codec.netflow_templates.items()})
    total, _ = ndist.gather_template_counts({(p << 16) | t: c for (p, t), c in mine.items()})
    q.put((rank, nrec, int(counts[first:last].sum()), total, last - first))
    dist.destroy_process_group()


def test_shards_balanced_by_records_gloo():
    """A skewed stream (2 000 MTU NetFlow v9 datagrams of 10 records, then 20 64 KB IPFIX messages
    of 1023) over 2 gloo ranks: shard_by_records cuts by the records the headers announce
    (message_records), so the ranks' decoded record counts differ by at most one message's records
    (an even message split would give one rank 1 000 datagrams = 10 000 records and the other
    30 460), the header estimate equals what each rank decodes, and the node-wide
    templates.usage equals a single codec's (flow_actor.rs:362-381)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import ngz_oracle as O
    from netgauze_amd import dist as ndist
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_skewed, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tmpl, data, _ = _skewed_stream()
    oc = O.FlowInfoCodec()
    for d in tmpl + data:
        oc.decode(bytearray(d))
    n_total = 20_000 + 20 * 1023
    assert sum(r[1] for r in res) == n_total
    assert all(r[1] == r[2] for r in res)               # header estimate == records decoded
    assert abs(res[0][1] - res[1][1]) <= 1023            # within one datagram of each other
    lo, hi = ndist.shard_range(len(data), 0, 2)          # the message split it replaces
    assert hi - lo == 1010 and sum(r[4] for r in res) == len(data)
    want = {(10 << 16) | t: v.processed_count for t, v in oc.ipfix_templates.items()}
    want.update({(9 << 16) | t: v.processed_count for t, v in oc.netflow_templates.items()})
    for r in res:
        assert r[3] == want


def test_shard_by_records_partitions():
    import numpy as np
    from netgauze_amd.dist import shard_by_records
    rng = np.random.default_rng(3)
    for n in (0, 1, 5, 1000):
        rec = rng.integers(0, 1100, n)
        for w in (1, 2, 3, 8):
            parts = [shard_by_records(rec, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            if n:
                loads = [int(rec[a:b].sum()) for a, b in parts]
                assert max(loads) - min(loads) <= 2 * int(rec.max()) + 1

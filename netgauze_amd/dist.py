"""Multi-GPU sharding for the decode path (one process per GPU).

Flow records are independent, and messages are independent once template
state is known, so a node shards its datagram batch by contiguous message
ranges (each rank = its own set of exporter peers / its own context, as the
reference's collector actors partition peers, flow_supervisor.rs:288-305).
No record bytes cross GPUs.  The only collective is the per-template
processed-count exchange that feeds netgauze.flow.decoder.templates.usage
(flow_actor.rs:362-381): an all-gather of a fixed [MAX_TEMPLATES x 3] int64
table (proto, template id, count) per rank over RCCL (backend "nccl") or gloo.
"""
import torch

MAX_TEMPLATES = 16


def shard_range(n, rank, world):
    """Contiguous [first, last) of n messages for this rank."""
    return n * rank // world, n * (rank + 1) // world


def pack_counts(counts, proto=10, device="cpu"):
    """{template_id: count} -> (MAX_TEMPLATES, 3) int64 [proto, id, count]; id -1 = empty."""
    t = torch.full((MAX_TEMPLATES, 3), -1, dtype=torch.int64, device=device)
    for i, (tid, c) in enumerate(sorted(counts.items())[:MAX_TEMPLATES]):
        t[i, 0] = proto
        t[i, 1] = tid
        t[i, 2] = c
    return t


def gather_template_counts(counts, proto=10, group=None, device="cpu"):
    """All-gather every rank's per-template processed counts.

    Returns {template_id: total} summed over ranks and the per-rank tables."""
    import torch.distributed as dist
    local = pack_counts(counts, proto, device)
    world = dist.get_world_size(group)
    tables = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(tables, local, group=group)
    total = {}
    for tab in tables:
        for row in tab.tolist():
            if row[1] >= 0 and row[0] == proto:
                total[row[1]] = total.get(row[1], 0) + row[2]
    return total, tables

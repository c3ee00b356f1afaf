"""Multi-GPU sharding for the decode path (one process per GPU).

Flow records are independent, and messages are independent once template
state is known, so a node shards its datagram batch by contiguous message
ranges (each rank = its own set of exporter peers / its own context, as the
reference's collector actors partition peers, flow_supervisor.rs:288-305).
No record bytes cross GPUs.  The only collective is the per-template
processed-count exchange that feeds netgauze.flow.decoder.templates.usage
(flow_actor.rs:362-381): an all-reduce(max) of the template count, then an
all-gather of a [max(16, templates) x 3] int64 table (proto, template id,
count) per rank over RCCL (backend "nccl") or gloo.
"""
import torch

MAX_TEMPLATES = 16


def shard_range(n, rank, world):
    """Contiguous [first, last) of n messages for this rank."""
    return n * rank // world, n * (rank + 1) // world


def pack_counts(counts, proto=10, device="cpu", rows=None):
    """{template_id: count} -> (rows, 3) int64 [proto, id, count]; id -1 = empty.
    rows defaults to max(MAX_TEMPLATES, len(counts)); a table never drops a template."""
    rows = max(MAX_TEMPLATES, len(counts)) if rows is None else rows
    if rows < len(counts):
        raise ValueError("%d templates do not fit a %d-row count table" % (len(counts), rows))
    t = torch.full((rows, 3), -1, dtype=torch.int64, device=device)
    for i, (tid, c) in enumerate(sorted(counts.items())):
        t[i, 0] = proto
        t[i, 1] = tid
        t[i, 2] = c
    return t


def gather_template_counts(counts, proto=10, group=None, device="cpu"):
    """All-gather every rank's per-template processed counts.

    Returns {template_id: total} summed over ranks and the per-rank tables."""
    import torch.distributed as dist
    # ranks agree on the table size first (8 bytes), so no rank's templates are dropped
    n = torch.tensor([len(counts)], dtype=torch.int64, device=device)
    dist.all_reduce(n, op=dist.ReduceOp.MAX, group=group)
    local = pack_counts(counts, proto, device, max(MAX_TEMPLATES, int(n.item())))
    world = dist.get_world_size(group)
    tables = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(tables, local, group=group)
    total = {}
    for tab in tables:
        for row in tab.tolist():
            if row[1] >= 0 and row[0] == proto:
                total[row[1]] = total.get(row[1], 0) + row[2]
    return total, tables

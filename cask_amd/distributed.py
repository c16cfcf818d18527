"""Multi-GPU layout of the scan: one process per GPU, data files sharded in contiguous file-id
ranges (so the per-key fold order is rank order, then file id, then position — SURVEY §8e), no
collective on the scan itself. The keydir rows meet on rank 0 through point-to-point transfers
(RCCL over xGMI on the GPU; gloo in the CPU tests), and the replay's max sequence
(cask.rs:350-352) is an all-reduce(max).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

ROW_FIELDS = ("pos", "seq", "vsz", "ksz", "status")


def shard_files(file_ids, world: int, rank: int):
    """Contiguous ranges of the sorted file ids, sizes differing by at most one."""
    ids = sorted(file_ids)
    n = len(ids)
    lo = rank * n // world
    hi = (rank + 1) * n // world
    return ids[lo:hi]


def allreduce_max_seq(local_max: int, device) -> int:
    t = torch.tensor([int(local_max)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def gather_rows(rows: dict, count: int, dst: int = 0, file_id=None):
    """Gather every rank's first `count` rows (SoA tensors) to `dst`, in rank order.

    Returns the list of per-rank row dicts on `dst` (None elsewhere). Row blocks are
    variable-sized: counts travel first (all_gather), then one send/recv per field per rank.
    `file_id` (optional int32 tensor, same length) travels along."""
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = rows["pos"].device
    cnt = torch.tensor([int(count)], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt)
    counts = [int(c.item()) for c in counts]
    fields = list(ROW_FIELDS) + (["file_id"] if file_id is not None else [])
    src = dict(rows)
    if file_id is not None:
        src["file_id"] = file_id
    if rank == dst:
        out = []
        ops = []
        for r in range(world):
            if r == dst:
                out.append({f: src[f][:counts[r]] for f in fields})
                continue
            d = {f: torch.empty(counts[r], dtype=src[f].dtype, device=dev) for f in fields}
            out.append(d)
            for f in fields:
                if counts[r]:
                    ops.append(dist.P2POp(dist.irecv, d[f], r))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return out
    ops = [dist.P2POp(dist.isend, src[f][:count].contiguous(), dst) for f in fields if count]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return None

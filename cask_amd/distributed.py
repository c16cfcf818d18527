"""Multi-GPU layout of the replay: one process per GPU, data files sharded in
contiguous file-id ranges, so that rank order, then file id, then position is the reference's
replay order (cask.rs:348). The scan needs no collective. Each rank reduces its rows to a keydir
block on its GPU (cask_amd.keydir.shard_keydir: the records that can decide the keydir, the
tombstones whose stale count depends on the ranks before, per-file put counts, key bytes); the
blocks meet on rank 0 through point-to-point transfers — RCCL over xGMI on the GPUs (torch's
"nccl" backend), gloo in the CPU tests — and rank 0 folds them in rank order
(cask_amd.keydir.KeydirFold). The replay's max sequence (cask.rs:350-352) travels in the blocks;
allreduce_max_seq gives it to every rank.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


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


def gather_blocks(block: torch.Tensor, dst: int = 0):
    """Gather every rank's keydir block (a uint8 tensor of any length, on the rank's device for
    RCCL, on the CPU for gloo) to `dst`, one message per rank. Returns the blocks in rank order on
    `dst`, None elsewhere."""
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = block.device
    n = torch.tensor([block.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    if rank == dst:
        out, ops = [], []
        for r in range(world):
            if r == dst:
                out.append(block)
                continue
            t = torch.empty(sizes[r], dtype=torch.uint8, device=dev)
            out.append(t)
            if sizes[r]:
                ops.append(dist.P2POp(dist.irecv, t, r))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return out
    if block.numel():
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, block.contiguous(), dst)]):
            w.wait()
    return None

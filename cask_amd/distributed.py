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


class RcclComm:
    """An RCCL communicator made by the library itself (cask_rccl_comm_init), for the C-ABI gather:
    the path a Rust host replacing cask.rs:346-382 takes, with no torch. `uid` is the 128-byte id
    from rccl_unique_id() on one rank, distributed by the caller (here: torch.distributed)."""

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int):
        import ctypes as C
        from . import _lib as L
        from .errors import raise_status
        self.lib = L.lib()
        buf = (C.c_uint8 * len(uid)).from_buffer_copy(uid)
        h = C.c_void_p()
        raise_status(self.lib.cask_rccl_comm_init(buf, nranks, rank, device, C.byref(h)), what="cask_rccl_comm_init")
        self._h = h
        self.nranks, self.rank = nranks, rank

    def close(self):
        if self._h:
            self.lib.cask_rccl_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def rccl_unique_id() -> bytes:
    import ctypes as C
    from . import _lib as L
    from .errors import raise_status
    lib = L.lib()
    buf = (C.c_uint8 * 128)()
    raise_status(lib.cask_rccl_unique_id(buf), what="cask_rccl_unique_id")
    return bytes(buf)


def rccl_comm_from_dist(device: int) -> RcclComm:
    """Rank 0 makes the id, torch.distributed carries it to the other ranks, every rank joins."""
    rank, world = dist.get_rank(), dist.get_world_size()
    uid = [rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    return RcclComm(uid[0], world, rank, device)


def gather_fold_rccl(ctx, comm: RcclComm, block: torch.Tensor, root: int = 0):
    """cask_keydir_gather_rccl: every rank's keydir block (uint8 CUDA tensor) to `root` over RCCL and
    root's fold of them in rank order. Returns (Cask handle on root / None elsewhere, gathered bytes,
    global max sequence)."""
    import ctypes as C
    from . import _lib as L
    from .cask import Cask
    from .errors import raise_status
    lib = L.lib()
    kd = lib.cask_keydir_new() if comm.rank == root else None
    if comm.rank == root and not kd:
        raise MemoryError("cask_keydir_new")
    got, mx = C.c_uint64(), C.c_uint64()
    ctx._inputs_ready()
    rc = lib.cask_keydir_gather_rccl(ctx._h, comm._h, C.c_void_p(block.data_ptr()) if block.numel() else None,
                                     block.numel(), root, kd, C.byref(got), C.byref(mx))
    if rc != L.OK:
        if kd:
            lib.cask_db_close(kd)
        raise_status(rc, what=f"cask_keydir_gather_rccl: {ctx.last_error()}")
    if kd is None:
        return None, int(got.value), int(mx.value)
    rc = lib.cask_keydir_finish(kd)
    if rc != L.OK:
        lib.cask_db_close(kd)
        raise_status(rc, what="cask_keydir_finish")
    return Cask(kd, ""), int(got.value), int(mx.value)

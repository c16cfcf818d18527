"""Multi-GPU layout of the replay: one process per GPU, data files sharded in
contiguous file-id ranges, so that rank order, then file id, then position is the reference's
replay order (cask.rs:348). The scan needs no collective. Each rank reduces its rows to a keydir
block on its GPU (cask_amd.keydir.shard_keydir: the records that can decide the keydir, the
tombstones whose stale count depends on the ranks before, per-file put counts, key bytes); then
either
  * the blocks meet on rank 0 through point-to-point transfers — RCCL over xGMI on the GPUs
    (torch's "nccl" backend, or the library's own RCCL communicator: gather_fold_rccl), gloo in the
    CPU tests — and rank 0 folds them in rank order (cask_amd.keydir.KeydirFold); or
  * for a keyspace too large for one host, every block is split by key owner and the parts go
    all-to-all (partitioned_fold over torch.distributed, exchange_fold_rccl through the C ABI):
    each rank folds the keys it owns, and every rank gets the whole replay's Stats.
The replay's max sequence (cask.rs:350-352) travels in the blocks; allreduce_max_seq gives it to
every rank.
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


def exchange_parts(parts):
    """The all-to-all of a partitioned replay: parts[o] (uint8 tensors, on the rank's device for
    RCCL, on the CPU for gloo) to rank o. Returns the parts every rank sent this one, in rank order
    (its own included)."""
    rank, world = dist.get_rank(), dist.get_world_size()
    assert len(parts) == world
    dev = parts[rank].device
    n = torch.tensor([p.numel() for p in parts], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    recv, ops = [], []
    for r in range(world):
        if r == rank:
            recv.append(parts[r].clone())
            continue
        t = torch.empty(int(sizes[r][rank].item()), dtype=torch.uint8, device=dev)
        recv.append(t)
        if parts[r].numel():
            ops.append(dist.P2POp(dist.isend, parts[r].contiguous(), r))
        if t.numel():
            ops.append(dist.P2POp(dist.irecv, t, r))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return recv


def all_gather_bytes(b: torch.Tensor):
    """Every rank's uint8 tensor (any length), in rank order, on every rank."""
    world = dist.get_world_size()
    n = torch.tensor([b.numel()], dtype=torch.int64, device=b.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = max(int(s.item()) for s in sizes)
    pad = torch.zeros(max(m, 1), dtype=torch.uint8, device=b.device)
    pad[:b.numel()] = b
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return [o[:int(s.item())] for o, s in zip(outs, sizes)]


def partitioned_fold(block):
    """The key-hash partitioned replay over torch.distributed (gloo on the CPU; the GPUs use
    exchange_fold_rccl): this rank's keydir block (host bytes / numpy / CPU tensor) split by key
    owner (cask_keydir_partition_host), part o to rank o, this rank's fold of the parts it owns in
    rank order, then the owners' terms to every rank. Returns this rank's Cask handle: its own keys,
    and the whole replay's Stats, files and sequence."""
    import numpy as np
    from .keydir import KeydirFold, partition_host
    world = dist.get_world_size()
    parts = [torch.from_numpy(np.ascontiguousarray(p)) for p in partition_host(block, world)]
    fold = KeydirFold()
    fold.merge_all(exchange_parts(parts))
    terms = all_gather_bytes(torch.from_numpy(fold.terms()))
    return fold.finish_terms(b"".join(t.numpy().tobytes() for t in terms))


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


def exchange_fold_rccl(ctx, comm: RcclComm, block: torch.Tensor):
    """cask_keydir_exchange_rccl: the key-hash all-to-all of every rank's keydir block (uint8 CUDA
    tensor) over RCCL, this rank's fold of the keys it owns and the Stats of the whole replay.
    Returns (Cask handle, bytes sent, bytes received)."""
    import ctypes as C
    from . import _lib as L
    from .cask import Cask
    from .errors import raise_status
    lib = L.lib()
    kd = lib.cask_keydir_new()
    if not kd:
        raise MemoryError("cask_keydir_new")
    sent, got = C.c_uint64(), C.c_uint64()
    ctx._inputs_ready()
    rc = lib.cask_keydir_exchange_rccl(ctx._h, comm._h, C.c_void_p(block.data_ptr()) if block.numel() else None,
                                       block.numel(), kd, C.byref(sent), C.byref(got))
    if rc != L.OK:
        lib.cask_db_close(kd)
        raise_status(rc, what=f"cask_keydir_exchange_rccl: {ctx.last_error()}")
    return Cask(kd, ""), int(sent.value), int(got.value)

"""Multi-GPU replay: a shard's keydir block from its device rows, and rank 0's fold
of the blocks in rank order. The block format and what it carries are described in
include/cask_scan.h and cask_amd/csrc/keydir_format.h; all work is in libcask_scan.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .cask import Cask, CaskOptions
from .errors import raise_status


def shard_keydir(ctx, files, rows: dict, count: int, file_row_offset):
    """The keydir block of the files one rank scanned: `files` [(file_id, uint8 CUDA tensor)] as
    passed to ctx.scan_device, its rows dict and ScanResult.count / file_row_offset (every row Ok).
    Returns a uint8 CUDA tensor (a copy: the context's buffer is reused by its next call)."""
    return _shard(ctx, ctx.lib.cask_shard_keydir, "cask_shard_keydir", files, rows, count, file_row_offset)


def shard_keydir_hints(ctx, bodies, rows: dict, count: int, file_row_offset):
    """The same block from hint-file bodies (the hint fast path, log.rs:121-135): `bodies`
    [(file_id, uint8 CUDA tensor without the trailer)] and the rows of ctx.parse_hints_device
    (every row Ok; their pos is rewritten to entry positions)."""
    return _shard(ctx, ctx.lib.cask_shard_keydir_hints, "cask_shard_keydir_hints", bodies, rows, count,
                  file_row_offset)


def _shard(ctx, fn, name, files, rows, count, file_row_offset):
    import torch
    n = len(files)
    views = (L.FileView * max(n, 1))()
    for i, (fid, t) in enumerate(files):
        views[i].file_id = int(fid)
        views[i].flags = L.VIEW_DEVICE
        views[i].data = t.data_ptr() if t.numel() else None
        views[i].len = t.numel()
    r = L.Rows()
    r.capacity = rows["pos"].numel()
    r.count = int(count)
    r.pos, r.seq = rows["pos"].data_ptr(), rows["seq"].data_ptr()
    r.vsz, r.ksz, r.status = rows["vsz"].data_ptr(), rows["ksz"].data_ptr(), rows["status"].data_ptr()
    off = (C.c_uint64 * (n + 1))(*[int(x) for x in file_row_offset])
    blk, nb = C.c_void_p(), C.c_uint64()
    ctx._inputs_ready()
    rc = fn(ctx._h, views, n, C.byref(r), off, C.byref(blk), C.byref(nb))
    raise_status(rc, what=f"{name}: {ctx.last_error()}")
    dev = torch.device("cuda", ctx.device)
    out = torch.empty(int(nb.value), dtype=torch.uint8, device=dev)
    ctx._inputs_ready()  # the allocation is ordered on torch's stream
    raise_status(ctx.lib.cask_copy(ctx._h, C.c_void_p(out.data_ptr()), blk, nb.value), what="cask_copy")
    return out


def _u8(block):
    """bytes / numpy uint8 / CPU uint8 tensor -> contiguous numpy uint8."""
    if hasattr(block, "numpy"):
        block = block.numpy()
    return np.ascontiguousarray(np.frombuffer(block, np.uint8) if isinstance(block, (bytes, bytearray)) else block,
                                dtype=np.uint8)


def key_owner(key: bytes, nparts: int) -> int:
    """cask_keydir_owner: the rank that holds `key` after a partitioned replay."""
    return int(L.lib().cask_keydir_owner(key, len(key), nparts))


def partition_host(block, nparts: int) -> list[np.ndarray]:
    """cask_keydir_partition_host: the block (host bytes) split by key owner into nparts blocks."""
    lib = L.lib()
    a = _u8(block)
    off = (C.c_uint64 * (nparts + 1))()
    rc = lib.cask_keydir_partition_host(a.ctypes.data, a.size, nparts, None, 0, off)
    if rc != L.E_CAPACITY:
        raise_status(rc, what="cask_keydir_partition_host")
    out = np.zeros(int(off[nparts]), np.uint8)
    raise_status(lib.cask_keydir_partition_host(a.ctypes.data, a.size, nparts, out.ctypes.data, out.size, off),
                 what="cask_keydir_partition_host")
    return [out[int(off[o]):int(off[o + 1])] for o in range(nparts)]


def partition_device(ctx, block, nparts: int):
    """cask_keydir_partition: a device block (uint8 CUDA tensor) split on its GPU; returns the parts
    as uint8 CUDA tensors (copies: the context's buffer is reused by its next call)."""
    import torch
    off = (C.c_uint64 * (nparts + 1))()
    parts = C.c_void_p()
    ctx._inputs_ready()
    rc = ctx.lib.cask_keydir_partition(ctx._h, C.c_void_p(block.data_ptr()), block.numel(), nparts, C.byref(parts), off)
    raise_status(rc, what=f"cask_keydir_partition: {ctx.last_error()}")
    out = torch.empty(int(off[nparts]), dtype=torch.uint8, device=block.device)
    ctx._inputs_ready()
    if out.numel():
        raise_status(ctx.lib.cask_copy(ctx._h, C.c_void_p(out.data_ptr()), parts, out.numel()), what="cask_copy")
    return [out[int(off[o]):int(off[o + 1])] for o in range(nparts)]


class KeydirFold:
    """Rank 0's fold (cask_keydir_new / _merge / _finish): merge the blocks in rank order, then
    finish() returns a Cask handle with the keydir, stats and sequence of the whole replay.

    In a partitioned replay each owner merges the parts it was sent (rank order), exchanges terms()
    with the other owners and calls finish_terms(all owners' terms): its handle then holds its own
    keys and the whole replay's Stats, files and sequence."""

    def __init__(self):
        self.lib = L.lib()
        self._h = self.lib.cask_keydir_new()
        if not self._h:
            raise MemoryError("cask_keydir_new")

    def merge(self, block):
        """block: bytes, a numpy uint8 array or a CPU uint8 tensor."""
        a = _u8(block)
        raise_status(self.lib.cask_keydir_merge(self._h, a.ctypes.data, a.size), what="cask_keydir_merge")

    def merge_all(self, blocks):
        """blocks merged in order in one pass (cask_keydir_merge_many): the same result as merge()
        of each in turn."""
        arrs = [_u8(b) for b in blocks]
        n = len(arrs)
        ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
        lens = (C.c_uint64 * max(n, 1))(*[a.size for a in arrs])
        raise_status(self.lib.cask_keydir_merge_many(self._h, ptrs, lens, n), what="cask_keydir_merge_many")

    def finish(self) -> Cask:
        raise_status(self.lib.cask_keydir_finish(self._h), what="cask_keydir_finish")
        h, self._h = self._h, None
        return Cask(h, "")

    def terms(self) -> np.ndarray:
        """This owner's per-file terms (KeydirTerm records, 56 B each) after its merges."""
        n = self.lib.cask_keydir_terms(self._h, None, 0)
        if n < 0:
            raise_status(int(n), what="cask_keydir_terms")
        out = np.zeros(int(n), np.uint8)
        got = self.lib.cask_keydir_terms(self._h, out.ctypes.data if n else None, out.size)
        if got != n:
            raise_status(int(got) if got < 0 else L.E_INVALID_ARG, what="cask_keydir_terms")
        return out

    def finish_terms(self, all_terms) -> Cask:
        """Finish with every owner's terms concatenated (this one's included)."""
        a = _u8(all_terms)
        raise_status(self.lib.cask_keydir_finish_terms(self._h, a.ctypes.data if a.size else None, a.size),
                     what="cask_keydir_finish_terms")
        h, self._h = self._h, None
        return Cask(h, "")

    def __del__(self):
        if getattr(self, "_h", None):
            self.lib.cask_db_close(self._h)


def open_multi(path: str, devices, options: CaskOptions | None = None) -> Cask:
    """cask_db_open_multi: Cask::open with the data files split over `devices` (GPU ordinals of
    this process, repeats allowed). Files with a valid hint file are replayed from it (parsed on the
    device); the others are scanned and, unless options.write_hints(False), get their hint files."""
    o = options or CaskOptions()
    lib = L.lib()
    opts = L.Options()
    lib.cask_options_default(C.byref(opts))
    opts.create = 1 if o._create else 0
    opts.write_hints = 1 if o._write_hints else 0
    opts.max_file_size = o._max_file_size
    devs = (C.c_int * len(devices))(*[int(d) for d in devices])
    err = L.OpenError()
    h = lib.cask_db_open_multi(path.encode(), C.byref(opts), devs, len(devices), C.byref(err))
    if not h:
        raise_status(err.status, err.file_id, err.pos, err.expected, err.found, what=path)
    return Cask(h, path, o)

"""The multi-rank control flow of the RCCL keydir paths (cask.rs:60-90 folded per shard,
driven by cask.rs:346-382) without a second GPU: 2-4 ranks as threads of this process, each with its
own context and stream on cuda:0, over tests/fake_rccl (a stand-in for librccl selected with the
CASK_RCCL_LIB test hook: collectives by rendezvous, point-to-point by device copies).

What real RCCL on one GPU cannot show: that every rank issues the same collectives whatever fails on
it — a root that cannot allocate the gathered blocks, a bad argument on one rank, a partition or a
fold that fails on one rank, an owner that cannot read its terms — so that all ranks return the same
status and none waits on a peer (the stand-in gives up after CASK_FAKE_RCCL_TIMEOUT seconds; a rank
left waiting would come back with CASK_E_DEVICE, not the agreed status). The clean runs check the
keydir, Stats and sequence against the oracle's single-process replay. Needs an MI355X.
"""
import ctypes as C
import os
import threading
import time

import numpy as np
import pytest

from test_shard_gpu import _files, _got, _make_db, _want

pytestmark = pytest.mark.gpu

FAKE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fake_rccl", "libfake_rccl.so")
TIMEOUT_S = 12.0
INJ_ROOT_ALLOC, INJ_PARTITION, INJ_TERMS, INJ_THROW, INJ_FOLD = 1, 2, 4, 8, 16


@pytest.fixture()
def fake_rccl(native):
    assert os.path.exists(FAKE), "tests/fake_rccl/libfake_rccl.so is built by make -C cask_amd"
    old = {k: os.environ.get(k) for k in ("CASK_RCCL_LIB", "CASK_FAKE_RCCL_TIMEOUT")}
    os.environ["CASK_RCCL_LIB"] = FAKE
    os.environ["CASK_FAKE_RCCL_TIMEOUT"] = str(TIMEOUT_S)
    try:
        yield native
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _shards(path, nranks):
    """Contiguous file-id ranges, one per rank (replay order = rank order)."""
    files = _files(path)
    cuts = [round(i * len(files) / nranks) for i in range(nranks + 1)]
    return [files[cuts[r]:cuts[r + 1]] for r in range(nranks)]


def _block(ctx, part):
    import torch
    from cask_amd.keydir import shard_keydir
    if not part:
        return torch.empty(0, dtype=torch.uint8, device="cuda:0")
    tens = [(fid, torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()) for fid, b in part]
    res = ctx.scan_device(tens)
    assert res.error is None
    blk = shard_keydir(ctx, tens, {"pos": res.pos, "seq": res.seq, "vsz": res.vsz, "ksz": res.ksz,
                                   "status": res.status}, res.count, res.file_row_offset)
    torch.cuda.synchronize()
    return blk


def _run_ranks(nranks, body):
    """body(rank) on a thread per rank; every rank must return within the stand-in's wait limit."""
    out, err, took = [None] * nranks, [None] * nranks, [None] * nranks

    def run(r):
        t0 = time.monotonic()
        try:
            out[r] = body(r)
        except BaseException as e:  # noqa: BLE001 (reported below)
            err[r] = e
        took[r] = time.monotonic() - t0

    th = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(nranks)]
    for t in th:
        t.start()
    for t in th:
        t.join(TIMEOUT_S * 4)
    assert not any(t.is_alive() for t in th), "a rank is still blocked"
    for e in err:
        if e is not None:
            raise e
    return out, took


class _Rank:
    """One rank's context, communicator and block."""

    def __init__(self, lib, uid, nranks, rank, part, inject=0):
        from cask_amd import ScanContext
        from cask_amd.distributed import RcclComm
        self.lib, self.rank = lib, rank
        self.ctx = ScanContext(0)
        self.blk = _block(self.ctx, part)
        self.comm = RcclComm(uid, nranks, rank, 0)  # (returns once every rank has joined)
        if inject:
            assert lib.cask_debug_inject(self.ctx._h, inject) == 0

    def gather(self, root):
        kd = self.lib.cask_keydir_new() if self.rank == root else None
        got, mx = C.c_uint64(), C.c_uint64()
        rc = self.lib.cask_keydir_gather_rccl(self.ctx._h, self.comm._h,
                                              C.c_void_p(self.blk.data_ptr()) if self.blk.numel() else None,
                                              self.blk.numel(), root, kd, C.byref(got), C.byref(mx))
        return rc, kd, int(got.value), int(mx.value)

    def exchange(self):
        kd = self.lib.cask_keydir_new()
        sent, got = C.c_uint64(), C.c_uint64()
        rc = self.lib.cask_keydir_exchange_rccl(self.ctx._h, self.comm._h,
                                                C.c_void_p(self.blk.data_ptr()) if self.blk.numel() else None,
                                                self.blk.numel(), kd, C.byref(sent), C.byref(got))
        return rc, kd, int(sent.value), int(got.value)

    def close(self):
        self.comm.close()


def _setup(lib, path, nranks, injects=None):
    from cask_amd.distributed import rccl_unique_id
    uid = rccl_unique_id()
    parts = _shards(path, nranks)
    injects = injects or {}
    ranks, _ = _run_ranks(nranks, lambda r: _Rank(lib, uid, nranks, r, parts[r], injects.get(r, 0)))
    return ranks


@pytest.mark.parametrize("nranks,root", [(2, 0), (3, 2), (4, 1)])
def test_gather_ranks_fold_equals_replay(fake_rccl, tmp_path, nranks, root):
    """2-4 ranks gather their shards' blocks to the root, which folds them in rank order: the keydir,
    Stats and sequence of the single-process replay; every rank reports the global max sequence."""
    from cask_amd.cask import Cask
    lib = fake_rccl
    path = str(tmp_path / "db")
    _make_db(path, 40 + nranks, nfiles=5)
    want = _want(path)
    ranks = _setup(lib, path, nranks)
    try:
        res, took = _run_ranks(nranks, lambda r: ranks[r].gather(root))
        assert [x[0] for x in res] == [0] * nranks
        assert {x[3] for x in res} == {want[2] - 1}
        kd = res[root][1]
        assert lib.cask_keydir_finish(kd) == 0
        with Cask(kd, "") as db:
            assert _got(db) == want
        assert res[root][2] == sum((rk.blk.numel() + 255) // 256 * 256 for rk in ranks)
    finally:
        for rk in ranks:
            rk.close()


@pytest.mark.parametrize("case", ["root_alloc", "bad_root", "root_mismatch", "root_fold"])
def test_gather_failure_on_one_rank_is_agreed(fake_rccl, tmp_path, case):
    """A root that cannot allocate the gathered blocks, one rank passing a root out of range, one
    rank naming a different (valid) root than the others, a root whose fold fails: every rank
    returns the same status (rccl_gather.cpp agree()), none blocks."""
    lib = fake_rccl
    path = str(tmp_path / "db")
    _make_db(path, 50, nfiles=3)
    nranks = 3
    inj = {"root_alloc": {0: INJ_ROOT_ALLOC}, "root_fold": {0: INJ_FOLD}}.get(case, {})
    ranks = _setup(lib, path, nranks, inj)
    try:
        roots = [0, {"bad_root": 99, "root_mismatch": 2}.get(case, 0), 0]
        res, took = _run_ranks(nranks, lambda r: ranks[r].gather(roots[r]))
        want = {"root_alloc": -13, "bad_root": -10, "root_mismatch": -10, "root_fold": -13}[case]
        assert [x[0] for x in res] == [want] * nranks
        assert max(took) < TIMEOUT_S / 2, took  # no rank waited for the stand-in to give up
        for x in res:
            if x[1]:
                lib.cask_db_close(x[1])
        # the communicator is still usable: a clean gather over it succeeds on every rank
        res, _ = _run_ranks(nranks, lambda r: ranks[r].gather(0))
        assert [x[0] for x in res] == [0] * nranks
        lib.cask_db_close(res[0][1])
    finally:
        for rk in ranks:
            rk.close()


@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_exchange_ranks_fold_equals_replay(fake_rccl, tmp_path, nranks):
    """The key-hash all-to-all over 2-4 ranks: no key is held by two owners, the owners' keydirs
    together are the replay's, and every owner has the replay's Stats and sequence."""
    from cask_amd.cask import Cask
    lib = fake_rccl
    path = str(tmp_path / "db")
    _make_db(path, 60 + nranks, nfiles=5, nkeys=3000)
    want = _want(path)
    ranks = _setup(lib, path, nranks)
    try:
        res, _ = _run_ranks(nranks, lambda r: ranks[r].exchange())
        assert [x[0] for x in res] == [0] * nranks
        kd_all = []
        for rc, kd, sent, got in res:
            with Cask(kd, "") as db:
                k, st, cs = _got(db)
                assert (st, cs) == (want[1], want[2])
                kd_all += k
        assert sorted(kd_all) == want[0]
        own = sum(x[3] for x in res) - sum(x[2] for x in res)  # received = sent by the others + own parts
        assert 0 <= own <= sum(rk.blk.numel() for rk in ranks)
    finally:
        for rk in ranks:
            rk.close()


@pytest.mark.parametrize("case", ["partition", "terms", "fold"])
def test_exchange_failure_on_one_rank_is_agreed(fake_rccl, tmp_path, case):
    """One rank's device partition runs out of memory, one owner cannot read its terms, one owner's
    fold fails: every rank returns that status and none blocks; the communicator stays usable."""
    lib = fake_rccl
    path = str(tmp_path / "db")
    _make_db(path, 70, nfiles=4, nkeys=2000)
    nranks = 3
    inj = {"partition": {1: INJ_PARTITION}, "terms": {0: INJ_TERMS}, "fold": {2: INJ_FOLD}}[case]
    ranks = _setup(lib, path, nranks, inj)
    try:
        res, took = _run_ranks(nranks, lambda r: ranks[r].exchange())
        want = {"partition": -13, "terms": -10, "fold": -13}[case]
        assert [x[0] for x in res] == [want] * nranks
        assert max(took) < TIMEOUT_S / 2, took
        for x in res:
            lib.cask_db_close(x[1])
        res, _ = _run_ranks(nranks, lambda r: ranks[r].exchange())
        assert [x[0] for x in res] == [0] * nranks
        for x in res:
            lib.cask_db_close(x[1])
    finally:
        for rk in ranks:
            rk.close()


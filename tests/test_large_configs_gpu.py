"""BASELINE configs[3] and configs[4] at full size on one MI355X, checked against the C oracle.

configs[3] (compaction merge, 64 x 1,073,741,820 B with 80 % of the records overwritten or deleted):
the files are generated on the device and written to /dev/shm, opened by cask_db_open_multi over two
ranges on the one device and by the product's open (scan, keydir reduced on the device, hint files) —
each keydir's digest, stats and sequence against the oracle's threaded replay —, compacted by the product (cask_db_compact_files) and by the oracle's restatement of
Cask::compact_files_aux (orc_compact_files_fn, cask.rs:451-523) from the same directory before it:
every new data and hint file must be byte-identical (the live region in file order; the tombstone
tail, whose order the reference leaves to a HashMap, in first-seen order on both sides — checked as a
multiset too), and the reopened database's keydir and stats must equal the oracle's replay of the
new files.

configs[4] (256 files over 8 GPUs, one rank's shard = 32 x 1,073,741,820 B of unique keys): two
consecutive shards are scanned on the device, each reduced to its keydir block (cask_shard_keydir),
and the blocks folded in rank order (cask_keydir_merge / _finish); keydir (digest of every entry),
stats and sequence equal the oracle's replay of the 64 files (scan + Index::update split by key
over host threads, orc_replay_parallel).
"""
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu

RPF = 3_702_558  # records of 290 B per 1,073,741,820-B file (configs[1] / configs[3] / configs[4])
THREADS = 16


_T0 = time.time()


_PROGRESS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out",
                         "progress_large_configs.log")


def _say(msg):
    """Progress line on stderr (seen with -s) and appended to gpurun_out/ (seen under pytest's capture):
    the GPU harness kills a command that writes nothing for 3 minutes."""
    line = f"[{time.time() - _T0:7.1f}s] {msg}"
    print(line, file=sys.stderr, flush=True)
    try:
        os.makedirs(os.path.dirname(_PROGRESS), exist_ok=True)
        with open(_PROGRESS, "a") as f:
            f.write(line + "\n")
    except OSError:
        pass


def _beat(label, fn, *args):
    """fn(*args) on a worker thread (ctypes calls drop the GIL) with a progress line every 30 s."""
    import threading
    out = {}

    def run():
        try:
            out["v"] = fn(*args)
        except BaseException as e:  # re-raised on the caller's thread
            out["e"] = e

    t = threading.Thread(target=run, daemon=True)
    t.start()
    while True:
        t.join(30)
        if not t.is_alive():
            break
        _say(f"{label}: running")
    if "e" in out:
        raise out["e"]
    return out["v"]


def _shm_dir(prefix):
    base = "/dev/shm" if os.path.isdir("/dev/shm") else None
    return tempfile.mkdtemp(prefix=prefix, dir=base)


def _digest_of_export(db):
    kb, off, kl, ents = db.export_arrays()
    n = len(kl)
    assert (kl == 16).all() and (off == np.arange(n, dtype=np.uint64) * 16).all()
    keys = kb.reshape(n, 16)
    return O.keydir_digest_np(keys, kl, ents["file_id"], ents["entry_pos"], ents["entry_size"], ents["sequence"]), n


def _stats_rows(db):
    return sorted([fid, *s] for fid, s in db.stats().items())


@pytest.mark.timeout(1800)
def test_cfg3_full_size_compaction_against_oracle(gpu_ctx):
    import torch
    from cask_amd import CaskOptions
    from cask_amd.workloads import variable_file
    ctx = gpu_ctx
    dev = torch.device("cuda", ctx.device)
    nfiles = 64
    n = nfiles * RPF
    g = torch.Generator(device=dev)
    g.manual_seed(0xC0FFEE)
    nkeys = n // 5
    kid = torch.randint(0, nkeys, (n,), generator=g, device=dev, dtype=torch.int64)
    last = torch.full((nkeys,), -1, dtype=torch.int64, device=dev)
    last.scatter_reduce_(0, kid, torch.arange(n, device=dev), reduce="amax")
    present = last >= 0
    tomb_key = (torch.rand(nkeys, generator=g, device=dev) < 0.1) & present
    vsz = torch.full((n,), 256, dtype=torch.int32, device=dev)
    vsz[last[tomb_key]] = -1  # 10 % of the keys end in a tombstone
    live_want = int((present & ~tomb_key).sum().item())
    del last, present, tomb_key
    work = _shm_dir("cask_cfg3_")
    try:
        path = os.path.join(work, "db")
        os.makedirs(path)
        for i in range(nfiles):
            sl = slice(i * RPF, (i + 1) * RPF)
            idx = torch.arange(i * RPF, (i + 1) * RPF, dtype=torch.int64, device=dev)
            ks = torch.full((RPF,), 16, dtype=torch.int16, device=dev)
            f = variable_file(ctx, i + 1, ks, vsz[sl].clone(), idx + 1, kid[sl].clone(), 0xC0FFEE + i)
            f.data.cpu().numpy().tofile(os.path.join(path, f"{i + 1:010}.cask.data"))
            del f
            if i % 8 == 7:
                _say(f"cfg3: wrote {i + 1} files")
        del kid, vsz
        torch.cuda.empty_cache()
        ids = list(range(1, nfiles + 1))
        maps = [np.memmap(os.path.join(path, f"{i:010}.cask.data"), np.uint8, "r") for i in ids]
        # the oracle's keydir (threaded replay), kept for the liveness of its compaction below
        _say("cfg3: oracle replay")
        pix = _beat("cfg3 oracle replay", O.PIndex, maps, ids, THREADS)
        assert pix.result.err_kind == 0 and pix.result.live == live_want
        # cask_db_open_multi over two ranges of the files on this one device (32 x 1 GiB each, read
        # to the device by the pinned ring's threads, rows sized from the record estimate), no hint
        # files written: keydir digest, stats and sequence equal the oracle's
        from cask_amd.keydir import open_multi
        _say("cfg3: open_multi devices=[0, 0]")
        t_m = time.time()
        with _beat("cfg3 open_multi", open_multi, path, [ctx.device, ctx.device],
                   CaskOptions().max_file_size(1 << 30).write_hints(False)) as mdb:
            _say(f"cfg3: open_multi took {time.time() - t_m:.2f} s")
            dg, nk = _beat("cfg3 open_multi digest", _digest_of_export, mdb)
            assert nk == live_want and dg == pix.result.digest
            assert _stats_rows(mdb) == pix.stats
            assert mdb.current_sequence == pix.result.max_seq + 1
        assert not any(f.endswith(".cask.hint") for f in os.listdir(path))
        # the product's open: scan on the device, keydir reduced there (every file scanned), hint
        # files recreated (they must be the oracle's)
        _say("cfg3: product open")
        t_o = time.time()
        with CaskOptions().max_file_size(1 << 30).open(path) as db:
            _say(f"cfg3: open took {time.time() - t_o:.2f} s")
            assert len(db) == live_want
            dg, nk = _beat("cfg3 open digest", _digest_of_export, db)
            assert nk == live_want and dg == pix.result.digest
            assert db.current_sequence == pix.result.max_seq + 1

            def check_hint(i, m):  # (the oracle's C calls drop the GIL: files checked on threads)
                hb = np.fromfile(os.path.join(path, f"{i:010}.cask.hint"), np.uint8)
                body = O.hint_body(m)
                ok = hb[:-4].tobytes() == body.tobytes() and \
                    int.from_bytes(hb[-4:].tobytes(), "little") == O.xxh32(body.tobytes())
                return i, ok

            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(8) as ex:
                for i, ok in ex.map(lambda im: check_hint(*im), zip(ids, maps)):
                    assert ok, i
                    if i % 16 == 0:
                        _say(f"cfg3: hint file {i} checked")
            _say("cfg3: hint files checked")
            # the oracle's compaction of the same files, first
            assert pix.stats == _stats_rows(db)
            want_dir = os.path.join(work, "oracle")
            os.makedirs(want_dir)
            _say("cfg3: oracle compaction")
            r, created = _beat("cfg3 oracle compaction", pix.compact_files, path, want_dir, ids, nfiles, 1 << 30)
            assert r.err_kind == 0 and r.live_records == live_want
            pix.close()
            del maps
            # the product's compaction in place
            _say("cfg3: product compaction")
            rep = _beat("cfg3 product compaction", db.compact_files, ids)
            assert rep["live_records"] == live_want and rep["tombstones"] == r.tombstones
            assert len(db) == live_want
        # every file the compaction created: same ids, same bytes (the live records in file order;
        # a tombstone tail that differs in order only is compared as a multiset over all files)
        _say("cfg3: comparing files")
        got = sorted(f for f in os.listdir(path) if f.endswith(".cask.data"))
        assert got == sorted(f"{fid:010}.cask.data" for fid, _ in created)
        tomb_a, tomb_b = [], []
        for fid, live in created:
            a = np.fromfile(os.path.join(path, f"{fid:010}.cask.data"), np.uint8)
            b = np.fromfile(os.path.join(want_dir, f"{fid:010}.cask.data"), np.uint8)
            ha = np.fromfile(os.path.join(path, f"{fid:010}.cask.hint"), np.uint8)
            hb = np.fromfile(os.path.join(want_dir, f"{fid:010}.cask.hint"), np.uint8)
            if a.size == b.size and np.array_equal(a, b):
                assert np.array_equal(ha, hb), fid
                continue
            assert a.size == b.size, fid
            for buf, acc in ((a, tomb_a), (b, tomb_b)):
                rows = O.scan(buf)
                assert (rows["status"] == 0).all(), fid
                t = rows[rows["vsz_raw"] == 0xFFFFFFFF]
                acc.extend((buf[int(p) + 18:int(p) + 18 + int(k)].tobytes(), int(q))
                           for p, k, q in zip(t["pos"], t["ksz"], t["seq"]))
            ra, rb = O.scan(a), O.scan(b)
            la, lb = ra[ra["vsz_raw"] != 0xFFFFFFFF], rb[rb["vsz_raw"] != 0xFFFFFFFF]
            assert np.array_equal(la, lb), fid
            end = int(la["pos"][-1]) + 18 + int(la["ksz"][-1]) + int(la["vsz_raw"][-1]) if la.size else 0
            assert np.array_equal(a[:end], b[:end]), fid
        assert sorted(tomb_a) == sorted(tomb_b)
        # reopen (hint fast path): keydir and stats equal the oracle's replay of the new files
        new_ids = sorted(fid for fid, _ in created)
        _say("cfg3: oracle replay of the new files; reopen")
        maps = [np.memmap(os.path.join(path, f"{i:010}.cask.data"), np.uint8, "r") for i in new_ids]
        want, want_stats = _beat("cfg3 oracle replay (new files)", O.replay_parallel, maps, new_ids, THREADS)
        del maps
        assert want.err_kind == 0 and want.live == live_want
        with CaskOptions().max_file_size(1 << 30).open(path) as db:
            dg, nk = _beat("cfg3 export + digest", _digest_of_export, db)
            assert nk == live_want and dg == want.digest
            assert _stats_rows(db) == want_stats
            assert db.current_sequence == want.max_seq + 1
    finally:
        shutil.rmtree(work, ignore_errors=True)


@pytest.mark.timeout(1800)
def test_cfg4_two_rank_shards_fold_against_oracle(gpu_ctx):
    """Two full configs[4] rank shards (cfg5's 290-B record shape), folded in rank order on one
    host — and routed through the key-hash partition (SURVEY §8e's huge-keyspace path): each block
    split on the device into two owners' parts, each owner folding its parts in rank order, Stats
    from the owners' terms — both against the oracle's replay digest."""
    import torch
    from cask_amd.keydir import KeydirFold, partition_device, shard_keydir
    from cask_amd.workloads import CFG2_KSZ, CFG2_VSZ, fixed_file
    ctx = gpu_ctx
    per_rank = 32
    fold = KeydirFold()
    owners = [KeydirFold(), KeydirFold()]
    hosts, ids = [], []
    for rank in range(2):  # ranks 0 and 1 of configs[4]: files 1..32 and 33..64
        files = []
        for i in range(per_rank):
            fid = rank * per_rank + i + 1
            seq0 = 1 + (fid - 1) * RPF
            files.append(fixed_file(ctx, fid, RPF, CFG2_KSZ, CFG2_VSZ, seq0, seq0, 0xC0FFEE + fid))
        torch.cuda.synchronize()
        views = [(f.file_id, f.data) for f in files]
        rows = ctx.alloc_rows(per_rank * RPF + 16)
        res = ctx.scan_device(views, rows)
        assert res.error is None and res.count == per_rank * RPF
        assert int((rows["status"][:res.count] != 0).sum().item()) == 0
        blk = shard_keydir(ctx, views, rows, res.count, res.file_row_offset)
        fold.merge(blk.cpu())
        parts = partition_device(ctx, blk, 2)
        for o in range(2):
            owners[o].merge(parts[o].cpu())
        del parts
        for f in files:
            hosts.append(f.data.cpu().numpy())
            ids.append(f.file_id)
        del files, views, rows, blk, res
        torch.cuda.empty_cache()
        _say(f"cfg4: rank {rank} shard scanned and folded")
    _say("cfg4: oracle replay")
    want, want_stats = _beat("cfg4 oracle replay", O.replay_parallel, hosts, ids, THREADS)
    _say("cfg4: oracle done")
    del hosts
    assert want.err_kind == 0 and want.records == 2 * per_rank * RPF
    db = _beat("cfg4 fold finish", fold.finish)
    _say("cfg4: finished; stats")
    try:
        assert len(db) == want.live == 2 * per_rank * RPF  # unique keys: every record is live
        assert db.current_sequence == want.max_seq + 1
        assert _stats_rows(db) == want_stats
        dg, _ = _beat("cfg4 export + digest", _digest_of_export, db)
        assert dg == want.digest
    finally:
        db.close()
    _say("cfg4: partitioned owners")
    terms = b"".join(f.terms().tobytes() for f in owners)
    dsum, nsum = 0, 0
    for f in owners:
        with _beat("cfg4 owner finish", f.finish_terms, terms) as odb:
            assert odb.current_sequence == want.max_seq + 1
            assert _stats_rows(odb) == want_stats
            dg, n = _beat("cfg4 owner digest", _digest_of_export, odb)
            assert n > 0
            dsum, nsum = (dsum + dg) % (1 << 64), nsum + n
    assert nsum == want.live and dsum == want.digest  # (the digest is a sum over entries)

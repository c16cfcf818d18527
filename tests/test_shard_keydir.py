"""The sharded replay's keydir blocks against the reference's in-order fold, on the CPU:
the restatement of the block (oracle/cask_shard.py) folded by the restatement of rank 0 and by the
native fold (cask_keydir_merge / cask_keydir_finish through the C ABI) must give the single-process
Cask::open keydir, stats and sequence (cask.rs:346-382, 60-90; stats.rs:23-48) for any split of the
files into contiguous shards — stale tombstones and resurrections included."""
import random

import pytest
from hypothesis import given, settings, strategies as st

import cask_ref as R
import cask_shard as S


def _full_fold(files):
    """files: [(file_id, [Row])] in order -> (keydir, stats, max seq) by Index::update."""
    ix = R.Index()
    mx = -1
    for fid, rows in files:
        for r in rows:
            mx = max(mx, r.seq)
            ix.update(r, fid)
    kd = {k: (e.file_id, e.entry_pos, e.entry_size, e.sequence) for k, e in ix.map.items()}
    return kd, {f: tuple(s) for f, s in ix.stats.map.items()}, mx


def _random_files(rng, nfiles, nrec, nkeys, tomb_p, back_p):
    keys = [rng.randbytes(rng.randrange(0, 6)) for _ in range(nkeys)]
    files, seq = [], 1
    for f in range(nfiles):
        rows, pos = [], 0
        for _ in range(rng.randrange(0, nrec)):
            k = rng.choice(keys)
            s = seq if rng.random() > back_p else max(0, seq - rng.randrange(1, 40))
            seq += 1
            if rng.random() < tomb_p:
                r = R.Row(pos=pos, seq=s, ksz=len(k), vsz_raw=R.ENTRY_TOMBSTONE, key=k)
            else:
                r = R.Row(pos=pos, seq=s, ksz=len(k), vsz_raw=rng.randrange(0, 50), key=k)
            pos += r.entry_size
            rows.append(r)
        files.append((f + 1, rows))
    return files


def _blocks(files, cuts):
    out = []
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        part = files[lo:hi]
        out.append(S.shard_block([f for f, _ in part], [(f, r) for f, rows in part for r in rows]))
    return out


@settings(max_examples=300, deadline=None)
@given(st.integers(0, 2 ** 32), st.integers(1, 6), st.integers(1, 4))
def test_shard_fold_equals_in_order_fold(seed, nfiles, nshards):
    rng = random.Random(seed)
    files = _random_files(rng, nfiles, 25, rng.choice([1, 2, 3, 8, 30]), rng.choice([0.0, 0.2, 0.5]),
                          rng.choice([0.0, 0.3]))
    nshards = min(nshards, nfiles)
    cuts = sorted(set([0, nfiles] + rng.sample(range(1, nfiles), nshards - 1) if nfiles > 1 else [0, nfiles]))
    assert S.fold_blocks(_blocks(files, cuts)) == _full_fold(files)


def test_hash_collisions_fold_record_by_record(monkeypatch):
    """Keys whose 64-bit hashes collide are sent whole (kRaw) and folded one record at a time."""
    rng = random.Random(3)
    files = _random_files(rng, 4, 40, 6, 0.3, 0.3)
    monkeypatch.setattr(S, "key_hash", lambda k: len(k) % 2)  # force collisions
    blocks = _blocks(files, [0, 2, 4])
    assert any(rec[0] == S.RAW for b in blocks for rec in S.parse_block(b)[0])
    assert S.fold_blocks(blocks) == _full_fold(files)


def _native_fold(native, blocks):
    import ctypes as C
    from cask_amd.cask import Cask
    lib = native
    h = lib.cask_keydir_new()
    for b in blocks:
        buf = (C.c_uint8 * len(b)).from_buffer_copy(b)
        assert lib.cask_keydir_merge(h, buf, len(b)) == 0
    assert lib.cask_keydir_finish(h) == 0
    db = Cask(h, "")
    kd = {k: (e.file_id, e.entry_pos, e.entry_size, e.sequence) for k, e in db.index().items()}
    out = kd, db.stats(), db.current_sequence - 1
    db.close()
    return out


@pytest.mark.parametrize("threads", [1, 5])
@pytest.mark.parametrize("seed", range(12))
def test_native_fold_matches(native, seed, threads, monkeypatch):
    """threads=5: the merge on threads by keydir table (CASK_PAR_FOLD_MIN=0 forces it)."""
    monkeypatch.setenv("CASK_PAR_FOLD_MIN", "0" if threads > 1 else str(1 << 62))
    monkeypatch.setenv("CASK_HOST_THREADS", str(threads))
    rng = random.Random(100 + seed)
    files = _random_files(rng, 7, 60, rng.choice([2, 10, 50]), 0.25, 0.25)
    want = _full_fold(files)
    for cuts in ([0, 7], [0, 3, 7], [0, 1, 2, 4, 7]):
        got = _native_fold(native, _blocks(files, cuts))
        assert got[0] == want[0] and got[1] == want[1]
        assert got[2] == max(want[2], 0)


def test_native_fold_rejects_bad_blocks(native):
    import ctypes as C
    h = native.cask_keydir_new()
    bad = (C.c_uint8 * 64)()
    assert native.cask_keydir_merge(h, bad, 64) == -10
    native.cask_db_close(h)

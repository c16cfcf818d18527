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


def _native_fold(native, blocks, many=False):
    """many: the blocks in one cask_keydir_merge_many call instead of one cask_keydir_merge each."""
    import ctypes as C
    from cask_amd.cask import Cask
    lib = native
    h = lib.cask_keydir_new()
    bufs = [(C.c_uint8 * len(b)).from_buffer_copy(b) for b in blocks]
    if many:
        ptrs = (C.c_void_p * max(len(bufs), 1))(*[C.addressof(x) for x in bufs])
        lens = (C.c_uint64 * max(len(bufs), 1))(*[len(b) for b in blocks])
        assert lib.cask_keydir_merge_many(h, ptrs, lens, len(bufs)) == 0
    for buf, b in zip(bufs, blocks):
        if many:
            break
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
        for many in (False, True):
            got = _native_fold(native, _blocks(files, cuts), many)
            assert got[0] == want[0] and got[1] == want[1]
            assert got[2] == max(want[2], 0)


def test_native_fold_rejects_bad_blocks(native):
    import ctypes as C
    h = native.cask_keydir_new()
    bad = (C.c_uint8 * 64)()
    assert native.cask_keydir_merge(h, bad, 64) == -10
    native.cask_db_close(h)


# ---- the key-hash partition (huge keyspace): every rank splits its block by key owner,
# owner o folds the parts it gets in rank order, and the owners' terms give the Stats ----

def _partitioned_native_fold(blocks, nparts):
    """Owner by owner: merge part o of every block in order, exchange terms, finish. Returns the
    union of the owners' keydirs, each owner's stats and sequence, and which owner held each key."""
    from cask_amd.keydir import KeydirFold, partition_host
    parts = [partition_host(b, nparts) for b in blocks]
    folds = [KeydirFold() for _ in range(nparts)]
    for o in range(nparts):
        for p in parts:
            folds[o].merge(p[o])
    terms = b"".join(f.terms().tobytes() for f in folds)
    kd, stats, seqs, where = {}, [], [], {}
    for o, f in enumerate(folds):
        db = f.finish_terms(terms)
        for k, e in db.index().items():
            assert k not in kd
            kd[k] = (e.file_id, e.entry_pos, e.entry_size, e.sequence)
            where[k] = o
        stats.append(db.stats())
        seqs.append(db.current_sequence - 1)
        db.close()
    return kd, stats, seqs, where


@settings(max_examples=200, deadline=None)
@given(st.integers(0, 2 ** 32), st.integers(1, 6), st.integers(1, 4), st.integers(1, 7))
def test_partition_native_matches_restatement(native, seed, nfiles, nshards, nparts):
    """cask_keydir_partition_host byte for byte the restatement (oracle/cask_shard.py partition_block)."""
    rng = random.Random(seed)
    files = _random_files(rng, nfiles, 25, rng.choice([1, 3, 30]), 0.3, 0.3)
    nshards = min(nshards, nfiles)
    cuts = sorted(set([0, nfiles] + rng.sample(range(1, nfiles), nshards - 1) if nfiles > 1 else [0, nfiles]))
    from cask_amd.keydir import key_owner, partition_host
    for b in _blocks(files, cuts):
        got = [bytes(p) for p in partition_host(b, nparts)]
        assert got == S.partition_block(b, nparts)
        for o, p in enumerate(got):  # every record of part o is owned by o
            for rec in S.parse_block(p)[0]:
                assert key_owner(rec[6], nparts) == o == S.key_owner(rec[6], nparts)


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
@pytest.mark.parametrize("seed", range(10))
def test_partitioned_fold_equals_in_order_fold(native, seed, nparts):
    """The owners together hold exactly the single-process keydir, each key on its owner, and every
    owner has the whole replay's Stats and sequence — stale tombstones across shards included."""
    from cask_amd.keydir import key_owner
    rng = random.Random(500 + seed)
    files = _random_files(rng, 7, 60, rng.choice([2, 10, 50, 400]), rng.choice([0.1, 0.3]), 0.25)
    want = _full_fold(files)
    for cuts in ([0, 7], [0, 3, 7], [0, 1, 2, 4, 7]):
        kd, stats, seqs, where = _partitioned_native_fold(_blocks(files, cuts), nparts)
        assert kd == want[0]
        assert all(s == want[1] for s in stats)
        assert all(q == max(want[2], 0) for q in seqs)
        assert all(key_owner(k, nparts) == o for k, o in where.items())


def test_partition_rejects_bad_blocks(native):
    import ctypes as C
    off = (C.c_uint64 * 3)()
    bad = (C.c_uint8 * 64)()
    assert native.cask_keydir_partition_host(bad, 64, 2, None, 0, off) == -10
    blk = S.shard_block([1], [(1, R.Row(pos=0, seq=1, ksz=3, vsz_raw=5, key=b"abc"))])
    buf = (C.c_uint8 * len(blk)).from_buffer_copy(blk)
    assert native.cask_keydir_partition_host(buf, len(blk), 0, None, 0, off) == -10
    assert native.cask_keydir_partition_host(buf, len(blk), 2, None, 0, off) == -12  # size asked
    assert off[2] == sum(len(p) for p in S.partition_block(blk, 2))
    h = native.cask_keydir_new()
    assert native.cask_keydir_finish_terms(h, None, 3) == -10  # not a whole number of terms
    native.cask_db_close(h)


@pytest.mark.parametrize("threads", [1, 8])
def test_native_fold_grows_tables(native, threads, monkeypatch):
    """Enough keys that every keydir table grows several times — from the first block's sizing, then
    on demand in the later blocks (tables that hold keys grow only when they fill) — with deletions
    and resurrections leaving deleted slots behind (rebuilds at the same size) and keys longer than
    the 16 inline bytes (the arena): the native merge equals the in-order fold."""
    monkeypatch.setenv("CASK_PAR_FOLD_MIN", "0" if threads > 1 else str(1 << 62))
    monkeypatch.setenv("CASK_HOST_THREADS", str(threads))
    rng = random.Random(4242)
    keys = [rng.randbytes(rng.randrange(0, 31)) for _ in range(60000)]
    files, seq = [], 1
    for f in range(5):
        rows, pos = [], 0
        lo = 12000 * f  # each file mostly new keys, some of every earlier file's
        for _ in range(30000):
            k = keys[rng.randrange(lo, lo + 12000)] if rng.random() < 0.7 else keys[rng.randrange(0, lo + 12000)]
            s = seq if rng.random() > 0.1 else max(0, seq - rng.randrange(1, 5000))
            seq += 1
            vsz = R.ENTRY_TOMBSTONE if rng.random() < 0.3 else rng.randrange(0, 50)
            r = R.Row(pos=pos, seq=s, ksz=len(k), vsz_raw=vsz, key=k)
            pos += r.entry_size
            rows.append(r)
        files.append((f + 1, rows))
    want = _full_fold(files)
    assert len(want[0]) > 20000
    for cuts, many in (([0, 5], False), ([0, 1, 2, 3, 4, 5], False), ([0, 1, 2, 3, 4, 5], True)):
        got = _native_fold(native, _blocks(files, cuts), many)
        assert got[0] == want[0] and got[1] == want[1]
        assert got[2] == max(want[2], 0)

"""Compaction merge (Cask::compact / compact_files / compact_files_aux, cask.rs:451-642).

CPU tests pin the Python restatement (oracle/cask_ref.py compact_files) by properties the
reference guarantees: the live keydir survives compaction (same keys, sequences and values), the
tombstones of absent keys are carried over, the new files re-open to the same keydir, and the
LogWriter rollover (log.rs:282-306) bounds every new file. The reference has no compaction test
of its own, so byte-level parity is "parity unpinned" beyond these properties.

GPU tests run the engine (cask_db_compact_files: hint liveness on the host, live records verified
by the device scan and copied by the device gather) against the restatement on a copy of the same
directory and require identical bytes in every file left on disk, identical keydir, stats and file
list, and the same error for corrupt or truncated live records.
"""
import os
import random
import shutil

import pytest

import cask_ref as R


def _workload(rng, n, nkeys, del_p=0.15, vmax=300):
    keys = [rng.randbytes(rng.randrange(1, 24)) for _ in range(nkeys)]
    ents = []
    for i in range(n):
        k = rng.choice(keys)
        if rng.random() < del_p:
            ents.append(R.entry_deleted(i + 1, k))
        else:
            ents.append(R.entry_new(i + 1, k, rng.randbytes(rng.randrange(0, vmax))))
    return ents


def _live_values(path, db):
    """key -> (sequence, value) of every live key, read back through read_entry."""
    out = {}
    for k, ie in db.index.map.items():
        e = R.read_entry(path, ie.file_id, ie.entry_pos)
        assert e.key == k and e.sequence == ie.sequence and not e.deleted
        out[k] = (e.sequence, e.value)
    return out


def _dir_bytes(path):
    out = {}
    for name in sorted(os.listdir(path)):
        if name.endswith(".cask.data") or name.endswith(".cask.hint"):
            with open(os.path.join(path, name), "rb") as f:
                out[name] = f.read()
    return out


# ----------------------------------------------------------------------------- oracle (CPU)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_compaction_preserves_live_keydir(tmp_path, seed):
    rng = random.Random(seed)
    path = str(tmp_path / "db")
    R.write_log(path, _workload(rng, 3000, 400), max_file_size=64 << 10)
    db = R.replay(path)
    before = _live_values(path, db)
    absent = {}
    for fid in db.files:
        for h in R.parse_hints(R._valid_hints(path, fid)):
            if h.deleted and h.key not in db.index.map:
                absent[h.key] = max(absent.get(h.key, 0), h.seq)
    files_before = list(db.files)
    compacted, new_files = R.compact_files(path, db, files_before, 64 << 10)
    assert compacted == files_before
    assert all(f > files_before[-1] for f in new_files)
    assert db.files == new_files
    assert _live_values(path, db) == before
    # every new data file respects the rollover bound (log.rs:286-289)
    for f in R.find_data_files(path):
        assert os.path.getsize(R.data_file_path(path, f)) <= 64 << 10
    # the compacted files are gone; re-open gives the same live keydir
    db2 = R.replay(path)
    assert {k: v.sequence for k, v in db2.index.map.items()} == {k: s for k, (s, _) in before.items()}
    # the tombstones of keys absent from the index were written, with their highest sequence
    tomb = {}
    for f in R.find_data_files(path):
        for r in R.scan_entries(open(R.data_file_path(path, f), "rb").read()):
            assert r.status == R.ROW_OK
            if r.deleted:
                tomb[r.key] = r.seq
    assert tomb == absent


def test_oracle_compaction_skips_files_without_hints(tmp_path):
    rng = random.Random(4)
    path = str(tmp_path / "db")
    files = R.write_log(path, _workload(rng, 800, 100), max_file_size=16 << 10)
    db = R.replay(path)  # writes nothing new: every file has a valid hint file
    os.remove(R.hint_file_path(path, files[1]))
    compacted, _ = R.compact_files(path, db, files, 16 << 10)
    assert files[1] not in compacted and files[1] in db.files
    assert os.path.exists(R.data_file_path(path, files[1]))


def test_oracle_compaction_checksum_error(tmp_path):
    path = str(tmp_path / "db")
    ents = [R.entry_new(i + 1, b"k%d" % i, b"v" * 40) for i in range(50)]
    R.write_log(path, ents, max_file_size=1 << 20)
    db = R.replay(path)
    ie = db.index.map[b"k7"]
    with open(R.data_file_path(path, ie.file_id), "r+b") as f:
        f.seek(ie.entry_pos + 30)
        f.write(b"X")
    with pytest.raises(R.CaskError) as ei:
        R.compact_files(path, db, list(db.files), 1 << 20)
    assert ei.value.kind == "checksum" and ei.value.pos == ie.entry_pos


def test_oracle_compact_select_defaults(tmp_path):
    """compact(): a file at >= 60 % fragmentation triggers; >= 40 % or <= 10 MiB joins."""
    path = str(tmp_path / "db")
    ents = [R.entry_new(i + 1, b"a%d" % (i % 10), b"x" * 10) for i in range(100)]  # 90 % dead
    R.write_log(path, ents, max_file_size=1 << 20)
    db = R.replay(path)
    trig, files = R.compact_select(path, db)
    assert trig and files == [1]
    ents = [R.entry_new(i + 1, b"u%d" % i, b"x") for i in range(10)]
    p2 = str(tmp_path / "db2")
    R.write_log(p2, ents, max_file_size=1 << 20)
    db2 = R.replay(p2)
    trig, files = R.compact_select(p2, db2)
    assert not trig and files == [1]  # small file, no trigger


# ----------------------------------------------------------------------------- engine, hint path (CPU)
@pytest.mark.parametrize("threads", [1, 3, 16])
@pytest.mark.parametrize("seed", [31, 32])
def test_engine_open_from_hints_matches_oracle(native, tmp_path, seed, threads, monkeypatch):
    """Every data file has a valid hint file, so Cask::open folds hints only (log.rs:121-135) and
    no device is needed: the keydir fold (Index::update + Stats, cask.rs:60-90) on 1, 3 and 16 host
    threads, split by key hash, against the restatement's replay."""
    from cask_amd import CaskOptions
    monkeypatch.setenv("CASK_PAR_FOLD_MIN", "0")
    monkeypatch.setenv("CASK_HOST_THREADS", str(threads))
    rng = random.Random(seed)
    path, ref = _both(tmp_path, _workload(rng, 20000, 1500, del_p=0.2), 32 << 10)
    rdb = R.replay(ref)
    with CaskOptions().max_file_size(32 << 10).open(path) as db:
        assert db.files() == rdb.files
        assert db.stats() == {f: tuple(s) for f, s in rdb.index.stats.map.items()}
        got = db.index()
        assert len(got) == len(rdb.index.map) == len(db)
        for k, v in rdb.index.map.items():
            e = got[k]
            assert (e.file_id, e.entry_pos, e.entry_size, e.sequence) == (v.file_id, v.entry_pos, v.entry_size,
                                                                           v.sequence)


def test_engine_open_bad_hint_body(native, tmp_path):
    """A hint file whose trailer checks but whose body ends inside a record: open() fails with the
    reference's UnexpectedEof (Hint::from_read's read_exact, data.rs:258-276), as the restatement's
    replay does."""
    from cask_amd import CaskOptions
    from cask_amd.errors import UnexpectedEof
    rng = random.Random(5)
    path = str(tmp_path / "db")
    files = R.write_log(path, _workload(rng, 500, 50), max_file_size=8 << 10)
    hp = R.hint_file_path(path, files[1])
    body = open(hp, "rb").read()[:-4][:-3]  # cut the last hint short
    with open(hp, "wb") as f:
        f.write(body + R.xxhash32(body).to_bytes(4, "little"))
    ref = str(tmp_path / "ref")
    shutil.copytree(path, ref)
    rerr = R.replay(ref).error
    with pytest.raises(UnexpectedEof) as ei:
        CaskOptions().open(path)
    assert rerr.kind == "eof" and ei.value.file_id == rerr.file_id == files[1]


# ----------------------------------------------------------------------------- engine (GPU)
def _both(tmp_path, ents, max_file_size, drop_hints=()):
    path = str(tmp_path / "db")
    R.write_log(path, ents, max_file_size=max_file_size)
    for f in drop_hints:
        os.remove(R.hint_file_path(path, f))
    ref = str(tmp_path / "ref")
    shutil.copytree(path, ref)
    return path, ref


def _check_same(native_db, path, ref_db, ref):
    assert native_db.files() == ref_db.files
    assert native_db.stats() == {f: tuple(s) for f, s in ref_db.index.stats.map.items()}
    got = native_db.index()
    assert len(got) == len(ref_db.index.map)
    for k, v in ref_db.index.map.items():
        e = got[k]
        assert (e.file_id, e.entry_pos, e.entry_size, e.sequence) == (v.file_id, v.entry_pos, v.entry_size,
                                                                       v.sequence)
    assert _dir_bytes(path) == _dir_bytes(ref)


@pytest.mark.gpu
@pytest.mark.parametrize("threads", [False, True], ids=["serial", "threaded"])
@pytest.mark.parametrize("seed,mfs", [(11, 64 << 10), (12, 1 << 20), (13, 4 << 10)])
def test_engine_compact_files_matches_oracle(native, tmp_path, seed, mfs, threads, monkeypatch):
    """threaded: the open fold sharded by key hash and the liveness lookups on threads
    (CASK_PAR_FOLD_MIN=0), and every device-to-host copy staged through the pinned ring on threads
    (CASK_STAGE_MIN=0), against the same oracle."""
    from cask_amd import CaskOptions
    monkeypatch.setenv("CASK_PAR_FOLD_MIN", "0" if threads else str(1 << 62))
    if threads:
        monkeypatch.setenv("CASK_STAGE_MIN", "0")
    rng = random.Random(seed)
    path, ref = _both(tmp_path, _workload(rng, 6000, 700, vmax=500), mfs)
    rdb = R.replay(ref)
    with CaskOptions().max_file_size(mfs).open(path) as db:
        files = db.files()
        rep = db.compact_files(files)
        rc, rn = R.compact_files(ref, rdb, files, mfs)
        assert rep["compacted"] == len(rc) and rep["new_files"] == len(rn)
        _check_same(db, path, rdb, ref)
        # a second compaction continues the file-id sequence
        files2 = db.files()
        db.compact_files(files2[: max(1, len(files2) // 2)])
        R.compact_files(ref, rdb, files2[: max(1, len(files2) // 2)], mfs)
        _check_same(db, path, rdb, ref)
    with CaskOptions().max_file_size(mfs).open(path) as db:  # the result re-opens
        assert {k: e.sequence for k, e in db.index().items()} == {k: v.sequence for k, v in rdb.index.map.items()}
    # the compacted files were renamed out of the data-file names at once and unlinked by the db's
    # reclaim thread, which the close joins: nothing but the database's own files is left
    left = sorted(f for f in os.listdir(path) if f != "cask.lock")
    assert left == sorted(os.listdir(ref)), (left, sorted(os.listdir(ref)))


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [1, 100_000, 300_000])
def test_engine_compact_many_batches_matches_oracle(native, tmp_path, batch, monkeypatch):
    """Source batches of ~`batch` bytes (test hook; a batch holds at least one source file), so the
    writer thread takes several batches while the next ones are copied and verified, and the
    rollover runs across batch boundaries: files, stats and keydir equal the oracle's."""
    from cask_amd import CaskOptions
    monkeypatch.setenv("CASK_COMPACT_BATCH", str(batch))
    rng = random.Random(51)
    path, ref = _both(tmp_path, _workload(rng, 8000, 900, vmax=400), 64 << 10)
    rdb = R.replay(ref)
    with CaskOptions().max_file_size(64 << 10).open(path) as db:
        files = db.files()
        assert len(files) >= 6
        rep = db.compact_files(files)
        rc, rn = R.compact_files(ref, rdb, files, 64 << 10)
        assert rep["compacted"] == len(rc) and rep["new_files"] == len(rn)
        _check_same(db, path, rdb, ref)


@pytest.mark.gpu
def test_engine_compact_into_many_output_files(native, tmp_path, monkeypatch):
    """Over a hundred output files placed while the writer thread finishes earlier ones (4-KiB
    files, small source batches): placement appends to the output list as the writer works through
    the batch before, which must not disturb the files the writer holds. Files, stats and keydir
    equal the oracle's."""
    from cask_amd import CaskOptions
    monkeypatch.setenv("CASK_COMPACT_BATCH", "40000")
    rng = random.Random(77)
    mfs = 4 << 10
    path, ref = _both(tmp_path, _workload(rng, 9000, 3000, vmax=400), mfs)
    rdb = R.replay(ref)
    with CaskOptions().max_file_size(mfs).open(path) as db:
        files = db.files()
        rep = db.compact_files(files)
        rc, rn = R.compact_files(ref, rdb, files, mfs)
        assert rep["compacted"] == len(rc) and rep["new_files"] == len(rn)
        assert len(rn) >= 100, len(rn)
        _check_same(db, path, rdb, ref)


@pytest.mark.gpu
def test_engine_compact_failure_in_a_later_batch(native, tmp_path, monkeypatch):
    """A checksum failure in the last source file, with one file per batch: the earlier batches
    were already handed to the writer thread; the error is the reference's and every file the call
    created is removed again."""
    from cask_amd import CaskOptions, errors
    monkeypatch.setenv("CASK_COMPACT_BATCH", "1")
    rng = random.Random(52)
    path, ref = _both(tmp_path, _workload(rng, 6000, 3000, del_p=0.0), 64 << 10)
    rdb = R.replay(ref)
    files = sorted(rdb.files)
    fl = files[-1]
    live = min((v for v in rdb.index.map.values() if v.file_id == fl), key=lambda v: v.entry_pos)
    for p in (path, ref):
        with open(R.data_file_path(p, fl), "r+b") as f:
            f.seek(live.entry_pos + 18)
            b = f.read(1)
            f.seek(live.entry_pos + 18)
            f.write(bytes([b[0] ^ 0x0F]))
    with pytest.raises(R.CaskError) as want:
        R.compact_files(ref, rdb, files, 64 << 10)
    with CaskOptions().max_file_size(64 << 10).open(path) as db:
        before = set(os.listdir(path))
        with pytest.raises(errors.InvalidChecksum) as got:
            db.compact_files(db.files())
        assert set(os.listdir(path)) == before
        assert db.files() == files  # (nothing was swapped)
    assert (got.value.file_id, got.value.pos, got.value.expected, got.value.found) == \
        (want.value.file_id, want.value.pos, want.value.expected, want.value.found)


@pytest.mark.gpu
def test_engine_compact_subset_and_missing_hints(native, tmp_path):
    from cask_amd import CaskOptions
    rng = random.Random(21)
    ents = _workload(rng, 4000, 300)
    path = str(tmp_path / "db")
    files = R.write_log(path, ents, max_file_size=32 << 10)
    ref = str(tmp_path / "ref")
    shutil.copytree(path, ref)
    rdb = R.replay(ref)
    with CaskOptions().max_file_size(32 << 10).open(path) as db:
        os.remove(R.hint_file_path(path, files[2]))
        os.remove(R.hint_file_path(ref, files[2]))
        sel = [files[0], files[2], files[3], files[-2]]
        db.compact_files(sel)
        R.compact_files(ref, rdb, sel, 32 << 10)
        _check_same(db, path, rdb, ref)


@pytest.mark.gpu
def test_engine_compact_corrupt_live_record(native, tmp_path):
    from cask_amd import CaskOptions, errors
    rng = random.Random(31)
    path, ref = _both(tmp_path, _workload(rng, 2000, 200), 64 << 10)
    rdb = R.replay(ref)
    k = sorted(rdb.index.map)[5]
    ie = rdb.index.map[k]
    for p in (path, ref):
        with open(R.data_file_path(p, ie.file_id), "r+b") as f:
            f.seek(ie.entry_pos + 18)
            b = f.read(1)
            f.seek(ie.entry_pos + 18)
            f.write(bytes([b[0] ^ 0x55]))
    with pytest.raises(R.CaskError) as want:
        R.compact_files(ref, rdb, list(rdb.files), 64 << 10)
    with CaskOptions().max_file_size(64 << 10).open(path) as db:
        with pytest.raises(errors.InvalidChecksum) as got:
            db.compact_files(db.files())
    assert (got.value.file_id, got.value.pos, got.value.expected, got.value.found) == \
        (want.value.file_id, want.value.pos, want.value.expected, want.value.found)


@pytest.mark.gpu
def test_engine_compact_truncated_live_record(native, tmp_path):
    from cask_amd import CaskOptions, errors
    rng = random.Random(32)
    path, ref = _both(tmp_path, _workload(rng, 2000, 200, del_p=0.0), 1 << 20)
    rdb = R.replay(ref)
    # the live record furthest into file 1: truncate the data file inside it (hints stay valid)
    last = max((v for v in rdb.index.map.values() if v.file_id == 1), key=lambda v: v.entry_pos)
    for p in (path, ref):
        os.truncate(R.data_file_path(p, 1), last.entry_pos + 10)
    with pytest.raises(R.CaskError) as want:
        R.compact_files(ref, rdb, [1], 1 << 20)
    assert want.value.kind == "eof"
    with CaskOptions().write_hints(False).open(path) as db:
        pass  # hints are valid: open trusts them and never scans the truncated file
    with CaskOptions().max_file_size(1 << 20).open(path) as db:
        with pytest.raises(errors.UnexpectedEof) as got:
            db.compact_files([1])
    assert (got.value.file_id, got.value.pos) == (want.value.file_id, want.value.pos)


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["checksum_first", "eof_first"])
def test_engine_compact_first_failure_in_write_order(native, tmp_path, order):
    """A live record whose checksum fails and a live record cut short by its file's end, in two
    files of one batch: the error is the one met first in write order (file order, then hint
    order), as the reference's loop meets it — the EOF comes from the host's pass over the mapped
    source, the checksum from the device."""
    from cask_amd import CaskOptions, errors
    rng = random.Random(41)
    path, ref = _both(tmp_path, _workload(rng, 6000, 3000, del_p=0.0), 64 << 10)
    rdb = R.replay(ref)
    files = sorted(rdb.files)
    assert len(files) >= 4
    fa, fb = (files[1], files[3]) if order == "checksum_first" else (files[3], files[1])
    live_a = min((v for v in rdb.index.map.values() if v.file_id == fa), key=lambda v: v.entry_pos)
    last_b = max((v for v in rdb.index.map.values() if v.file_id == fb), key=lambda v: v.entry_pos)
    for p in (path, ref):
        with open(R.data_file_path(p, fa), "r+b") as f:  # a key byte of fa's first live record
            f.seek(live_a.entry_pos + 18)
            b = f.read(1)
            f.seek(live_a.entry_pos + 18)
            f.write(bytes([b[0] ^ 0x55]))
        os.truncate(R.data_file_path(p, fb), last_b.entry_pos + 10)  # inside fb's last live record
    with pytest.raises(R.CaskError) as want:
        R.compact_files(ref, rdb, files, 64 << 10)
    assert want.value.kind == ("checksum" if order == "checksum_first" else "eof")
    with CaskOptions().max_file_size(64 << 10).open(path) as db:  # (valid hints: nothing is scanned)
        before = set(os.listdir(path))
        with pytest.raises((errors.InvalidChecksum, errors.UnexpectedEof)) as got:
            db.compact_files(db.files())
        assert set(os.listdir(path)) == before  # the files this call created are gone again
    assert isinstance(got.value, errors.InvalidChecksum if want.value.kind == "checksum" else errors.UnexpectedEof)
    assert (got.value.file_id, got.value.pos) == (want.value.file_id, want.value.pos)
    if want.value.kind == "checksum":
        assert (got.value.expected, got.value.found) == (want.value.expected, want.value.found)


@pytest.mark.gpu
def test_engine_compact_missing_data_file_is_io(native, tmp_path):
    """A compacted file whose hint file is there but whose data file is not: File::open fails in
    Log::read_entry (log.rs:150-166), an Io error naming that file; nothing is left behind."""
    from cask_amd import CaskOptions, errors
    rng = random.Random(42)
    path, _ = _both(tmp_path, _workload(rng, 3000, 1500, del_p=0.0), 64 << 10)
    with CaskOptions().max_file_size(64 << 10).open(path) as db:
        files = db.files()
        os.remove(os.path.join(path, "%010d.cask.data" % files[2]))
        before = set(os.listdir(path))
        with pytest.raises(errors.Io) as got:
            db.compact_files(files)
        assert set(os.listdir(path)) == before
    assert got.value.file_id == files[2]


@pytest.mark.gpu
def test_engine_compact_trigger(native, tmp_path):
    from cask_amd import CaskOptions
    ents = [R.entry_new(i + 1, b"a%d" % (i % 10), b"x" * 10) for i in range(100)]
    ents += [R.entry_deleted(101, b"a3")]
    path, ref = _both(tmp_path, ents, 1 << 20)
    rdb = R.replay(ref)
    trig, sel = R.compact_select(ref, rdb)
    assert trig
    R.compact_files(ref, rdb, sel, 1 << 20)
    with CaskOptions().max_file_size(1 << 20).open(path) as db:
        rep = db.compact()
        assert rep is not None and rep["compacted"] == len(sel)
        _check_same(db, path, rdb, ref)
        assert db.compact() is None  # the new file has no dead entries and no trigger fires


@pytest.mark.gpu
def test_device_memory_flat_over_repeated_open_compact(native, tmp_path):
    """Round-1 advice: contexts and per-open buffers must not leak HBM. The engine keeps one
    context and its buffers per device for the process (sized to the largest open so far), so
    after the first open + compaction, repeating them leaves free device memory where it was; a
    ScanContext created and destroyed in a loop gives back what it took."""
    import torch
    from cask_amd import CaskOptions, ScanContext
    rng = random.Random(31)
    path = str(tmp_path / "db")
    R.write_log(path, _workload(rng, 20000, 3000), max_file_size=256 << 10, write_hints=False)

    def cycle():
        for f in os.listdir(path):  # every open scans (no hint files), every compaction rewrites
            if f.endswith(".cask.hint"):
                os.remove(os.path.join(path, f))
        with CaskOptions().max_file_size(256 << 10).open(path) as db:
            db.compact_files(db.files())
        torch.cuda.synchronize()

    cycle()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(4):
        cycle()
    assert abs(torch.cuda.mem_get_info()[0] - free0) < (64 << 20)
    x = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")  # ScanContext scratch is per context
    for _ in range(5):
        ctx = ScanContext(0)
        ctx.scan_device([(1, x)])
        ctx.close()
    torch.cuda.synchronize()
    assert abs(torch.cuda.mem_get_info()[0] - free0) < (64 << 20)

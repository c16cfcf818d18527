"""Pin the CPU oracle before trusting it (CPU only).

* XXH32 (oracle/cask_oracle.c) against libxxhash 0.8.2 values in tests/golden/kat.json and the
  published XXH32 test values; streaming in any split equals one-shot (data.rs:102-108 vs :83).
* The reference's own test_serialization / test_deleted (data.rs:285-327).
* The C oracle and the independent Python restatement (oracle/cask_ref.py) reproduce every
  golden fixture: scan rows, recreated hint bytes, keydir, stats, sequence, first error.
"""
import json
import os
import random
import shutil

import numpy as np
import pytest

from conftest import GOLDEN, golden_cases

import cask_ref as R
import oracle_ffi as O


def load_kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def kat_bytes(spec: str) -> bytes:
    if spec.startswith("pattern:"):
        n = int(spec.split(":")[1])
        return bytes((i * 7 + 3) & 0xFF for i in range(n))
    return bytes.fromhex(spec)


def test_xxh32_published_values(oracle_lib):
    # XXH32 seed 0 values from the xxHash specification / reference implementation
    assert O.xxh32(b"") == 0x02CC5D05
    assert O.xxh32(b"a") == 0x550D7456
    assert O.xxh32(b"abc") == 0x32D153FF


def test_xxh32_kat(oracle_lib):
    for spec, want in load_kat()["xxh32"]:
        data = kat_bytes(spec)
        assert O.xxh32(data) == want, spec[:40]
        assert R.xxhash32(data) == want


def test_xxh32_streaming_equals_oneshot(oracle_lib):
    rng = random.Random(7)
    for n in [0, 1, 3, 15, 16, 17, 31, 32, 33, 100, 1000]:
        data = bytes(rng.getrandbits(8) for _ in range(n))
        for cuts in [(0,), (n // 2,), (14, 17), (1, 2, 3)]:
            h = R.XxHash32()
            last = 0
            for c in cuts:
                c = min(c, n)
                h.update(data[last:c])
                last = c
            h.update(data[last:])
            assert h.get() == O.xxh32(data)


def test_reference_serialization(oracle_lib):
    """data.rs:285-318: 24-byte live record, round trips; tombstone has no value bytes."""
    k = load_kat()["test_serialization"]
    live = O.entry_encode(0, b"\0\0\0", b"\0\0\0")
    assert len(live) == 24
    assert live.hex() == k["live_to_bytes"] == k["live_write_bytes"]
    dead = O.entry_encode(0, b"\0\0\0", b"", deleted=True)
    assert len(dead) == 21
    assert dead.hex() == k["deleted_to_bytes"] == k["deleted_write_bytes"]
    rows = O.scan(live + dead)
    assert [int(r["status"]) for r in rows] == [0, 0]
    assert int(rows[1]["vsz_raw"]) == 0xFFFFFFFF and int(rows[1]["pos"]) == 24


def test_reference_deleted():
    """data.rs:320-327."""
    e = R.entry_deleted(0, b"\0\0\0")
    assert e.deleted and len(e.value) == 0


def _file_bytes(case, fid):
    with open(R.data_file_path(os.path.join(GOLDEN, case), fid), "rb") as f:
        return f.read()


def _expected(case):
    with open(os.path.join(GOLDEN, case, "expected.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", golden_cases())
def test_c_oracle_rows(oracle_lib, case):
    exp = _expected(case)
    for fe in exp["files"]:
        buf = _file_bytes(case, fe["file_id"])
        assert len(buf) == fe["len"]
        rows = O.scan(buf)
        got = [[int(r["pos"]), int(r["seq"]), int(r["ksz"]), int(r["vsz_raw"]), int(r["status"]),
                int(r["expected"]), int(r["found"])] for r in rows]
        assert got == fe["rows"]
        assert O.hint_file_bytes(buf, rows).hex() == fe["recreated_hint_hex"]


@pytest.mark.parametrize("case", golden_cases())
def test_python_restatement_rederives_fixture(case, tmp_path):
    exp = _expected(case)
    for fe in exp["files"]:
        rows = R.scan_entries(_file_bytes(case, fe["file_id"]))
        assert [[r.pos, r.seq, r.ksz, r.vsz_raw, r.status, r.expected, r.found] for r in rows] == fe["rows"]
    d = tmp_path / case
    shutil.copytree(os.path.join(GOLDEN, case), d)
    os.remove(d / "expected.json")
    res = R.replay(str(d))
    rep = exp["replay"]
    assert res.sequence == rep["sequence"]
    if rep["error"] is None:
        assert res.error is None
        assert sorted([k.hex(), v.file_id, v.entry_pos, v.entry_size, v.sequence]
                      for k, v in res.index.map.items()) == rep["keydir"]
        assert sorted([f, *s] for f, s in res.index.stats.map.items()) == rep["stats"]
    else:
        e = res.error
        assert {"kind": e.kind, "file_id": e.file_id, "pos": e.pos, "expected": e.expected,
                "found": e.found} == rep["error"]
    for fid, hx in rep["hint_files_after"].items():
        with open(R.hint_file_path(str(d), int(fid)), "rb") as f:
            assert f.read().hex() == hx


@pytest.mark.parametrize("case", [c for c in golden_cases() if not c.startswith("hints")])
def test_c_oracle_fold_matches_replay(oracle_lib, case):
    """C Index::update + Stats over the scan rows == the fixture's replay (scan path only)."""
    exp = _expected(case)
    rep = exp["replay"]
    ix = O.Index()
    seq = 0
    err = None
    for fe in exp["files"]:
        buf = _file_bytes(case, fe["file_id"])
        rows = O.scan(buf)
        for r in rows:
            if int(r["status"]) != 0:
                err = (fe["file_id"], int(r["pos"]))
                break
            seq = max(seq, int(r["seq"]))
            p, k = int(r["pos"]), int(r["ksz"])
            ix.update(buf[p + 18:p + 18 + k], fe["file_id"], p, int(r["vsz_raw"]), int(r["seq"]))
        if err:
            break
    assert seq == rep["sequence"]
    if rep["error"] is None:
        assert err is None
        assert ix.export() == rep["keydir"]
        assert ix.stats() == rep["stats"]
    else:
        assert err == (rep["error"]["file_id"], rep["error"]["pos"])


@pytest.mark.parametrize("case", ["basic", "multi_file", "corrupt_value", "truncated_value", "edge_sizes"])
def test_c_oracle_faithful_replay(oracle_lib, case, tmp_path):
    """The timed CPU baseline (read(2)/write(2) replay) reproduces the fixture and hint bytes."""
    exp = _expected(case)
    rep = exp["replay"]
    ix = O.Index()
    seq = 0
    err = None
    for fe in exp["files"]:
        hp = str(tmp_path / f"{fe['file_id']}.hint")
        r = O.replay_faithful(R.data_file_path(os.path.join(GOLDEN, case), fe["file_id"]), hp, fe["file_id"], ix)
        seq = max(seq, int(r.max_seq))
        with open(hp, "rb") as f:  # on a failing file too: RecreateHints::drop drains (log.rs:466-470)
            assert f.read().hex() == fe["recreated_hint_hex"]
        if r.err_kind:
            err = {"kind": {1: "checksum", 2: "eof"}[r.err_kind], "file_id": int(r.err_file_id),
                   "pos": int(r.err_pos), "expected": int(r.err_expected), "found": int(r.err_found)}
            break
    assert seq == rep["sequence"]
    if rep["error"] is None:
        assert err is None
        assert ix.export() == rep["keydir"]
        assert ix.stats() == rep["stats"]
    else:
        if rep["error"]["kind"] == "eof":
            rep["error"]["expected"] = 0
        assert err == rep["error"]


def test_fold_random_cross_check(oracle_lib):
    """C fold == Python fold on 20k random updates with collisions, tombstones, equal seqs."""
    rng = random.Random(11)
    keys = [bytes([rng.randrange(4)]) * rng.randrange(1, 3) for _ in range(8)]
    ix = O.Index()
    py = R.Index()
    for i in range(20000):
        k = rng.choice(keys)
        fid = rng.randrange(1, 6)
        seq = rng.randrange(0, 50)
        vsz = 0xFFFFFFFF if rng.random() < 0.25 else rng.randrange(0, 100)
        pos = rng.randrange(0, 10000)
        ix.update(k, fid, pos, vsz, seq)
        py.update(R.Row(pos=pos, seq=seq, ksz=len(k), vsz_raw=vsz, key=k), fid)
    assert ix.export() == sorted([k.hex(), v.file_id, v.entry_pos, v.entry_size, v.sequence] for k, v in py.map.items())
    assert ix.stats() == sorted([f, *s] for f, s in py.stats.map.items())


# ---------------------------------------------------------------------------------------------
# The C oracle's compaction (orc_compact_files) and threaded replay (orc_replay_parallel), used as
# the checkers of the full-size configs[3] / configs[4] GPU tests, pinned against the Python
# restatement here at sizes it finishes in seconds.
# ---------------------------------------------------------------------------------------------
def _log_entries(rng, n, nkeys, p_del=0.1, vmax=300):
    keys = [rng.randbytes(rng.randrange(1, 24)) for _ in range(nkeys)]
    out = []
    for i in range(n):
        k = rng.choice(keys)
        if rng.random() < p_del:
            out.append(R.entry_deleted(i + 1, k))
        else:
            out.append(R.entry_new(i + 1, k, rng.randbytes(rng.randrange(0, vmax))))
    return out


def _py_index_to_oracle(db):
    ix = O.Index()
    # rebuild the keydir entries as they stand (one update per live key reproduces the entries)
    for k, e in db.index.map.items():
        ix.update(k, e.file_id, e.entry_pos, e.entry_size - 18 - len(k), e.sequence)
    return ix


@pytest.mark.parametrize("seed,mfs", [(1, 8 << 10), (2, 64 << 10), (3, 700)])
def test_c_compaction_matches_restatement(oracle_lib, tmp_path, seed, mfs):
    """orc_compact_files writes the same bytes as cask_ref.compact_files (both restate
    compact_files_aux, cask.rs:451-523, with first-seen tombstone order): every new data and hint file,
    the file ids and which files the live records started (new_files)."""
    rng = random.Random(seed)
    ents = _log_entries(rng, 4000, nkeys=600)
    src, py = str(tmp_path / "src"), str(tmp_path / "py")
    R.write_log(src, ents, max_file_size=mfs)
    shutil.copytree(src, py)
    db = R.replay(py)
    ix = _py_index_to_oracle(db)
    files = db.files[:-1] if len(db.files) > 1 else db.files
    seq0 = db.file_id_seq
    out = str(tmp_path / "c")
    os.makedirs(out)
    r, created = O.compact_files(src, out, ix, files, seq0, mfs)
    assert r.err_kind == 0
    compacted, new_files = R.compact_files(py, db, files, mfs)
    assert r.n_compacted == len(compacted)
    assert [f for f, live in created if live] == new_files
    assert r.file_id_seq == db.file_id_seq
    for fid, _ in created:
        for ext in ("data", "hint"):
            a = open(os.path.join(out, f"{fid:010}.cask.{ext}"), "rb").read()
            b = open(os.path.join(py, f"{fid:010}.cask.{ext}"), "rb").read()
            assert a == b, (fid, ext)


def test_c_compaction_reports_corrupt_live_entry(oracle_lib, tmp_path):
    """A live record whose bytes no longer verify ends compaction with InvalidChecksum at its
    position (Log::read_entry, log.rs:150-166), as the restatement's read_entry does."""
    rng = random.Random(5)
    ents = _log_entries(rng, 1500, nkeys=200)
    src = str(tmp_path / "src")
    R.write_log(src, ents, max_file_size=16 << 10)
    db = R.replay(src)
    ix = _py_index_to_oracle(db)
    fid = db.files[0]
    live = [(k, e) for k, e in db.index.map.items() if e.file_id == fid]
    k, e = live[len(live) // 2]
    p = R.data_file_path(src, fid)
    b = bytearray(open(p, "rb").read())
    b[e.entry_pos + 18 + len(k) - 1 if e.entry_size == 18 + len(k) else e.entry_pos + e.entry_size - 1] ^= 0x40
    open(p, "wb").write(bytes(b))
    out = str(tmp_path / "c")
    os.makedirs(out)
    r, _ = O.compact_files(src, out, ix, [fid], db.file_id_seq, 16 << 10)
    with pytest.raises(R.CaskError) as ex:
        R.compact_files(src, R.replay(src, write_hints=False), [fid], 16 << 10)
    err = ex.value
    assert (r.err_kind, r.err_file_id) == ((1 if err.kind == "checksum" else 2), fid)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_parallel_replay_matches_serial(oracle_lib, threads):
    """orc_replay_parallel (scan on threads, fold split by key) equals the serial fold of the same
    files in order: keydir digest, size, stats, max sequence — with overwrites, stale and
    resurrecting tombstones across files — and stops at the first failure in replay order."""
    rng = random.Random(100 + threads)
    ents = _log_entries(rng, 6000, nkeys=400, p_del=0.15)
    rng.shuffle(ents)  # sequences out of order across files: stale records and tombstones
    bufs, fids = [], []
    for i in range(0, len(ents), 700):
        bufs.append(b"".join(e.write_bytes() for e in ents[i:i + 700]))
        fids.append(len(fids) + 3)
    ix = O.Index()
    mx = 0
    for b, f in zip(bufs, fids):
        rr = O.replay_fast(np.frombuffer(b, np.uint8), f, ix)
        assert rr.err_kind == 0
        mx = max(mx, rr.max_seq)
    r, stats = O.replay_parallel(bufs, fids, threads)
    assert r.err_kind == 0 and r.records == len(ents)
    assert (r.live, r.max_seq, r.digest) == (len(ix), mx, ix.digest())
    assert stats == ix.stats()
    # a corrupted record in file 3: the fold stops there (rows before it still count)
    bad = bytearray(bufs[3])
    bad[len(bad) // 2] ^= 0x01
    bufs2 = bufs[:3] + [bytes(bad)] + bufs[4:]
    r2, _ = O.replay_parallel(bufs2, fids, threads)
    want = O.scan(bytes(bad))
    first = want[want["status"] != 0][0]
    assert (r2.err_kind, r2.err_file_id, r2.err_pos) == (int(first["status"]), fids[3], int(first["pos"]))


@pytest.mark.parametrize("threads", [2, 8])
def test_parallel_replay_splits_one_file_over_threads(oracle_lib, threads):
    """A sample of one large file uses every thread (the checksums split by byte range) and still
    folds in order; a corrupted value size (a record cut short: UnexpectedEof) and a checksum
    failure before it end the replay where the serial scan's first failure is."""
    rng = random.Random(7 + threads)
    ents = _log_entries(rng, 5000, nkeys=700, p_del=0.1)
    buf = b"".join(e.write_bytes() for e in ents)
    ix = O.Index()
    rr = O.replay_fast(np.frombuffer(buf, np.uint8), 9, ix)
    r, stats = O.replay_parallel([buf], [9], threads)
    assert r.err_kind == 0 and r.records == len(ents) == rr.records
    assert (r.live, r.max_seq, r.digest) == (len(ix), rr.max_seq, ix.digest())
    assert stats == ix.stats()
    offs = np.cumsum([0] + [len(e.write_bytes()) for e in ents])
    for cut, flip in ((3000, None), (3000, 1200), (4999, 10)):
        bad = bytearray(buf)
        bad[offs[cut] + 17] = 0x7F  # value size's high byte: the record runs past the file's end
        if flip is not None:
            bad[offs[flip] + 20] ^= 0x40  # a key byte of an earlier record: its checksum fails
        want = O.scan(bytes(bad))
        k = int(np.flatnonzero(want["status"] != 0)[0])  # the replay keeps the rows before it
        r2, _ = O.replay_parallel([bytes(bad)], [9], threads)
        assert (r2.err_kind, r2.err_pos, r2.records) == (int(want["status"][k]), int(want["pos"][k]), k), (cut, flip)


def test_keydir_digest_numpy_equals_c(oracle_lib):
    """The vectorised digest the GPU tests apply to a product export equals the C oracle's."""
    rng = np.random.default_rng(3)
    n = 1000
    keys = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    fid = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    pos, size, seq = (rng.integers(0, 1 << 63, n, dtype=np.uint64) for _ in range(3))
    want = 0
    for i in range(n):
        want = (want + O.entry_digest(keys[i].tobytes(), int(fid[i]), int(pos[i]), int(size[i]), int(seq[i]))) % (1 << 64)
    got = O.keydir_digest_np(keys, np.full(n, 16), fid, pos, size, seq)
    assert got == want


def test_pindex_compaction_equals_serial_index(oracle_lib, tmp_path):
    """Compaction with the threaded replay's keydir (orc_pindex) writes the same files as with the
    serial one, and orc_hint_body reproduces the restatement's recreated hint bodies."""
    rng = random.Random(21)
    ents = _log_entries(rng, 3000, nkeys=500)
    src = str(tmp_path / "src")
    R.write_log(src, ents, max_file_size=8 << 10)
    db = R.replay(src, write_hints=False)
    bufs = [np.fromfile(R.data_file_path(src, f), np.uint8) for f in db.files]
    for b, f in zip(bufs, db.files):
        body = open(R.hint_file_path(src, f), "rb").read()[:-4]
        assert O.hint_body(b).tobytes() == body
    pix = O.PIndex(bufs, db.files, 4)
    ix = _py_index_to_oracle(db)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    os.makedirs(a)
    os.makedirs(b)
    r1, c1 = pix.compact_files(src, a, db.files, db.file_id_seq, 8 << 10)
    r2, c2 = O.compact_files(src, b, ix, db.files, db.file_id_seq, 8 << 10)
    assert r1.err_kind == r2.err_kind == 0 and c1 == c2 and r1.live_records == r2.live_records
    assert sorted(os.listdir(a)) == sorted(os.listdir(b))
    for f in os.listdir(a):
        assert open(os.path.join(a, f), "rb").read() == open(os.path.join(b, f), "rb").read(), f
    assert pix.result.live == len(db.index.map)

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

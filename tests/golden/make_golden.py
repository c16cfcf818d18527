"""Generate the committed golden fixtures under tests/golden/.

Run from the repo root:  python tests/golden/make_golden.py

Inputs are synthetic (seeded) Cask databases written with the restated LogWriter/Entry codec
(oracle/cask_ref.py, data.rs:90-121, log.rs:282-395). Expected outputs are the restated
Entries scan (log.rs:403-429 + data.rs:161-206), hint-file bytes (log.rs:367-395, 449-471) and
Cask::open replay (cask.rs:335-382: keydir, stats, sequence, first error). XXH32 values come
from python-xxhash 3.8.1 (libxxhash 0.8.2). The reference's own test_serialization records
(data.rs:285-318) are included verbatim as KATs.
"""
from __future__ import annotations

import json
import os
import random
import shutil
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import cask_ref as R  # noqa: E402


def rng_bytes(rng: random.Random, n: int) -> bytes:
    return bytes(rng.getrandbits(8) for _ in range(n)) if n < 4096 else rng.randbytes(n)


def expected_for_dir(path: str, write_hints: bool) -> dict:
    files = []
    for fid in R.find_data_files(path):
        with open(R.data_file_path(path, fid), "rb") as f:
            buf = f.read()
        rows = R.scan_entries(buf)
        files.append({
            "file_id": fid,
            "len": len(buf),
            "rows": [[r.pos, r.seq, r.ksz, r.vsz_raw, r.status, r.expected, r.found] for r in rows],
            "recreated_hint_hex": R.hint_file_bytes(rows).hex(),
        })
    # replay on a scratch copy so the fixture directory is not modified
    scratch = path + ".replay_tmp"
    shutil.rmtree(scratch, ignore_errors=True)
    shutil.copytree(path, scratch)
    res = R.replay(scratch, write_hints=write_hints)
    hints_after = {}
    for fid in res.files:
        hp = R.hint_file_path(scratch, fid)
        if os.path.exists(hp):
            with open(hp, "rb") as f:
                hints_after[str(fid)] = f.read().hex()
    shutil.rmtree(scratch)
    err = None
    if res.error is not None:
        e = res.error
        err = {"kind": e.kind, "file_id": e.file_id, "pos": e.pos, "expected": e.expected, "found": e.found}
    keydir = sorted([k.hex(), v.file_id, v.entry_pos, v.entry_size, v.sequence] for k, v in res.index.map.items())
    stats = sorted([fid, s[0], s[1], s[2]] for fid, s in res.index.stats.map.items())
    return {
        "files": files,
        "replay": {
            "error": err,
            "sequence": res.sequence,
            "current_sequence": res.current_sequence,
            "keydir": keydir if err is None else None,
            "stats": stats if err is None else None,
            "hint_files_after": hints_after,
        },
    }


def write_case(name: str, entries: list, max_file_size: int = 1 << 30, hints: bool = False,
               mutate=None, note: str = ""):
    d = os.path.join(HERE, name)
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    R.write_log(d, entries, max_file_size, write_hints=hints)
    if mutate is not None:
        mutate(d)
    exp = expected_for_dir(d, write_hints=True)
    exp["note"] = note
    with open(os.path.join(d, "expected.json"), "w") as f:
        json.dump(exp, f, indent=0, sort_keys=True)
    # the case directory holds only the inputs + expected.json
    print(f"{name}: {len(exp['files'])} files, error={exp['replay']['error']}")


def flip_byte(fid: int, off: int, mask: int = 0x01):
    def m(d):
        p = R.data_file_path(d, fid)
        with open(p, "r+b") as f:
            f.seek(off)
            b = f.read(1)[0]
            f.seek(off)
            f.write(bytes([b ^ mask]))
    return m


def truncate(fid: int, new_len: int):
    def m(d):
        with open(R.data_file_path(d, fid), "r+b") as f:
            f.truncate(new_len)
    return m


def main():
    rng = random.Random(0xC0FFEE)

    # --- KATs: XXH32 + the reference's own test_serialization records (data.rs:285-318)
    kat = {"xxh32": []}
    for n in list(range(0, 70)) + [100, 255, 256, 1000, 4096, 65535, 100000]:
        data = bytes((i * 7 + 3) & 0xFF for i in range(n))
        kat["xxh32"].append([data.hex() if n <= 256 else f"pattern:{n}", R.xxhash32(data)])
    for s in [b"", b"a", b"abc", b"message digest", b"abcdefghijklmnopqrstuvwxyz"]:
        kat["xxh32"].append([s.hex(), R.xxhash32(s)])
    live = R.entry_new(0, b"\x00\x00\x00", b"\x00\x00\x00")
    dead = R.entry_deleted(0, b"\x00\x00\x00")
    assert len(live.to_bytes()) == 24  # data.rs:293
    assert live.to_bytes() == live.write_bytes()
    kat["test_serialization"] = {
        "live_to_bytes": live.to_bytes().hex(),
        "live_write_bytes": live.write_bytes().hex(),
        "deleted_to_bytes": dead.to_bytes().hex(),
        "deleted_write_bytes": dead.write_bytes().hex(),
    }
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=0)

    # --- serialization: the two test records as a data file
    write_case("serialization", [live, R.Entry(b"\x00\x00\x00", b"", 1, True)],
               note="data.rs:285-318 records as a one-file database")

    # --- basic: 200 puts with overwrites in one file
    keys = [rng_bytes(rng, rng.randint(1, 24)) for _ in range(60)]
    ents, seq = [], 0
    for _ in range(200):
        ents.append(R.entry_new(seq, rng.choice(keys), rng_bytes(rng, rng.randint(0, 120))))
        seq += 1
    write_case("basic", ents, note="200 puts over 60 keys, one file")

    # --- multi_file: rollover, overwrites, deletes, equal-seq duplicates across files
    ents, seq = [], 1
    live_keys = {}
    for i in range(400):
        k = rng.choice(keys)
        if rng.random() < 0.15 and k in live_keys:
            ents.append(R.entry_deleted(seq, k))
            live_keys.pop(k)
        else:
            e = R.entry_new(seq, k, rng_bytes(rng, rng.randint(0, 90)))
            ents.append(e)
            live_keys[k] = e
        seq += 1
    # post-compaction shape: re-append some live entries with their original sequence
    for k, e in list(live_keys.items())[:10]:
        ents.append(R.Entry(e.key, e.value, e.sequence, False))
    write_case("multi_file", ents, max_file_size=3000,
               note="rollover at 3000 B; 15% deletes; 10 equal-seq duplicates at the end")

    # --- fold edge cases (cask.rs:60-90)
    K = b"key-A"
    write_case("stale_tombstone",
               [R.entry_new(10, K, b"v10"), R.entry_new(11, b"other", b"x"), R.entry_deleted(3, K)],
               note="tombstone older than the occupant: counted entry+dead in its own file")
    write_case("resurrection",
               [R.entry_deleted(9, K), R.entry_new(2, K, b"v2"),
                R.entry_new(5, b"B", b"v5"), R.entry_deleted(7, b"B"), R.entry_new(6, b"B", b"v6"),
                R.entry_new(8, b"C", b"v8"), R.entry_new(8, b"C", b"v8b")],
               max_file_size=60,
               note="vacant tombstone is a no-op; lower-seq put after a tombstone resurrects; equal seq: later wins")

    # --- corruption (data.rs:193-198 / :163,172,181)
    ents = [R.entry_new(i + 1, f"k{i:04}".encode(), rng_bytes(rng, 40 + (i % 17))) for i in range(80)]
    sizes = [e.size() for e in ents]
    pos5 = sum(sizes[:5])
    write_case("corrupt_value", ents, mutate=flip_byte(1, pos5 + 18 + 5 + 3),
               note="bit flip inside the value of record 5 -> InvalidChecksum; later rows still scanned")
    write_case("corrupt_checksum_field", ents, mutate=flip_byte(1, sum(sizes[:7]) + 1),
               note="bit flip in the stored checksum of record 7")
    write_case("corrupt_ksz", ents, mutate=flip_byte(1, sum(sizes[:9]) + 12, 0x40),
               note="ksz of record 9 corrupted: the chain desynchronises after it")
    total = sum(sizes)
    write_case("truncated_header", ents, mutate=truncate(1, total - sizes[-1] + 10),
               note="last record cut inside its header -> UnexpectedEof")
    write_case("truncated_key", ents, mutate=truncate(1, total - sizes[-1] + 18 + 2),
               note="last record cut inside its key")
    write_case("truncated_value", ents, mutate=truncate(1, total - 3),
               note="last record cut inside its value")
    write_case("empty_file", [R.entry_new(1, b"a", b"b")], mutate=truncate(1, 0),
               note="a zero-length data file")

    # --- record-size edges (data.rs:13-14)
    big_key = rng_bytes(rng, 65535)
    write_case("edge_sizes",
               [R.entry_new(1, b"", b""), R.entry_new(2, b"k", b""), R.entry_new(3, b"", b"v" * 17),
                R.entry_new(4, big_key, b"x" * 5), R.entry_deleted(5, b""), R.entry_deleted(6, b"k"),
                R.entry_new(7, b"long", rng_bytes(rng, 70000)), R.entry_new(8, b"after", b"tail")],
               note="ksz 0, vsz 0, ksz 65535, tombstones with ksz 0, a 70000 B value")

    # --- adversarial for speculative boundary search: values are serialized records
    inner = [R.entry_new(1000 + i, f"in{i}".encode(), b"zz" * (i + 1)).write_bytes() for i in range(40)]
    ents = []
    for i in range(120):
        v = b"".join(inner[(i + j) % 40] for j in range(i % 5 + 1))
        ents.append(R.entry_new(i + 1, f"outer{i}".encode(), v))
    write_case("embedded_records", ents, note="every value is a run of valid serialized records")
    ents = [R.entry_new(i + 1, b"\x00" * 8, b"\x00" * (i % 50)) for i in range(150)]
    write_case("zeros", ents, note="all-zero keys and values")

    # --- hint fast path (log.rs:121-135, 512-539)
    ents = [R.entry_new(i + 1, f"h{i % 30}".encode(), rng_bytes(rng, 30)) for i in range(100)]
    write_case("hints_valid", ents, max_file_size=1500, hints=True,
               note="valid hint files: replay trusts them and never scans")

    def corrupt_hint(d):
        p = R.hint_file_path(d, 2)
        with open(p, "r+b") as f:
            f.seek(3)
            f.write(b"\xAA")
    write_case("hints_corrupt", ents, max_file_size=1500, hints=True, mutate=corrupt_hint,
               note="file 2's hint trailer mismatches: that file is rescanned and its hint recreated")


if __name__ == "__main__":
    main()

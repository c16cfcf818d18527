"""The batched write path (§8f rank 4): Entry::write_bytes (data.rs:90-121) on the device for
caller-supplied keys and values, and the bulk LogWriter (log.rs:282-306, 317-395) built on it,
against the restatement's encoder and write_log, byte for byte."""
import os
import random

import numpy as np
import pytest

import cask_ref as R

pytestmark = pytest.mark.gpu


def _entries(rng, n, nkeys=None, vmax=600, del_p=0.12):
    keys = [rng.randbytes(rng.randrange(0, 40)) for _ in range(nkeys or n)]
    out = []
    for i in range(n):
        k = rng.choice(keys)
        if rng.random() < del_p:
            out.append(R.entry_deleted(1000 + 3 * i, k))
        else:
            out.append(R.entry_new(1000 + 3 * i, k, rng.randbytes(rng.randrange(0, vmax))))
    return out


def test_encode_caller_keys_matches_oracle(gpu_ctx):
    """cask_encode_device: keys/values from caller buffers (not contiguous with the records, keys
    shared between records), every byte equal to the restatement's Entry::write_bytes."""
    import torch
    rng = random.Random(77)
    ents = _entries(rng, 4000, nkeys=900)
    ents.append(R.entry_new(5, b"", b""))                      # empty key and value
    ents.append(R.entry_new(6, b"k" * 65535, b"v" * 70000))   # maximum key, value past the 4 KiB halo
    ents.append(R.entry_deleted(7, b"t" * 65535))
    n = len(ents)
    # caller layout: every distinct key once (in reverse order), values in a separate buffer
    uniq = sorted({e.key for e in ents}, reverse=True)
    kpos, kbuf = {}, bytearray()
    for k in uniq:
        kpos[k] = len(kbuf)
        kbuf += k
    vbuf = bytearray(b"\xAA" * 13)
    val_off = np.zeros(n, dtype=np.int64)
    for i, e in enumerate(ents):
        if not e.deleted:
            val_off[i] = len(vbuf)
            vbuf += e.value
    ksz = np.array([len(e.key) for e in ents], dtype=np.uint16)
    vsz = np.array([0xFFFFFFFF if e.deleted else len(e.value) for e in ents], dtype=np.uint32)
    size = np.array([e.size() for e in ents], dtype=np.int64)
    off = np.cumsum(size) - size
    dev = torch.device("cuda")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = torch.full((int(size.sum()),), 0x5C, dtype=torch.uint8, device=dev)
    gpu_ctx.encode(t(off), t(np.array([e.sequence for e in ents], dtype=np.int64)), t(ksz.view(np.int16)),
                   t(vsz.view(np.int32)), t(np.frombuffer(bytes(kbuf), dtype=np.uint8)),
                   t(np.array([kpos[e.key] for e in ents], dtype=np.int64)),
                   t(np.frombuffer(bytes(vbuf), dtype=np.uint8)), t(val_off), out)
    assert out.cpu().numpy().tobytes() == b"".join(e.write_bytes() for e in ents)


def _dir(path):
    return {f: open(os.path.join(path, f), "rb").read() for f in sorted(os.listdir(path))
            if f.endswith(".cask.data") or f.endswith(".cask.hint")}


@pytest.mark.parametrize("seed,mfs", [(1, 4 << 10), (2, 64 << 10), (3, 1 << 30), (4, 600)])
def test_log_write_matches_oracle(tmp_path, seed, mfs):
    """Data and hint files byte-identical to the restatement's LogWriter (rollover at mfs; at 600 B
    some records exceed the limit and get a file each), and the result opens to the same keydir."""
    from cask_amd import CaskOptions
    from cask_amd.writer import log_write
    rng = random.Random(seed)
    ents = _entries(rng, 3000, nkeys=700)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    os.makedirs(a)
    ids = log_write(a, [(e.sequence, e.key, None if e.deleted else e.value) for e in ents], mfs, first_file_id=7)
    want = R.write_log(b, ents, max_file_size=mfs, first_file_id=7)
    assert ids == want
    assert _dir(a) == _dir(b)
    rdb = R.replay(b)
    with CaskOptions().max_file_size(mfs).open(a) as db:
        assert {k: e.sequence for k, e in db.index().items()} == {k: v.sequence for k, v in rdb.index.map.items()}
        assert db.stats() == {f: tuple(s) for f, s in rdb.index.stats.map.items()}


def test_log_write_no_hints_then_open_scans(tmp_path):
    """write_hints=False leaves data files only: open() scans them on the device and recreates the
    hint files the writer would have left."""
    from cask_amd import CaskOptions
    from cask_amd.writer import log_write
    rng = random.Random(9)
    ents = _entries(rng, 2000, nkeys=300)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    os.makedirs(a)
    log_write(a, [(e.sequence, e.key, None if e.deleted else e.value) for e in ents], 16 << 10, write_hints=False)
    R.write_log(b, ents, max_file_size=16 << 10)
    assert not any(f.endswith(".hint") for f in os.listdir(a))
    with CaskOptions().max_file_size(16 << 10).open(a) as db:
        assert len(db) == len(R.replay(b).index.map)
    assert _dir(a) == _dir(b)


def test_log_write_empty(tmp_path):
    from cask_amd.writer import log_write
    assert log_write(str(tmp_path), [], 1 << 20) == []
    assert os.listdir(str(tmp_path)) == []


def test_log_write_no_hints_over_stale_hint_files(tmp_path):
    """write_hints=False over a directory whose ids already have valid hint files (from other
    data): those hint files go, so the next open scans the new data instead of trusting hints that
    describe other bytes (the reference's HintWriter::new truncates them, log.rs:373-380)."""
    from cask_amd import CaskOptions
    from cask_amd.writer import log_write
    rng = random.Random(11)
    old = _entries(rng, 1500, nkeys=200)
    new = _entries(random.Random(12), 1500, nkeys=900)
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    os.makedirs(a)
    log_write(a, [(e.sequence, e.key, None if e.deleted else e.value) for e in old], 16 << 10)
    assert any(f.endswith(".hint") for f in os.listdir(a))
    log_write(a, [(e.sequence, e.key, None if e.deleted else e.value) for e in new], 16 << 10, write_hints=False)
    R.write_log(b, new, max_file_size=16 << 10)
    # files of the old log beyond the new one's ids keep their data and hints: drop them from both sides
    keep = set(os.listdir(b)) | {f.replace(".hint", ".data") for f in os.listdir(b)}
    for f in os.listdir(a):
        if f.replace(".hint", ".data") not in keep:
            os.remove(os.path.join(a, f))
    with CaskOptions().max_file_size(16 << 10).open(a) as db:
        rdb = R.replay(b)
        assert {k: e.sequence for k, e in db.index().items()} == {k: v.sequence for k, v in rdb.index.map.items()}
    assert _dir(a) == _dir(b)

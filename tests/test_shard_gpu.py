"""The sharded replay on the GPU: the device's keydir blocks against the restatement
(byte for byte), two shards scanned and reduced in one process on cuda:0 and folded in rank order
against the single-process Cask::open replay (cask.rs:346-382), and cask_db_open_multi. Needs an MI355X.
"""
import os
import random
import shutil

import numpy as np
import pytest

import cask_ref as R
import cask_shard as S

pytestmark = pytest.mark.gpu


def _make_db(path, seed, nfiles=6, nrec=3000, nkeys=400, tomb_p=0.12, back_p=0.1, max_vsz=300):
    """Data files of overwrites, deletes and out-of-order sequences (stale records)."""
    rng = random.Random(seed)
    keys = [rng.randbytes(rng.randrange(0, 24)) for _ in range(nkeys)]
    seq = 1
    os.makedirs(path, exist_ok=True)
    for fid in range(1, nfiles + 1):
        recs = []
        for _ in range(nrec):
            k = rng.choice(keys)
            s = seq if rng.random() > back_p else max(0, seq - rng.randrange(1, 5000))
            seq += 1
            if rng.random() < tomb_p:
                recs.append(R.entry_deleted(s, k).write_bytes())
            else:
                recs.append(R.entry_new(s, k, rng.randbytes(rng.randrange(0, max_vsz))).write_bytes())
        with open(R.data_file_path(path, fid), "wb") as f:
            f.write(b"".join(recs))


def _files(path):
    out = []
    for fid in R.find_data_files(path):
        with open(R.data_file_path(path, fid), "rb") as f:
            out.append((fid, f.read()))
    return out


def _device_block(ctx, part):
    import torch
    from cask_amd.keydir import shard_keydir
    tens = [(fid, torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()) for fid, b in part]
    res = ctx.scan_device(tens)
    assert res.error is None
    return shard_keydir(ctx, tens, {"pos": res.pos, "seq": res.seq, "vsz": res.vsz, "ksz": res.ksz,
                                    "status": res.status}, res.count, res.file_row_offset).cpu().numpy().tobytes()


def _oracle_block(part):
    rows = []
    for fid, b in part:
        for r in R.scan_entries(b):
            assert r.status == R.ROW_OK
            rows.append((fid, r))
    return S.shard_block([fid for fid, _ in part], rows)


def _want(path):
    ref = str(path) + "_ref"
    shutil.copytree(path, ref)
    rep = R.replay(ref, write_hints=False)
    assert rep.error is None
    kd = sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence] for k, e in rep.index.map.items())
    return kd, sorted([f, *s] for f, s in rep.index.stats.map.items()), rep.current_sequence


def _got(db):
    return (sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence] for k, e in db.index().items()),
            sorted([f, *s] for f, s in db.stats().items()), db.current_sequence)


@pytest.mark.parametrize("seed", [1, 2])
def test_device_block_equals_restatement(gpu_ctx, tmp_path, seed):
    path = str(tmp_path / "db")
    _make_db(path, seed, nfiles=4, nrec=2500, nkeys=300 if seed == 1 else 5000)
    files = _files(path)
    for part in (files, files[:1], files[1:3]):
        assert _device_block(gpu_ctx, part) == _oracle_block(part)


def test_two_shards_in_process_fold(gpu_ctx, tmp_path):
    """Two shards' HIP scan + keydir blocks on cuda:0, folded in rank order, against the replay."""
    from cask_amd.keydir import KeydirFold
    path = str(tmp_path / "db")
    _make_db(path, 7)
    files = _files(path)
    want = _want(path)
    for cut in (1, 3, 5):
        fold = KeydirFold()
        for part in (files[:cut], files[cut:]):
            fold.merge(_device_block(gpu_ctx, part))
        with fold.finish() as db:
            assert _got(db) == want


def test_open_multi_matches_replay(native, tmp_path):
    from cask_amd import CaskOptions
    from cask_amd.keydir import open_multi
    path = str(tmp_path / "db")
    _make_db(path, 11, nfiles=7)
    want = _want(path)
    for devices in ([0], [0, 0], [0, 0, 0, 0], [0] * 9):
        with open_multi(path, devices, CaskOptions().write_hints(False)) as db:
            assert _got(db) == want, devices
            assert db.files() == R.find_data_files(path)
    assert not any(f.endswith(".hint") for f in os.listdir(path))


def test_open_multi_hint_files(native, tmp_path):
    """The hint fast path on the multi-GPU replay: the scanned files get their hint files (byte for
    byte the restatement's RecreateHints output); a second open takes the hints — parsed on the
    device — even for data files corrupted since (the reference trusts a valid hint file,
    log.rs:121-135); a mix of hinted and scanned files in one shard; a truncated hint body."""
    from cask_amd import errors
    from cask_amd.keydir import open_multi
    path = str(tmp_path / "db")
    _make_db(path, 13, nfiles=6)
    want = _want(path)
    ref = str(tmp_path) + "/ref_hints"
    shutil.copytree(path, ref)
    R.replay(ref)  # writes the hint files
    with open_multi(path, [0, 0, 0]) as db:
        assert _got(db) == want
    for f in R.find_data_files(path):
        assert open(R.hint_file_path(path, f), "rb").read() == open(R.hint_file_path(ref, f), "rb").read()
    # corrupt every data file: the hints are trusted
    for f in R.find_data_files(path):
        p = R.data_file_path(path, f)
        b = bytearray(open(p, "rb").read())
        b[len(b) // 2] ^= 0x20
        open(p, "wb").write(bytes(b))
    for devices in ([0], [0, 0], [0] * 4):
        with open_multi(path, devices) as db:
            assert _got(db) == want, devices
    # mixed: files 2 and 5 lose their hint files (restore their data first)
    for f in (2, 5):
        shutil.copy(R.data_file_path(ref, f), R.data_file_path(path, f))
        os.remove(R.hint_file_path(path, f))
    with open_multi(path, [0, 0]) as db:
        assert _got(db) == want
    assert os.path.exists(R.hint_file_path(path, 2))
    # a hint body cut short inside a record (valid trailer): Io(UnexpectedEof), as Hints::next
    hp = R.hint_file_path(path, 4)
    body = open(hp, "rb").read()[:-4][:-7]
    open(hp, "wb").write(body + R.xxhash32(body).to_bytes(4, "little"))
    with pytest.raises(errors.UnexpectedEof) as ei:
        open_multi(path, [0, 0])
    assert ei.value.file_id == 4


def test_hint_block_equals_data_block(gpu_ctx, tmp_path):
    """A shard's block from its hint bodies (parsed on the device) is byte for byte the block from
    its data files."""
    import torch
    from cask_amd.keydir import shard_keydir_hints
    path = str(tmp_path / "db")
    _make_db(path, 14, nfiles=4, nrec=4000)
    R.replay(path)
    files = _files(path)
    for part in (files, files[1:3]):
        bodies = [(fid, torch.from_numpy(np.frombuffer(open(R.hint_file_path(path, fid), "rb").read()[:-4],
                                                       np.uint8).copy()).cuda()) for fid, _ in part]
        res = gpu_ctx.parse_hints_device(bodies)
        assert res.error is None
        blk = shard_keydir_hints(gpu_ctx, bodies, {"pos": res.pos, "seq": res.seq, "vsz": res.vsz, "ksz": res.ksz,
                                                   "status": res.status}, res.count, res.file_row_offset)
        assert blk.cpu().numpy().tobytes() == _device_block(gpu_ctx, part)


def test_open_multi_reports_first_failure(native, tmp_path):
    from cask_amd import errors
    from cask_amd.keydir import open_multi
    path = str(tmp_path / "db")
    _make_db(path, 12, nfiles=4, nrec=500)
    for fid, at in ((4, 0.5), (2, 0.3)):  # the failure of the earlier file wins
        p = R.data_file_path(path, fid)
        b = bytearray(open(p, "rb").read())
        b[int(len(b) * at)] ^= 0x40
        open(p, "wb").write(bytes(b))
    ref = str(tmp_path / "ref")
    shutil.copytree(path, ref)
    want = R.replay(ref, write_hints=True).error  # (writes the reference's hint files into ref/)
    with pytest.raises((errors.InvalidChecksum, errors.UnexpectedEof)) as ei:
        open_multi(path, [0, 0])
    assert (ei.value.file_id, ei.value.pos) == (want.file_id, want.pos)
    # the replay stops at the first Err (cask.rs:357-368): hint files of the files up to the failing
    # one (it included, with its Ok records), none after it — though the second range ran in parallel
    assert want.file_id == 2
    for fid in R.find_data_files(path):
        hp, hr = R.hint_file_path(path, fid), R.hint_file_path(ref, fid)
        assert os.path.exists(hp) == os.path.exists(hr) == (fid <= 2), fid
        if fid <= 2:
            assert open(hp, "rb").read() == open(hr, "rb").read(), fid
    assert not [f for f in os.listdir(path) if f.endswith(".part")]


def test_sharded_keydir_unique_keys_large(gpu_ctx):
    """configs[4]'s record shape (unique keys, 290-B records) at 8 files x 200,000 records in 4
    shards: every row is kept, the fold has every key with its last position, stats are puts only."""
    import torch
    from cask_amd.keydir import KeydirFold, shard_keydir
    from cask_amd.workloads import fixed_file
    nrec, fold = 200_000, KeydirFold()
    files = [fixed_file(gpu_ctx, fid, nrec, 16, 256, 1 + (fid - 1) * nrec, (fid - 1) * nrec, 77 + fid) for fid in range(1, 9)]
    for s in range(4):
        part = [(f.file_id, f.data) for f in files[2 * s:2 * s + 2]]
        res = gpu_ctx.scan_device(part)
        assert res.error is None and res.count == 2 * nrec
        blk = shard_keydir(gpu_ctx, part, {"pos": res.pos, "seq": res.seq, "vsz": res.vsz, "ksz": res.ksz,
                                           "status": res.status}, res.count, res.file_row_offset)
        assert blk.numel() == 64 + 2 * nrec * (32 + 16) + 2 * 40
        fold.merge(blk.cpu())
    with fold.finish() as db:
        assert len(db) == 8 * nrec and db.current_sequence == 8 * nrec + 1
        assert db.stats() == {f: (nrec, 0, 0) for f in range(1, 9)}
        host = files[5].data[:290 * 3].cpu().numpy().tobytes()
        e = db.get_entry(host[290 * 2 + 18:290 * 2 + 34])
        assert (e.file_id, e.entry_pos, e.entry_size, e.sequence) == (6, 580, 290, 1 + 5 * nrec + 2)
    del files
    torch.cuda.empty_cache()


def test_rccl_c_abi_gather_single_rank(gpu_ctx, tmp_path):
    """cask_keydir_gather_rccl on a one-rank communicator made through the C ABI (unique id, comm
    init): the rank's block goes to itself and is folded there; keydir, stats and sequence equal the
    replay, and the gathered byte count and max sequence are reported. (Two or more ranks need as
    many GPUs: bench.py --gpus N runs it on the driver's node.)"""
    import torch
    from cask_amd.distributed import RcclComm, gather_fold_rccl, rccl_unique_id
    path = str(tmp_path / "db")
    _make_db(path, 9, nfiles=3)
    files = _files(path)
    want = _want(path)
    tens = [(fid, torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()) for fid, b in files]
    res = gpu_ctx.scan_device(tens)
    assert res.error is None
    from cask_amd.keydir import shard_keydir
    blk = shard_keydir(gpu_ctx, tens, {"pos": res.pos, "seq": res.seq, "vsz": res.vsz, "ksz": res.ksz,
                                       "status": res.status}, res.count, res.file_row_offset)
    comm = RcclComm(rccl_unique_id(), 1, 0, gpu_ctx.device)
    try:
        db, got, mx = gather_fold_rccl(gpu_ctx, comm, blk, root=0)
        with db:
            assert _got(db) == want
            assert mx == want[2] - 1
        assert got == (blk.numel() + 255) // 256 * 256
        # an empty block from the rank (no files) folds to an empty keydir
        db2, got2, _ = gather_fold_rccl(gpu_ctx, comm, torch.empty(0, dtype=torch.uint8, device=blk.device))
        with db2:
            assert len(db2) == 0 and got2 == 0
    finally:
        comm.close()


@pytest.mark.parametrize("seed", [1, 2])
def test_device_partition_equals_host(gpu_ctx, tmp_path, seed):
    """cask_keydir_partition (on the device) byte for byte cask_keydir_partition_host and the
    restatement, for blocks with overwrites, tombstones and stale records, into 1, 2, 3, 8 and 64
    owners; and the owners' fold of the parts equals the replay."""
    import torch
    from cask_amd.keydir import KeydirFold, partition_device, partition_host
    path = str(tmp_path / "db")
    _make_db(path, 30 + seed, nfiles=4, nrec=2500, nkeys=300 if seed == 1 else 5000)
    files = _files(path)
    want = _want(path)
    blocks = [_device_block(gpu_ctx, part) for part in (files[:1], files[1:3], files[3:])]
    for nparts in (1, 2, 3, 8, 64):
        owners = [KeydirFold() for _ in range(nparts)]
        for b in blocks:
            dev = torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()
            got = [p.cpu().numpy().tobytes() for p in partition_device(gpu_ctx, dev, nparts)]
            assert got == [p.tobytes() for p in partition_host(b, nparts)] == S.partition_block(b, nparts)
            for o in range(nparts):
                owners[o].merge(got[o])
        terms = b"".join(f.terms().tobytes() for f in owners)
        kd = []
        for f in owners:
            with f.finish_terms(terms) as db:
                k, st, cs = _got(db)
                kd += k
                assert (st, cs) == (want[1], want[2])
        assert sorted(kd) == want[0]


def test_rccl_c_abi_exchange_single_rank(gpu_ctx, tmp_path):
    """cask_keydir_exchange_rccl on a one-rank communicator: the block is partitioned on the device
    (one part), sent to itself, folded and finished from its own terms — the replay's keydir, stats
    and sequence. (More ranks need as many GPUs: bench.py --gpus N runs it on the driver's node.)"""
    import torch
    from cask_amd.distributed import RcclComm, exchange_fold_rccl, rccl_unique_id
    path = str(tmp_path / "db")
    _make_db(path, 10, nfiles=3)
    files = _files(path)
    want = _want(path)
    blk = torch.from_numpy(np.frombuffer(_device_block(gpu_ctx, files), np.uint8).copy()).cuda()
    comm = RcclComm(rccl_unique_id(), 1, 0, gpu_ctx.device)
    try:
        db, sent, got = exchange_fold_rccl(gpu_ctx, comm, blk)
        with db:
            assert _got(db) == want
        assert sent == 0 and got == blk.numel()
    finally:
        comm.close()

"""Multi-rank path on CPU (gloo, world_size 2): file sharding, the max-sequence all-reduce, the
gather of the ranks' keydir blocks and rank 0's native fold of them. Blocks come from
the oracle's restatement here (no GPU in this container; tests/test_scan_gpu.py checks that the
device builds the same bytes); on the GPU box the same functions run over RCCL (bench.py --gpus N).

Rank 0 folds only what it received — no data file is read there — and the result must equal a
single-process replay of the same directory (cask.rs:346-382), including stale tombstones whose
stats depend on the global fold order.
"""
import json
import os
import random
import socket

import pytest
import torch
import torch.multiprocessing as mp

import cask_ref as R
from cask_amd.distributed import shard_files


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _make_db(path):
    """Four data files; keys overwritten and deleted across files (fold order matters)."""
    rng = random.Random(11)
    keys = [rng.randbytes(rng.randrange(1, 12)) for _ in range(40)]
    entries = []
    seq = 1
    for i in range(600):
        k = rng.choice(keys)
        if rng.random() < 0.15:
            entries.append(R.entry_deleted(seq, k))
        else:
            entries.append(R.entry_new(seq, k, rng.randbytes(rng.randrange(0, 90))))
        # some sequences go backwards: stale records that the fold must count as dead
        seq += 1 if rng.random() < 0.9 else -3
        seq = max(seq, 1)
    R.write_log(path, entries, max_file_size=16 * 1024)
    # an empty data file at the end: the rank that owns it contributes no rows
    last = max(R.find_data_files(path))
    open(R.data_file_path(path, last + 1), "wb").close()


def _worker(rank, world, port, path, out):
    """Each rank scans its own files (oracle rows: no GPU here), builds its keydir block, and the
    blocks meet on rank 0, which folds them with the native fold — it reads no data file."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist
    import cask_shard as S
    import oracle_ffi as O
    from cask_amd.distributed import allreduce_max_seq, gather_blocks, shard_files as shard
    from cask_amd.keydir import KeydirFold
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard(R.find_data_files(path), world, rank)
        rows, local_max = [], 0
        for fid in mine:
            with open(R.data_file_path(path, fid), "rb") as f:
                buf = f.read()
            for r in O.scan(buf):
                assert int(r["status"]) == 0
                p, k = int(r["pos"]), int(r["ksz"])
                rows.append((fid, R.Row(pos=p, seq=int(r["seq"]), ksz=k, vsz_raw=int(r["vsz_raw"]),
                                        key=buf[p + 18:p + 18 + k])))
                local_max = max(local_max, int(r["seq"]))
        block = torch.from_numpy(np.frombuffer(S.shard_block(mine, rows), np.uint8).copy())
        gmax = allreduce_max_seq(local_max, torch.device("cpu"))
        got = gather_blocks(block, dst=0)
        if rank == 0:
            fold = KeydirFold()
            for b in got:
                fold.merge(b)
            db = fold.finish()
            res = {"max_seq": gmax, "current_sequence": db.current_sequence, "sizes": [int(b.numel()) for b in got],
                   "keydir": sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence]
                                    for k, e in db.index().items()),
                   "stats": sorted([f, *s] for f, s in db.stats().items())}
            db.close()
            with open(out, "w") as f:
                json.dump(res, f)
    finally:
        dist.destroy_process_group()


def _pworker(rank, world, port, path, out):
    """The key-hash partitioned replay (huge keyspace): each rank scans its files (oracle
    rows), builds its block, splits it by key owner with the native partitioner, sends part o to rank
    o, folds the parts it owns in rank order and exchanges per-file terms. Each rank reports its keys
    and its (whole-replay) stats."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import cask_shard as S
    import oracle_ffi as O
    from cask_amd.distributed import partitioned_fold, shard_files as shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard(R.find_data_files(path), world, rank)
        rows = []
        for fid in mine:
            with open(R.data_file_path(path, fid), "rb") as f:
                buf = f.read()
            for r in O.scan(buf):
                p, k = int(r["pos"]), int(r["ksz"])
                rows.append((fid, R.Row(pos=p, seq=int(r["seq"]), ksz=k, vsz_raw=int(r["vsz_raw"]),
                                        key=buf[p + 18:p + 18 + k])))
        db = partitioned_fold(S.shard_block(mine, rows))
        res = {"current_sequence": db.current_sequence,
               "keydir": sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence]
                                for k, e in db.index().items()),
               "stats": sorted([f, *s] for f, s in db.stats().items()),
               "files": db.files()}
        db.close()
        with open(out + f".{rank}", "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_partitioned_fold_matches_single_process(tmp_path, world):
    """No rank holds more than its keys, yet together they hold exactly the single-process keydir,
    each key on its owner, and every rank has the whole replay's Stats, files and sequence —
    including stale tombstones whose shard and owner differ."""
    from cask_amd.keydir import key_owner
    path = str(tmp_path / "db")
    os.makedirs(path)
    _make_db(path)
    want = R.replay(path, write_hints=False)
    assert want.error is None
    out = str(tmp_path / "rank")
    mp.start_processes(_pworker, args=(world, _free_port(), path, out), nprocs=world, join=True, start_method="spawn")
    got = []
    for r in range(world):
        with open(out + f".{r}") as f:
            got.append(json.load(f))
    union = sorted(x for g in got for x in g["keydir"])
    assert union == sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence]
                           for k, e in want.index.map.items())
    for r, g in enumerate(got):
        assert all(key_owner(bytes.fromhex(x[0]), world) == r for x in g["keydir"])
        assert g["stats"] == sorted([f, *s] for f, s in want.index.stats.map.items())
        assert g["current_sequence"] == want.current_sequence
        assert g["files"] == sorted(R.find_data_files(path))
    assert all(g["keydir"] for g in got)  # (40 keys: every owner holds some)


def test_shard_files_contiguous_balanced():
    for n in range(0, 40):
        ids = random.Random(n).sample(range(1, 1000), n)
        for world in (1, 2, 3, 8):
            parts = [shard_files(ids, world, r) for r in range(world)]
            assert sum(parts, []) == sorted(ids)  # rank order = file-id order
            sizes = [len(p) for p in parts]
            assert max(sizes) - min(sizes) <= 1


def test_gloo_world2_gather_fold_matches_single_process(tmp_path):
    path = str(tmp_path / "db")
    os.makedirs(path)
    _make_db(path)
    want = R.replay(path, write_hints=False)
    assert want.error is None
    out = str(tmp_path / "rank0.json")
    mp.start_processes(_worker, args=(2, _free_port(), path, out), nprocs=2, join=True, start_method="spawn")
    with open(out) as f:
        got = json.load(f)
    assert got["max_seq"] == want.sequence
    assert got["current_sequence"] == want.current_sequence
    assert got["sizes"][1] > 64 and got["sizes"][0] > 64
    assert got["keydir"] == sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence]
                                   for k, e in want.index.map.items())
    assert got["stats"] == sorted([f, *s] for f, s in want.index.stats.map.items())

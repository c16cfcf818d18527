"""Multi-rank path on CPU (gloo, world_size 2): file sharding, the max-sequence all-reduce and the
rank-ordered row gather that feeds the keydir fold. Rows come from the CPU oracle
here (no GPU in this container); on the GPU box the same functions run over RCCL with rows from
the HIP scan (bench.py --gpus N).

The gathered, rank-ordered fold must equal a single-process replay of the same directory
(cask.rs:346-382), including stale tombstones whose stats depend on the global fold order.
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
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import oracle_ffi as O
    from cask_amd.distributed import allreduce_max_seq, gather_rows, shard_files as shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard(R.find_data_files(path), world, rank)
        cols = {f: [] for f in ("pos", "seq", "vsz", "ksz", "status")}
        fids = []
        local_max = 0
        for fid in mine:
            with open(R.data_file_path(path, fid), "rb") as f:
                buf = f.read()
            rows = O.scan(buf)
            cols["pos"] += [int(x) for x in rows["pos"]]
            cols["seq"] += [int(x) for x in rows["seq"]]
            cols["vsz"] += [int(x) for x in rows["vsz_raw"]]
            cols["ksz"] += [int(x) for x in rows["ksz"]]
            cols["status"] += [int(x) for x in rows["status"]]
            fids += [fid] * len(rows)
            local_max = max([local_max] + [int(x) for x in rows["seq"]])
        t = {"pos": torch.tensor(cols["pos"], dtype=torch.int64),
             "seq": torch.tensor(cols["seq"], dtype=torch.int64),
             "vsz": torch.tensor(cols["vsz"], dtype=torch.int64).to(torch.int32),
             "ksz": torch.tensor(cols["ksz"], dtype=torch.int32).to(torch.int16),
             "status": torch.tensor(cols["status"], dtype=torch.uint8)}
        gmax = allreduce_max_seq(local_max, torch.device("cpu"))
        got = gather_rows(t, len(fids), dst=0, file_id=torch.tensor(fids, dtype=torch.int32))
        if rank == 0:
            index = R.Index()
            bufs = {}
            for blk in got:
                for i in range(blk["pos"].numel()):
                    fid = int(blk["file_id"][i])
                    if fid not in bufs:
                        with open(R.data_file_path(path, fid), "rb") as f:
                            bufs[fid] = f.read()
                    p, k = int(blk["pos"][i]), int(blk["ksz"][i]) & 0xFFFF
                    row = R.Row(pos=p, seq=int(blk["seq"][i]), ksz=k, vsz_raw=int(blk["vsz"][i]) & 0xFFFFFFFF,
                                status=int(blk["status"][i]), key=bufs[fid][p + 18:p + 18 + k])
                    assert row.status == R.ROW_OK
                    index.update(row, fid)
            res = {"max_seq": gmax, "counts": [int(b["pos"].numel()) for b in got],
                   "keydir": sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence]
                                    for k, e in index.map.items()),
                   "stats": sorted([f, *s] for f, s in index.stats.map.items())}
            with open(out, "w") as f:
                json.dump(res, f)
    finally:
        dist.destroy_process_group()


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
    assert sum(got["counts"]) == sum(len(R.scan_entries(open(R.data_file_path(path, fid), "rb").read()))
                                     for fid in want.files)
    assert got["counts"][1] > 0 and got["counts"][0] > 0
    assert got["keydir"] == sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence]
                                   for k, e in want.index.map.items())
    assert got["stats"] == sorted([f, *s] for f, s in want.index.stats.map.items())

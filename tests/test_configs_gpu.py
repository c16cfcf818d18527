"""BASELINE configs at their full sizes on the GPU, checked against the C oracle and the generator
(SURVEY §8d): configs[0] (one file of 2^20 records of 82 B) row for row and through Cask::open;
configs[2] (32 GiB of Zipf-length records in 2-GiB files) clean against the generator, then with
bytes flipped in long and short records at 64-chunk run boundaries and a broken header, row for
row against the oracle's scan of every file (on host threads). Needs an MI355X.
"""
import concurrent.futures as cf
import os

import numpy as np
import pytest

import oracle_ffi as O

pytestmark = pytest.mark.gpu

FIELDS = ("pos", "seq", "ksz", "vsz", "status")


def _dev_rows(res, sl):
    return {"pos": res.pos[sl].cpu().numpy().view(np.uint64), "seq": res.seq[sl].cpu().numpy().view(np.uint64),
            "ksz": res.ksz[sl].cpu().numpy().view(np.uint16), "vsz": res.vsz[sl].cpu().numpy().view(np.uint32),
            "status": res.status[sl].cpu().numpy()}


def _assert_rows_equal(got, want, what):
    assert len(got["pos"]) == len(want), (what, len(got["pos"]), len(want))
    for f, w in (("pos", want["pos"]), ("seq", want["seq"]), ("ksz", want["ksz"].astype(np.uint16)),
                 ("vsz", want["vsz_raw"].astype(np.uint32)), ("status", want["status"].astype(np.uint8))):
        if not np.array_equal(got[f], w):
            i = int(np.nonzero(got[f] != w)[0][0])
            raise AssertionError(f"{what}: field {f} row {i}: got {got[f][i]} want {w[i]}")


def test_cfg0_full_size_bit_exact(gpu_ctx, tmp_path):
    """configs[0]: 2^20 records, 16 B keys / 48 B values, one file; rows bit-exact and Cask::open's
    keydir, stats and sequence equal to the oracle's replay of the same bytes."""
    from cask_amd import CaskOptions
    from cask_amd.workloads import fixed_file
    n = 1 << 20
    f = fixed_file(gpu_ctx, 1, n, 16, 48, 1, 0, 0xC0FFEE + 1)
    res = gpu_ctx.scan_device([(1, f.data)])
    assert res.count == n and res.error is None
    assert gpu_ctx.last_counters()["dense_path"] == 1
    host = f.data.cpu().numpy()
    _assert_rows_equal(_dev_rows(res, slice(0, n)), O.scan(host), "configs[0]")
    path = tmp_path / "db"
    path.mkdir()
    host.tofile(str(path / "0000000001.cask.data"))
    ix = O.Index()
    rr = O.replay_fast(host, 1, ix)
    assert rr.err_kind == 0
    with CaskOptions().open(str(path)) as db:
        assert len(db) == len(ix) == n
        assert sorted([fid, *s] for fid, s in db.stats().items()) == ix.stats()
        assert db.current_sequence == n + 1
        got = sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence] for k, e in db.index().items())
        assert got == sorted(ix.export())


@pytest.fixture(scope="module")
def cfg2(gpu_ctx):
    import torch
    from cask_amd.workloads import zipf_files
    files, vsz, n, rl = zipf_files(gpu_ctx, 32.0, 2 ** 31)
    yield files, vsz, n, rl
    del files, vsz, rl
    torch.cuda.empty_cache()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("mode", ["chunk", "narrow", "walk"])
def test_cfg2_full_size_against_generator(gpu_ctx, cfg2, mode, monkeypatch):
    """Both speculative passes: k_scan_chunks (forced, with either halo) and the walk mode (what the
    library picks for these records: k_walk_search, k_walk_chase, k_run_hash), every row against
    the generator."""
    import torch
    monkeypatch.setenv("CASK_SCAN_MODE", mode)
    files, vsz, n, rl = cfg2
    dev = vsz.device
    rows = gpu_ctx.alloc_rows(n + 16)
    res = gpu_ctx.scan_device([(f.file_id, f.data) for f, _ in files], rows)
    assert res.error is None and res.count == n
    cnt = gpu_ctx.last_counters()
    assert cnt["walked"] == 0 and cnt["walk_mode"] == (mode == "walk"), cnt
    assert cnt["long_records"] > 1_000_000 if mode != "walk" else cnt["dense_path"] == 1, cnt
    assert sum(f.data.numel() for f, _ in files) > 31 * 2 ** 30 and len(files) >= 16
    assert int((rows["status"][:n] != 0).sum().item()) == 0
    assert bool((rows["seq"][:n].to(torch.int64) == torch.arange(1, n + 1, device=dev)).all())
    assert bool((rows["vsz"][:n].to(torch.int64) == vsz[:n].to(torch.int64)).all())
    assert bool((rows["ksz"][:n].to(torch.int64) == 16).all())
    for i, (f, idx) in enumerate(files):
        sl = res.file_rows(i)
        rlf = rl[idx]
        assert bool((rows["pos"][sl].to(torch.int64) == torch.cumsum(rlf, 0) - rlf).all()), i


@pytest.mark.timeout(900)
def test_cfg2_full_size_corrupted_against_oracle(gpu_ctx, cfg2):
    """Value bytes flipped in records that cross or follow 2-MiB boundaries (64 chunks of 32 KiB: a
    run of the chunk scan on large logs) — long records hashed by k_long_hash and short ones hashed
    in LDS — and one record's value_size field broken (the chain after it changes: repair path);
    every row of every file against the oracle's scan, and the first failure."""
    import torch
    files, vsz, n, rl = cfg2
    run = 64 * 32768
    flipped = []
    for fi in (0, 3, 7, len(files) - 1):
        f, idx = files[fi]
        rlf = rl[idx]
        off = torch.cumsum(rlf, 0) - rlf
        end = off + rlf
        # long records crossing a run boundary, short ones starting just after one
        cross = torch.nonzero((off // run) != ((end - 1) // run)).flatten()
        cross = cross[rlf[cross] > 32768][:3]
        after = torch.nonzero((off % run < 512) & (rlf < 1024)).flatten()[:3]
        for r in torch.cat([cross, after]).tolist():
            p = int(off[r]) + 34 + int(rlf[r] - 34) // 2  # a value byte
            f.data[p] ^= 0x5A
            flipped.append((f.file_id, int(off[r])))
    f, idx = files[5]
    rlf = rl[idx]
    off = torch.cumsum(rlf, 0) - rlf
    r = int(torch.nonzero(rlf > 4096).flatten()[100])
    f.data[int(off[r]) + 14] ^= 0x01  # value_size low byte: the chain after this record changes
    hosts = [fd.data.cpu().numpy() for fd, _ in files]
    with cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        want = list(ex.map(O.scan, hosts))  # ctypes releases the GIL: files scan in parallel
    first = None
    for i, ((fd, _), w) in enumerate(zip(files, want)):
        bad = np.nonzero(w["status"] != 0)[0]
        if first is None and bad.size:
            b = w[bad[0]]
            first = (int(b["status"]), fd.file_id, int(b["pos"]), int(b["expected"]),
                     int(b["found"]) if int(b["status"]) == 1 else 0)
    assert len(flipped) >= 12
    for mode in ("chunk", "narrow", "walk"):  # both speculative passes, both halos
        os.environ["CASK_SCAN_MODE"] = mode
        try:
            res = gpu_ctx.scan_device([(fd.file_id, fd.data) for fd, _ in files])
            assert gpu_ctx.last_counters()["walk_mode"] == (mode == "walk")
        finally:
            del os.environ["CASK_SCAN_MODE"]
        for i, ((fd, _), w) in enumerate(zip(files, want)):
            _assert_rows_equal(_dev_rows(res, res.file_rows(i)), w, f"{mode}: file {fd.file_id}")
        e = res.error
        assert (e.kind, e.file_id, e.pos, e.expected, e.found) == first, mode


def test_stream_ceiling_measures_resident_bytes():
    """bench.py's stream ceiling on a few resident buffers: a positive rate in both load policies,
    below the 8 TB/s peak (it reads what it says it reads: 3 buffers, 16-B-rounded lengths)."""
    import torch
    import bench
    dev = torch.device("cuda", 0)
    bufs = [torch.ones(n, dtype=torch.uint8, device=dev) for n in (1 << 30, (512 << 20) + 7, 256 << 20)]
    c = bench.stream_ceiling(torch, dev, [(i + 1, b) for i, b in enumerate(bufs)], passes=3)
    assert c is not None and "error" not in c, c
    assert c["bytes_per_pass"] == sum(b.numel() for b in bufs)
    for k in ("plain", "nontemporal"):
        assert 100.0 < c[k]["gbps"] < bench.HBM_PEAK_GBPS, c

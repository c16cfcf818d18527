"""Measurements of the BASELINE configs other than the headline (configs[1], bench.py).

  cfg3     configs[2]: 32 GiB of records with Zipf-distributed value sizes (16 B .. 64 KiB) in files
           of at most 2 GiB (LogWriter rollover, log.rs:282-306), device-resident scan. Checked:
           every record found, in order, at its offset, with its sequence/sizes, checksum OK.
  compact  configs[3] shape, scaled to --files data files of configs[1] records: 80 % of records
           overwritten or deleted (keys drawn from 20 % as many ids; 10 % of keys end in a
           tombstone). The files are written to disk, Cask::open replays them (GPU scan + hint
           recreation + keydir fold) and Cask::compact_files rewrites the live records (GPU verify
           + GPU gather). Phase times come from the engine; the live keydir is checked unchanged.

Prints one JSON object per measurement (also written to --out).
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cfg3(ctx, torch, steps, total_gib, max_file):
    dev = torch.device("cuda", ctx.device)
    from cask_amd.workloads import zipf_files
    files, vsz, n, rl = zipf_files(ctx, total_gib, max_file)
    views = [(f.file_id, f.data) for f, _ in files]
    nbytes = sum(f.data.numel() for f, _ in files)
    rows = ctx.alloc_rows(n + 16)
    res = ctx.scan_device(views, rows)
    assert res.error is None and res.count == n, (res.count, n, res.error)
    assert int((rows["status"][:n] != 0).sum().item()) == 0
    seq = rows["seq"][:n].to(torch.int64)
    assert bool((seq == torch.arange(1, n + 1, device=dev)).all())
    assert bool((rows["vsz"][:n].to(torch.int64) == vsz[:n].to(torch.int64)).all())
    assert bool((rows["ksz"][:n].to(torch.int64) == 16).all())
    for i, (f, idx) in enumerate(files):  # positions: exclusive prefix of record lengths per file
        sl = res.file_rows(i)
        rlf = rl[idx]
        want = torch.cumsum(rlf, 0) - rlf
        assert bool((rows["pos"][sl].to(torch.int64) == want).all()), i
    counters = ctx.last_counters()
    for _ in range(2):
        ctx.scan_device(views, rows)
    torch.cuda.synchronize(dev)
    k_ms, p_ms = [], []
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.scan_device(views, rows)
        t = ctx.last_timings()
        k_ms.append(t["chunk_scan_ms"])
        p_ms.append(t)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    kavg = sum(k_ms) / len(k_ms)
    brk = {k: sum(d[k] for d in p_ms) / len(p_ms) for k in p_ms[0]}
    return {"config": "configs[2]: 32 GiB, Zipf(1.1) value sizes 16 B-64 KiB, 1 GPU, device-resident",
            "files": len(files), "records": n, "bytes": nbytes, "mean_record_bytes": nbytes / n,
            "gibps": nbytes * steps / el / 2 ** 30, "ms_per_step": el * 1e3 / steps,
            "log_bytes_over_step_frac_of_8TBps": nbytes * steps / el / 8e12,
            "first_pass_kernel": "k_walk_runs" if counters.get("walk_mode") else "k_scan_chunks",
            "first_pass_ms": kavg, "breakdown_ms": brk,
            "counters": counters, "parity": "rows == generator (count, pos, seq, ksz, vsz, status)"}


def write_cfg3(ctx, torch, nfiles, path, live=0.2):
    """configs[3]-shaped data files 1..nfiles in `path`: 290-B records, a key space of a fifth of
    the records (`live`: another fraction), 10 % of keys ending in a tombstone. Returns (bytes,
    live keys, records, seconds)."""
    from cask_amd.workloads import CFG2_RECORDS_PER_FILE, variable_file
    dev = torch.device("cuda", ctx.device)
    rpf = CFG2_RECORDS_PER_FILE
    n = nfiles * rpf
    g = torch.Generator(device=dev)
    g.manual_seed(0xC0FFEE)
    nkeys = max(1, int(n * live))
    kid = torch.randint(0, nkeys, (n,), generator=g, device=dev, dtype=torch.int64)
    last = torch.full((nkeys,), -1, dtype=torch.int64, device=dev)
    last.scatter_reduce_(0, kid, torch.arange(n, device=dev), reduce="amax")
    present = last >= 0
    tomb_key = (torch.rand(nkeys, generator=g, device=dev) < 0.1) & present
    vsz = torch.full((n,), 256, dtype=torch.int32, device=dev)
    vsz[last[tomb_key]] = -1  # 10 % of keys end in a tombstone
    live_want = int((present & ~tomb_key).sum().item())
    t0 = time.perf_counter()
    nbytes = 0
    for i in range(nfiles):
        sl = slice(i * rpf, (i + 1) * rpf)
        idx = torch.arange(i * rpf, (i + 1) * rpf, dtype=torch.int64, device=dev)
        ks = torch.full((rpf,), 16, dtype=torch.int16, device=dev)
        f = variable_file(ctx, i + 1, ks, vsz[sl].clone(), idx + 1, kid[sl].clone(), 0xC0FFEE + i)
        host = f.data.cpu().numpy()
        nbytes += host.size
        with open(os.path.join(path, f"{i + 1:010}.cask.data"), "wb") as fh:
            fh.write(host.tobytes())
        del f, host
        if (i + 1) % 8 == 0:
            print(f"wrote {i + 1}/{nfiles} files", file=sys.stderr, flush=True)
    write_s = time.perf_counter() - t0
    del kid, last, present, tomb_key, vsz
    torch.cuda.empty_cache()
    return nbytes, live_want, n, write_s


def compact(ctx, torch, nfiles, workdir, live=0.2):
    from cask_amd import CaskOptions
    from cask_amd.workloads import CFG2_RECORDS_PER_FILE
    rpf = CFG2_RECORDS_PER_FILE
    path = os.path.join(workdir, "db")
    os.makedirs(path)
    nbytes, live_want, n, write_s = write_cfg3(ctx, torch, nfiles, path, live)
    out = {"config": f"configs[3] shape scaled to {nfiles} files x {rpf} records (290 B, 80 % overwritten/"
                     f"deleted, 10 % of keys end in a tombstone), on disk, 1 GPU",
           "files": nfiles, "records": n, "bytes": nbytes, "write_files_s": write_s, "key_space_fraction": live}
    t0 = time.perf_counter()
    print(f"files written in {write_s:.1f} s; opening", file=sys.stderr, flush=True)
    with CaskOptions().max_file_size(1 << 30).open(path) as db:
        print("opened; compacting", file=sys.stderr, flush=True)
        out["open_s"] = time.perf_counter() - t0
        out["open_timings_ms"] = db.open_timings()
        out["open_gibps_e2e"] = nbytes / out["open_s"] / 2 ** 30
        assert len(db) == live_want, (len(db), live_want)
        before = {k: e.sequence for k, e in db.index().items()} if n <= 4_000_000 else None
        t0 = time.perf_counter()
        rep = db.compact_files(db.files())
        out["compact_s"] = time.perf_counter() - t0
        out["compact_report"] = rep
        out["compact_in_gibps_e2e"] = nbytes / out["compact_s"] / 2 ** 30
        assert len(db) == live_want
        assert rep["live_records"] == live_want
        if before is not None:
            assert {k: e.sequence for k, e in db.index().items()} == before
        out["files_after"] = len(db.files())
    t0 = time.perf_counter()
    with CaskOptions().open(path) as db:  # re-open the compacted database (hints fast path)
        out["reopen_s"] = time.perf_counter() - t0
        assert len(db) == live_want
    out["live_records"] = live_want
    return out


def open_ab(ctx, torch, nfiles, workdir, rounds=2):
    """Cask::open of the same configs[3]-shaped files, in turn: cask_db_open with the keydir reduced
    on the device (the default when every file is scanned), cask_db_open with the host fold of every
    hint row (CASK_OPEN_DEVFOLD=0, a test hook), and cask_db_open_multi over one and two ranges on
    device 0; no hint files are written, so every open scans. Timings: [read, device, hint files,
    fold, total] ms."""
    from cask_amd import CaskOptions
    from cask_amd.keydir import open_multi
    path = os.path.join(workdir, "db")
    os.makedirs(path)
    nbytes, live_want, n, write_s = write_cfg3(ctx, torch, nfiles, path)
    out = {"files": nfiles, "records": n, "bytes": nbytes, "runs": []}
    for r in range(rounds):
        for name in ("open_devfold", "open_hostfold", "open_multi_1", "open_multi_2"):
            os.environ["CASK_OPEN_DEVFOLD"] = "0" if name == "open_hostfold" else "1"
            t0 = time.perf_counter()
            if name.startswith("open_multi"):
                db = open_multi(path, [0] * int(name[-1]), CaskOptions().write_hints(False))
            else:
                db = CaskOptions().write_hints(False).open(path)
            with db:
                dt = time.perf_counter() - t0
                tm = db.open_timings()
                assert len(db) == live_want
            out["runs"].append({"round": r, "what": name, "s": dt, "timings_ms": tm})
            print(f"{name} {dt:.2f} s {tm}", file=sys.stderr, flush=True)
    os.environ.pop("CASK_OPEN_DEVFOLD", None)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="+", choices=["cfg3", "compact", "openab"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--gib", type=float, default=32.0)
    ap.add_argument("--max-file", type=int, default=2 ** 31)
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--out", default="")
    ap.add_argument("--dir", default=None, help="parent directory of the compaction database")
    ap.add_argument("--lib", default="", help="an A/B build of the library (cask_amd._lib.use_library)")
    ap.add_argument("--live", type=float, default=0.2, help="compact: key space as a fraction of the records")
    args = ap.parse_args()
    if "openab" in args.what:  # (open_ab switches the open's fold with a test hook)
        os.environ["CASK_TEST_HOOKS"] = "1"
    import torch
    torch.cuda.set_device(0)
    if args.lib:
        import cask_amd
        cask_amd._lib.use_library(args.lib)
    from cask_amd import ScanContext
    ctx = ScanContext(0)
    results = []
    for w in args.what:
        if w == "cfg3":
            r = cfg3(ctx, torch, args.steps, args.gib, args.max_file)
        else:
            wd = tempfile.mkdtemp(prefix="cask_compact_", dir=args.dir)
            try:
                r = compact(ctx, torch, args.files, wd, args.live) if w == "compact" else open_ab(ctx, torch, args.files, wd)
            finally:
                shutil.rmtree(wd, ignore_errors=True)
        r["what"] = w
        print(json.dumps(r), flush=True)
        results.append(r)
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()

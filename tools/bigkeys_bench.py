"""What keys over 4,351 B cost a walk-mode scan (such keys send the runs that start
after them to the repair path, by design of k_walk_search's candidate test, k_walk.hip:103).

The same Zipf(1.1) value sizes as configs[2] (16 B .. 64 KiB) over --gib GiB in 2-GiB files; every
record's key 16 B, except a fraction --frac of records (evenly spread) whose key is --big bytes.
For each fraction: rows checked against the generator (count, sequence, key and value sizes, status),
then the mean of --steps device-resident scans, and the call's counters (repaired chunks, repair
passes). python tools/bigkeys_bench.py [--gib 8] [--fracs 0,1e-4,1e-3,1e-2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def files_with_keys(ctx, torch, gib, frac, big, max_file=2 ** 31, seed=0x5A1F):
    from cask_amd.workloads import variable_file, zipf_sizes
    dev = torch.device("cuda", ctx.device)
    target = int(gib * 2 ** 30)
    n = int(target / (34 + 5085) * 1.05) + 1024
    vsz = zipf_sizes(n, seed=seed, device=dev)
    ksz = torch.full((n,), 16, dtype=torch.int16, device=dev)
    if frac > 0:
        step = max(1, int(round(1 / frac)))
        ksz[step // 2::step] = big
    rl = 18 + ksz.to(torch.int64) + vsz.to(torch.int64)
    cum = torch.cumsum(rl, 0)
    n = int(torch.searchsorted(cum, torch.tensor([target], device=dev, dtype=torch.int64)).item())
    files, base, r0 = [], 0, 0
    while r0 < n:
        r1 = int(torch.searchsorted(cum, torch.tensor([base + max_file], device=dev, dtype=torch.int64),
                                    right=True).item())
        r1 = min(max(r1, r0 + 1), n)
        idx = torch.arange(r0, r1, dtype=torch.int64, device=dev)
        f = variable_file(ctx, 1 + len(files), ksz[r0:r1].clone(), vsz[r0:r1].clone(), idx + 1, idx,
                          seed + len(files))
        files.append(f)
        base = int(cum[r1 - 1].item())
        r0 = r1
    torch.cuda.synchronize(dev)
    return files, ksz[:n], vsz[:n], n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    ap.add_argument("--fracs", default="0,1e-4,1e-3,1e-2")
    ap.add_argument("--big", type=int, default=5000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from cask_amd import ScanContext
    ctx = ScanContext(0)
    dev = torch.device("cuda", 0)
    res = []
    for frac in [float(x) for x in args.fracs.split(",")]:
        files, ksz, vsz, n = files_with_keys(ctx, torch, args.gib, frac, args.big)
        views = [(f.file_id, f.data) for f in files]
        nbytes = sum(f.data.numel() for f in files)
        rows = ctx.alloc_rows(n + 16)
        r = ctx.scan_device(views, rows)
        assert r.error is None and r.count == n, (r.count, n, r.error)
        assert int((rows["status"][:n] != 0).sum().item()) == 0
        assert bool((rows["seq"][:n].to(torch.int64) == torch.arange(1, n + 1, device=dev)).all())
        assert bool((rows["ksz"][:n].to(torch.int64) == ksz.to(torch.int64)).all())
        assert bool((rows["vsz"][:n].to(torch.int64) == vsz.to(torch.int64)).all())
        counters = ctx.last_counters()
        for _ in range(2):
            ctx.scan_device(views, rows)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ctx.scan_device(views, rows)
        torch.cuda.synchronize(dev)
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        o = {"frac_big_keys": frac, "big_key_bytes": args.big, "records": n, "big_records": int((ksz > 16).sum().item()),
             "bytes": nbytes, "ms_per_scan": ms, "gibps": nbytes / (ms * 1e-3) / 2 ** 30, "counters": counters,
             "breakdown_ms": ctx.last_timings()}
        print(json.dumps(o), flush=True)
        res.append(o)
        del files, views, rows
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

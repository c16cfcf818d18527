"""A/B timing of library builds on one box (tools only; bench.py always times the product build).

  python tools/ab.py [--rounds 3] [--steps 20] NAME=PATH[@VAR=VALUE,...] [NAME=PATH ...]

Each build runs in its own process (the library is picked with cask_amd._lib.use_library, never by
an environment variable the package reads); the builds alternate `--rounds` times so box drift
hits them alike. Prints the headline loop's GiB/s and the chunk-scan kernel time per run.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(path, steps, files, zipf_gib):
    sys.path.insert(0, ROOT)
    import torch
    import cask_amd
    if path != "product":
        cask_amd._lib.use_library(path)
    ctx = cask_amd.ScanContext(0)
    want = None
    if zipf_gib > 0:  # configs[2]-shaped
        from cask_amd.workloads import zipf_files
        fs, vsz_all, n, _ = zipf_files(ctx, zipf_gib, 2 ** 31)
        want = (n, vsz_all[:n].clone())
        fs = [f for f, _ in fs]
    else:
        from cask_amd.workloads import cfg2_files
        fs = cfg2_files(ctx, nfiles=files)
        n = sum(f.nrec for f in fs)
    views = [(f.file_id, f.data) for f in fs]
    rows = ctx.alloc_rows(n + 16)
    nbytes = sum(f.data.numel() for f in fs)
    seg = False
    call = (lambda: ctx.scan_device(views, rows))
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    k = []
    t0 = time.perf_counter()
    for _ in range(steps):
        call()
        k.append(ctx.last_timings()["chunk_scan_ms"])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if os.environ.get("AB_NOCHECK") == "1":  # timing diagnostics whose rows are known wrong
        want = None
    if want is not None and not seg:  # the last call's rows against the generator (a variant that
        res = call()                   # is fast and wrong fails here)
        torch.cuda.synchronize()
        wn, wv = want
        assert res.error is None and res.count == wn, (res.error, res.count, wn)
        assert int((rows["status"][:wn] != 0).sum().item()) == 0
        assert torch.equal(rows["vsz"][:wn].to(torch.int64), wv.to(torch.int64))
        assert torch.equal(rows["seq"][:wn].to(torch.int64), torch.arange(1, wn + 1, device=wv.device))
        assert int((rows["ksz"][:wn] != 16).sum().item()) == 0
    print(json.dumps({"gibps": nbytes * steps / el / 2 ** 30, "ms_per_step": el * 1e3 / steps,
                      "k_scan_ms": sum(k) / len(k), "timings": ctx.last_timings(),
                      "geometry": ctx.last_counters()["geometry"]}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--files", type=int, default=8)
    ap.add_argument("--child", default="")
    ap.add_argument("--zipf-gib", type=float, default=0.0, help="configs[2]-shaped files of this size")
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a.child, a.steps, a.files, a.zipf_gib)
    for r in range(a.rounds):
        for spec in a.libs:
            name, path = spec.split("=", 1)
            env = dict(os.environ)
            if "@" in path:  # NAME=PATH@VAR=VALUE[,VAR=VALUE]: environment of that run only
                path, kv = path.split("@", 1)
                env.update(x.split("=", 1) for x in kv.split(","))
            out = subprocess.run([sys.executable, __file__, "--child", path, "--steps", str(a.steps),
                                  "--files", str(a.files), "--zipf-gib", str(a.zipf_gib)],
                                 capture_output=True, text=True, timeout=300, env=env)
            if out.returncode != 0:
                print(name, "FAILED", out.stderr[-2000:])
                sys.exit(1)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            print(f"round {r} {name}: {d['gibps']:.1f} GiB/s  {d['ms_per_step']:.4f} ms/step  "
                  f"k_scan {d['k_scan_ms']:.4f} ms  {json.dumps(d['timings'])} geo {d.get('geometry')}", flush=True)


if __name__ == "__main__":
    main()

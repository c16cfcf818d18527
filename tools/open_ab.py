"""A/B of open() (Cask::open without hint files: read, scan, hint files, fold) between library
builds on one box: one configs[3]-shaped database in /dev/shm, opened in turn by each build in its
own process, its hint files removed before every open (tools only).

  python tools/open_ab.py [--files 64] [--rounds 2] NAME=PATH [NAME=PATH ...]   (PATH "product")
"""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, path, live):
    sys.path.insert(0, ROOT)
    import cask_amd
    if lib != "product":
        cask_amd._lib.use_library(lib)
    from cask_amd import CaskOptions, ScanContext
    ScanContext(0)  # (the HIP runtime initialised before the clock starts, as in a running process)
    for h in glob.glob(os.path.join(path, "*.cask.hint")):
        os.unlink(h)
    nbytes = sum(os.path.getsize(f) for f in glob.glob(os.path.join(path, "*.cask.data")))
    t0 = time.perf_counter()
    with CaskOptions().max_file_size(1 << 30).open(path) as db:
        el = time.perf_counter() - t0
        assert len(db) == live, (len(db), live)
        print(json.dumps({"open_s": el, "gibps": nbytes / el / 2 ** 30, "timings_ms": db.open_timings()}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", nargs=3)
    ap.add_argument("--precat", action="store_true", help="read every data file once before the rounds")
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a.child[0], a.child[1], int(a.child[2]))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    work = tempfile.mkdtemp(prefix="cask_open_ab_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        path = os.path.join(work, "db")
        os.makedirs(path)
        p = subprocess.run([sys.executable, "-c", f"""
import sys, json; sys.path.insert(0, {ROOT!r}); sys.path.insert(0, {os.path.join(ROOT, 'tools')!r})
import torch; from cask_amd import ScanContext; import bench_configs as B
ctx = ScanContext(0); print(json.dumps(B.write_cfg3(ctx, torch, {a.files}, {path!r})))"""],
                           capture_output=True, text=True, timeout=600)
        if p.returncode:
            print(p.stderr[-3000:])
            sys.exit(1)
        nbytes, live, n, ws = json.loads(p.stdout.strip().splitlines()[-1])
        print(f"{a.files} files, {nbytes} bytes, {n} records, {live} live keys, written in {ws:.1f} s", flush=True)
        if a.precat:  # (is the first open's slower read the open's, or the freshly written pages'?)
            t0 = time.perf_counter()
            for f in sorted(glob.glob(os.path.join(path, "*.cask.data"))):
                with open(f, "rb") as fh:
                    while fh.read(64 << 20):
                        pass
            print(f"files read once in {time.perf_counter() - t0:.1f} s", flush=True)
        for r in range(a.rounds):
            for spec in a.libs:
                name, lib = spec.split("=", 1)
                out = subprocess.run([sys.executable, __file__, "--child", lib, path, str(live)],
                                     capture_output=True, text=True, timeout=600)
                if out.returncode:
                    print(name, "FAILED", out.stderr[-2000:])
                    sys.exit(1)
                d = json.loads(out.stdout.strip().splitlines()[-1])
                print(f"round {r} {name}: open {d['open_s']:.3f} s = {d['gibps']:.2f} GiB/s "
                      f"{ {k: round(v) for k, v in d['timings_ms'].items()} }", flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()

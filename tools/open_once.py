"""configs[3]-shaped files written to a temporary directory (tools/bench_configs.py write_cfg3), then
cask_db_open with the keydir reduced on the device, --opens times, no hint files written: a short
program to run under rocprofv3 for the open's kernels (the block build, k_kd_* and the sort).
python tools/open_once.py [--files 64] [--opens 2] [--dir /dev/shm]"""
import argparse
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=64)
    ap.add_argument("--opens", type=int, default=2)
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    from cask_amd import CaskOptions, ScanContext
    from bench_configs import write_cfg3
    ctx = ScanContext(0)
    wd = tempfile.mkdtemp(prefix="cask_open_", dir=a.dir)
    try:
        path = os.path.join(wd, "db")
        os.makedirs(path)
        _, live, n, _ = write_cfg3(ctx, torch, a.files, path)
        del ctx
        torch.cuda.empty_cache()
        for i in range(a.opens):
            t0 = time.perf_counter()
            with CaskOptions().write_hints(False).open(path) as db:
                dt = time.perf_counter() - t0
                assert len(db) == live
                print(f"open {i}: {dt:.2f} s {db.open_timings()}", flush=True)
    finally:
        shutil.rmtree(wd, ignore_errors=True)


if __name__ == "__main__":
    main()

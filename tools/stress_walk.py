"""Repeated walk-mode scans (k_finish beside k_run_hash, k_hash_fix after) of Zipf-length files with
checksum failures spread over many chunks, every call's rows against the oracle's (tools only: a
concurrency check of the side-stream path). python tools/stress_walk.py [--calls 200]"""
import argparse
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    import numpy as np
    import torch
    import cask_amd
    import test_scan_gpu as T
    ctx = cask_amd.ScanContext(0)
    rng = random.Random(7)
    sets = []
    for k in range(3):
        buf = bytearray(T.make_records(rng, 20000, lambda r: 16, T._zipf_vsz(rng), tomb_p=0.02, seq0=1 + 100000 * k))
        for _ in range(40 * (k + 1)):
            buf[rng.randrange(len(buf))] ^= 1 << rng.randrange(8)
        sets.append([bytes(buf), bytes(buf[: len(buf) // 2])])
    want = []
    for bufs in sets:
        rows = [T.oracle_rows(b)[0] for b in bufs]
        want.append(rows)
    dev = [[torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda() for b in bufs] for bufs in sets]
    t0 = time.time()
    for c in range(a.calls):
        i = c % len(sets)
        res = ctx.scan_device(list(enumerate(dev[i], start=1)))
        res.pos, res.seq, res.vsz, res.ksz, res.status = [t[:res.count].cpu().numpy() for t in
                                                          (res.pos, res.seq, res.vsz, res.ksz, res.status)]
        for f, w in enumerate(want[i]):
            got = T.rows_list(res, res.file_rows(f))
            assert got == w, (c, f)
        if c % 50 == 0:
            print(f"call {c}: ok ({time.time() - t0:.1f} s), walk_mode {ctx.last_counters()['walk_mode']}", flush=True)
    print(f"{a.calls} calls, every row equal to the oracle's")


if __name__ == "__main__":
    main()

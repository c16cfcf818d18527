"""Diagnostic for the search fallback A/B: one configs[2]-shaped GiB scanned by a library build, its
counters (repaired chunks = speculated run starts that k_finish rejected), and a host model of the
fallback rule over the same bytes for the runs whose first `--win` windows hold no short record.

  python tools/search_fallback_check.py LIB [--win 2]
"""
import argparse
import sys
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--win", type=int, default=2)
    ap.add_argument("--gib", type=float, default=1.0)
    a = ap.parse_args()
    import torch
    import cask_amd
    if a.lib != "product":
        cask_amd._lib.use_library(a.lib)
    from cask_amd.workloads import zipf_files
    ctx = cask_amd.ScanContext(0)
    fs, vsz, n, rl = zipf_files(ctx, a.gib, 2 ** 31)
    res = ctx.scan_device([(f.file_id, f.data) for f, _ in fs])
    print("counters", ctx.last_counters(), "error", res.error, flush=True)
    # host model over the first file
    f, idx = fs[0]
    buf = f.data.cpu().numpy()
    L = len(buf)
    rlh = rl[int(idx[0]):int(idx[-1]) + 1].cpu().numpy()
    starts = np.concatenate([[0], np.cumsum(rlh)[:-1]])
    W = 8192 - 16 - 18

    def hdr(p):
        ksz = int(buf[p + 12]) | int(buf[p + 13]) << 8
        v = int(buf[p + 14]) | int(buf[p + 15]) << 8 | int(buf[p + 16]) << 16 | int(buf[p + 17]) << 24
        return ksz, v, 18 + ksz + (0 if v == 0xFFFFFFFF else v)

    def probe(p):
        for j in range(4):
            if p == L:
                return j > 0
            if p + 18 > L:
                return False
            ksz, v, r = hdr(p)
            if ksz > 4096 or p + r > L:
                return False
            p += r
        return True

    good = bad = none = tried = 0
    for b0 in range(1 << 20, L - (2 << 20), 1 << 20):
        lim = min(b0 + (2 << 20), L)
        k = np.searchsorted(starts, b0)
        s_true = int(starts[k])
        span = b0 + a.win * W
        reals = [int(x) for x in starts[k:k + 64] if x < span]
        if any(rlh[np.searchsorted(starts, x)] <= 2048 for x in reals):
            continue
        tried += 1
        lst = []
        seg = buf[b0:span + 18]
        cand = np.flatnonzero(((seg[17:] == 0) | (seg[17:] == 255)) & (seg[13:len(seg) - 4] <= 0x10)) + b0
        for x in cand:
            x = int(x)
            if x >= span or x + 18 > L:
                continue
            ksz, v, r = hdr(x)
            if r > 2048 and x + r <= lim:
                lst.append((x, x + r))
        passing = [x for x, e in lst if probe(e)]
        if not passing:
            none += 1
            continue
        t = min(passing)
        while True:
            c = [s for s, e in lst if s < t and e == t]
            if not c:
                break
            t = min(c)
        if t == s_true:
            good += 1
        else:
            bad += 1
            if bad <= 5:
                print("bad run at", b0, "true", s_true, "picked", min(passing), "hopped to", t, "list", len(lst))
    print(f"host model over file 1: runs tried {tried} good {good} bad {bad} none {none}")


if __name__ == "__main__":
    main()

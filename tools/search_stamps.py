"""Phase breakdown of k_walk_search (split walk path) from the diagnostic build (make -C cask_amd
stamps): configs[2]-shaped files (--gib). Per-wave s_memtime cycle sums: shares of the search's time,
and per search the windows staged and candidate rounds hashed."""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STAMPS_LIB = os.path.join(ROOT, "cask_amd", "build", "stamps", "libcask_scan.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=32.0)
    ap.add_argument("--calls", type=int, default=3)
    ap.add_argument("--lib", default=STAMPS_LIB, help="a stamps build (make stamps, or a variant with -DCASK_STAMPS)")
    args = ap.parse_args()
    import torch
    import cask_amd
    cask_amd._lib.use_library(args.lib)
    from cask_amd.workloads import zipf_files
    L = cask_amd.lib()
    L.cask_debug_stamps.restype = C.c_int
    L.cask_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    ctx = cask_amd.ScanContext(0)
    files = [f for f, _ in zipf_files(ctx, args.gib, 2 ** 31)[0]]
    views = [(f.file_id, f.data) for f in files]
    for _ in range(args.calls):
        res = ctx.scan_device(views)
        torch.cuda.synchronize()
    st = (C.c_uint64 * 16)()
    L.cask_debug_stamps(ctx._h, st)
    names = ["total", "stage", "phase1 decode", "phase2 hash", "hop back", "windows", "hash rounds", "searches"]
    for i, n in enumerate(names):
        print(f"{n:14s} {st[i]}")
    tot = st[0] or 1
    ns = st[7] or 1
    print(f"shares: stage {st[1] / tot:.2f} phase1 {st[2] / tot:.2f} phase2 {st[3] / tot:.2f} hop {st[4] / tot:.2f}; "
          f"per search: {st[0] / ns:.0f} cycles, {st[5] / ns:.2f} windows, {st[6] / ns:.2f} hash rounds")
    print("timings", ctx.last_timings(), "counters", ctx.last_counters(), "rows", res.count)
    # per-search records of the last call: start / end (100 MHz real-time clock), windows, wave
    import numpy as np
    nr = 65536
    L.cask_debug_search_stamps.restype = C.c_int
    L.cask_debug_search_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint64]
    buf = (C.c_uint64 * (4 * nr))()
    L.cask_debug_search_stamps(ctx._h, buf, 4 * nr)
    a = np.frombuffer(buf, np.uint64).reshape(nr, 4).astype(np.int64)
    a = a[a[:, 1] > 0]
    if a.size:
        t0 = a[:, 0].min()
        st, en, win = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0, a[:, 2]
        dur = en - st
        print(f"searches {len(a)}: kernel span {en.max():.1f} us; per search us mean {dur.mean():.1f} "
              f"p50/p90/p99/max {' / '.join(f'{x:.1f}' for x in np.percentile(dur, [50, 90, 99, 100]))}")
        print(f"windows mean {win.mean():.2f} max {win.max()}; us per window {dur.sum() / max(win.sum(), 1):.2f}")
        hist = np.bincount(np.minimum(win, 32))
        print("windows histogram (searches with k windows, k = 0..31, 32+):", hist.tolist())
        for lo, hi in ((0, 2), (3, 5), (6, 10), (11, 20), (21, 1 << 30)):
            m = (win >= lo) & (win <= hi)
            print(f"  windows {lo}-{hi if hi < 1 << 30 else 'max'}: {int(m.sum())} searches, {dur[m].sum():.0f} us total")
        w_last = a[np.argmax(a[:, 1]), 3]
        mine = a[a[:, 3] == w_last]
        print(f"last wave {w_last}: {len(mine)} searches, windows {mine[:, 2].tolist()}, "
              f"durations {[round(x, 1) for x in ((mine[:, 1] - mine[:, 0]) / 100.0).tolist()]}")
        ends = {}
        for e_, w_ in zip(en, a[:, 3]):
            ends[w_] = max(ends.get(w_, 0.0), e_)
        ev = np.array(sorted(ends.values()))
        print(f"waves {len(ev)}: end percentiles 0/10/50/90/99/100 = "
              f"{' / '.join(f'{x:.1f}' for x in np.percentile(ev, [0, 10, 50, 90, 99, 100]))} us")


if __name__ == "__main__":
    main()

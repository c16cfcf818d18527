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
    args = ap.parse_args()
    import torch
    import cask_amd
    cask_amd._lib.use_library(STAMPS_LIB)
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


if __name__ == "__main__":
    main()

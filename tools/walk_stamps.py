"""Phase breakdown of k_walk_runs from the diagnostic build (make -C cask_amd stamps): configs[2]-shaped
files (--gib), walk mode forced. Prints per-wave s_memtime cycle sums (shares, not wall time) and counts."""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STAMPS_LIB = os.path.join(ROOT, "cask_amd", "build", "stamps", "libcask_scan.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=8.0)
    args = ap.parse_args()
    os.environ["CASK_SCAN_MODE"] = "walk"
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
    for it in range(3):
        res = ctx.scan_device(views)
        torch.cuda.synchronize()
    st = (C.c_uint64 * 16)()
    L.cask_debug_stamps(ctx._h, st)
    names = ["search cyc", "chase stage cyc", "flush hash cyc", "total cyc", "stages", "records", "searches", "-"]
    for i, n in enumerate(names):
        print(f"{n:18s} {st[i]}")
    tot = st[3] or 1
    print(f"shares: search {st[0] / tot:.2f} stage {st[1] / tot:.2f} hash {st[2] / tot:.2f} "
          f"rest {(tot - st[0] - st[1] - st[2]) / tot:.2f}")
    print("timings", ctx.last_timings(), "counters", ctx.last_counters(), "rows", res.count)


if __name__ == "__main__":
    main()

"""Phase breakdown of k_run_hash (split walk path) from the diagnostic build (make -C cask_amd
stamps): configs[2]-shaped files (--gib). Per-wave s_memtime cycle sums over the loop's phases
(shares of the kernel's wave time) and iterations per wave."""
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
    h = [st[8 + i] for i in range(8)]
    names = ["total", "plan+issue", "claim", "mix(+fin)", "finalize", "wait", "iterations", "-"]
    for n, v in zip(names, h):
        print(f"{n:12s} {v}")
    tot = h[0] or 1
    print(f"shares: plan+issue {h[1] / tot:.3f} claim {h[2] / tot:.3f} mix {h[3] / tot:.3f} (finalize {h[4] / tot:.3f}) "
          f"wait {h[5] / tot:.3f}; per iteration {h[0] / max(h[6], 1):.0f} cycles; iterations {h[6]}")
    print("timings", ctx.last_timings(), "rows", res.count)


if __name__ == "__main__":
    main()

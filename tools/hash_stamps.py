"""Per-wave timing of k_run_hash (split walk path) from the diagnostic build (make -C cask_amd
stamps): configs[2]-shaped files (--gib). Each wave's start, end and the time its runs ran out
(the kernel's tail), overall and per XCD. (Round 4's per-phase cycle sums belonged to the
quad-per-instruction kernel that k_run_hash replaced in round 5.)"""
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
    ctx = cask_amd.ScanContext(0)
    files = [f for f, _ in zipf_files(ctx, args.gib, 2 ** 31)[0]]
    views = [(f.file_id, f.data) for f in files]
    for _ in range(args.calls):
        res = ctx.scan_device(views)
        torch.cuda.synchronize()
    print("timings", ctx.last_timings(), "rows", res.count)
    # per-wave start/end (100 MHz real-time clock) of the last call's k_run_hash
    nw = 8192
    L.cask_debug_wave_stamps.restype = C.c_int
    L.cask_debug_wave_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint64]
    ws = (C.c_uint64 * (2 * nw))()
    L.cask_debug_wave_stamps(ctx._h, ws, 2 * nw)
    import numpy as np
    a = np.frombuffer(ws, np.uint64).reshape(nw, 2).astype(np.int64)
    a = a[a[:, 1] > 0]
    if a.size:
        t0 = a[:, 0].min()
        st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0  # us
        span = en.max()
        q = np.percentile(en, [0, 10, 50, 90, 99, 100])
        print(f"waves {len(a)}: span {span:.1f} us; start spread {st.max():.1f} us; end percentiles "
              f"0/10/50/90/99/100 = {' / '.join(f'{x:.1f}' for x in q)} us")
        print(f"idle after finishing: {np.mean(span - en) / span:.3f} of wave-time; "
              f"tail (max - median end) {span - q[2]:.1f} us")
        # per wave: when its runs ran out (the claim counter was past the last unit) -> its end
        L.cask_debug_dry_stamps.restype = C.c_int
        L.cask_debug_dry_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_uint64]
        dr = (C.c_uint64 * nw)()
        L.cask_debug_dry_stamps(ctx._h, dr, nw)
        full = np.frombuffer(ws, np.uint64).reshape(nw, 2).astype(np.int64)
        dry = np.frombuffer(dr, np.uint64).astype(np.int64)
        ok = (full[:, 1] > 0) & (dry > 0)
        if ok.any():
            dry_t = (dry[ok] - t0) / 100.0
            drain = (full[ok, 1] - dry[ok]) / 100.0
            print(f"runs ran out at p10/p50/p90/max {' / '.join(f'{x:.0f}' for x in np.percentile(dry_t, [10, 50, 90, 100]))} us; "
                  f"drain after that p10/p50/p90/max {' / '.join(f'{x:.0f}' for x in np.percentile(drain, [10, 50, 90, 100]))} us")
        # per XCD (workgroups are dealt to the 8 XCDs round-robin: XCD = workgroup % 8)
        wid = np.flatnonzero(np.frombuffer(ws, np.uint64).reshape(nw, 2)[:, 1] > 0)
        xcd = (wid // 4) % 8
        for x in range(8):
            e = en[xcd == x]
            if e.size:
                print(f"  XCD {x}: {e.size} waves, end p10/p50/p90/max "
                      f"{' / '.join(f'{v:.0f}' for v in np.percentile(e, [10, 50, 90, 100]))} us")


if __name__ == "__main__":
    main()

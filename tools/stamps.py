"""Phase breakdown of k_scan_chunks from the diagnostic build (make -C cask_amd stamps).

python tools/stamps.py [--files N]   (after make -C cask_amd stamps)
Prints the average s_memtime cycles per workgroup spent in each phase (shares, not wall time:
the stamps serialise what the real kernel overlaps).
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STAMPS_LIB = os.path.join(ROOT, "cask_amd", "build", "stamps", "libcask_scan.so")

PHASES = ["search", "walk", "hash+slots", "stage wait+store", "(iterations)", "prefetch issue", "end barrier", "TOTAL loop", "  rec hdr+hash", "  rec store issue"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=2)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--zipf-gib", type=float, default=0.0, help="configs[2]-shaped files instead of configs[1]")
    args = ap.parse_args()
    import torch
    import cask_amd
    cask_amd._lib.use_library(STAMPS_LIB)
    from cask_amd.workloads import cfg2_files
    L = cask_amd.lib()
    L.cask_debug_stamps.restype = C.c_int
    L.cask_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    ctx = cask_amd.ScanContext(0)
    if args.zipf_gib > 0:
        from cask_amd.workloads import zipf_files
        files = [f for f, _ in zipf_files(ctx, args.zipf_gib, 2 ** 31)[0]]
    else:
        files = cfg2_files(ctx, nfiles=args.files)
    views = [(f.file_id, f.data) for f in files]
    rows = ctx.alloc_rows(sum(f.nrec for f in files) + 16)
    res = None
    for _ in range(args.iters):
        try:
            res = ctx.scan_device(views, rows)
        except Exception as e:  # CASK_NO_REPAIR: an unrepaired speculative pass reports status 1
            if not os.environ.get("CASK_NO_REPAIR"):
                raise
            print("unrepaired pass:", e)
    st = (C.c_uint64 * 16)()
    L.cask_debug_stamps(ctx._h, st)
    chunks = ctx.last_counters()["chunks"] or None
    t = ctx.last_timings()
    print(f"chunks={chunks} rows={res.count if res else '-'} timings={t}")
    tot = st[7]
    chunks = chunks or max(st[4], 1)
    print(f"chunk iterations stamped: {st[4]}")
    if st[13]:
        mean_ns = st[11] * 10.0 / st[13]
        print(f"workgroups {st[13]}: mean life {mean_ns / 1e3:.1f} us, max {st[12] * 10.0 / 1e3:.1f} us "
              f"(summed over {args.iters} calls); s_memtime units per ns {st[7] / (st[11] * 10.0):.3f}")
    for i, p in enumerate(PHASES):
        print(f"{p:14s} {st[i] / chunks:12.0f} cyc/WG  {100.0 * st[i] / max(tot, 1):5.1f}%")


if __name__ == "__main__":
    main()

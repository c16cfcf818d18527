"""Diagnostic: best-of chunk-scan time of the library at $CASK_LIB_PATH on the configs[1] files
(dense output as bench.py, or segmented with CASK_TV_SEGMENTED=1; repair off), to compare kernel
variants built with `make variant`."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["CASK_NO_REPAIR"] = "1"


def main():
    import cask_amd
    from cask_amd.workloads import cfg2_files
    ctx = cask_amd.ScanContext(0)
    files = cfg2_files(ctx, nfiles=8)
    views = [(f.file_id, f.data) for f in files]
    total = sum(f.data.numel() for f in files)
    seg = bool(os.environ.get("CASK_TV_SEGMENTED"))
    rows = None if seg else ctx.alloc_rows(sum(f.nrec for f in files))
    ms = []
    for it in range(8):
        try:
            ctx.scan_device_segmented(views) if seg else ctx.scan_device(views, rows)
        except Exception as e:  # diagnostic builds produce wrong rows; only the timing matters
            if it == 0:
                print(f"  ({type(e).__name__}: {str(e)[:120]})")
        ms.append(ctx.last_timings()["chunk_scan_ms"])
    if max(ms) == 0:
        print("no timing recorded")
        return
    best = min(ms[2:])
    label = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("CASK_LIB_PATH", "default")
    print(f"{label}: k_scan {best:.3f} ms  {total / best / 1e6:.0f} GB/s  (all: {[round(m, 3) for m in ms]})")


if __name__ == "__main__":
    main()

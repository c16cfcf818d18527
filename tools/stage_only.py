"""Diagnostic: time k_scan_chunks built with -DCASK_STAGE_ONLY (staging + prefetch, no
processing) on the configs[1] files, to separate the memory side from the processing side."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CASK_LIB_PATH", os.path.join(ROOT, "cask_amd", "build", "stageonly", "libcask_scan.so"))
os.environ["CASK_NO_REPAIR"] = "1"


def main():
    import cask_amd
    from cask_amd.workloads import cfg2_files
    ctx = cask_amd.ScanContext(0)
    files = cfg2_files(ctx, nfiles=8)
    views = [(f.file_id, f.data) for f in files]
    total = sum(f.data.numel() for f in files)
    ms = []
    for it in range(8):
        try:
            ctx.scan_device_segmented(views)
        except Exception:
            pass
        ms.append(ctx.last_timings()["chunk_scan_ms"])
    best = min(ms[2:])
    print(f"stage-only k_scan: {best:.3f} ms  {total / best / 1e6:.0f} GB/s  (all: {[round(m, 3) for m in ms]})")


if __name__ == "__main__":
    main()

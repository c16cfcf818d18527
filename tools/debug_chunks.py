"""Diagnostic: speculative-pass chunk table for cfg2 files vs the exact layout (diagnostic build)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CASK_LIB_PATH", os.path.join(ROOT, "cask_amd", "build", "stamps", "libcask_scan.so"))
os.environ["CASK_NO_REPAIR"] = "1"


def main():
    nfiles = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import cask_amd
    from cask_amd.workloads import cfg2_files
    L = cask_amd.lib()
    L.cask_debug_chunks.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_uint64]
    ctx = cask_amd.ScanContext(0)
    files = cfg2_files(ctx, nfiles=nfiles)
    views = [(f.file_id, f.data) for f in files]
    rows = ctx.alloc_rows(sum(f.nrec for f in files))
    for it in range(3):
        try:
            ctx.scan_device(views, rows)
        except Exception as e:  # rc 1 = invalid chunks present
            print("scan raised:", e)
        CH0 = {"0": 32768, "1": 16384, "2": 8192}[os.environ.get("CASK_SCAN_GEOMETRY", "0")]
        n = nfiles * ((files[0].data.numel() + CH0 - 1) // CH0)
        spec = np.zeros(n, np.uint64); ex = np.zeros(n, np.uint64); tin = np.zeros(n, np.uint64)
        cnt = np.zeros(n, np.uint32)
        L.cask_debug_chunks(ctx._h, spec.ctypes.data, ex.ctypes.data, tin.ctypes.data, cnt.ctypes.data, n)
        CH = CH0
        per_file = n // nfiles
        c = np.arange(per_file, dtype=np.uint64)
        c0 = c * CH
        length = files[0].data.numel()
        c1 = np.minimum(c0 + CH, length)
        want_spec = (c0 + 289) // 290 * 290
        want_exit = (c1 + 289) // 290 * 290
        want_cnt = (want_exit - want_spec) // 290
        bad = 0
        for f in range(nfiles):
            sl = slice(f * per_file, (f + 1) * per_file)
            ws = want_spec.copy(); ws[0] = 0
            wrong = np.nonzero((spec[sl] != ws) | (ex[sl] != want_exit) | (cnt[sl] != want_cnt))[0]
            bad += len(wrong)
            for w in wrong[:5]:
                print(f"iter {it} file {f} chunk {w}: spec {spec[sl][w]} want {ws[w]} exit {ex[sl][w]} want {want_exit[w]} "
                      f"count {cnt[sl][w]} want {want_cnt[w]} tin {tin[sl][w]}")
        print(f"iter {it}: {bad} wrong chunks of {n}")


if __name__ == "__main__":
    main()

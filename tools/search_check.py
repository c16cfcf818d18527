"""Diagnostic (stamps build, CASK_NO_REPAIR): k_walk_search's speculative run starts against the true
first record start of each run, on a configs[1]-shaped file (fixed 290-B records) and a Zipf file,
walk mode forced. Prints the mismatches."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STAMPS_LIB = os.path.join(ROOT, "cask_amd", "build", "stamps", "libcask_scan.so")


def main():
    os.environ["CASK_TEST_HOOKS"] = "1"
    os.environ["CASK_SCAN_MODE"] = "walk"
    os.environ["CASK_NO_REPAIR"] = "1"
    import numpy as np
    import torch
    import cask_amd
    cask_amd._lib.use_library(STAMPS_LIB)
    from cask_amd.workloads import cfg2_files, zipf_files
    L = cask_amd.lib()
    L.cask_debug_chunks.restype = C.c_int
    L.cask_debug_chunks.argtypes = [C.c_void_p] + [C.c_void_p] * 4 + [C.c_uint64]
    ctx = cask_amd.ScanContext(0)
    for name in ("cfg1", "zipf"):
        if name == "cfg1":
            f = cfg2_files(ctx, nfiles=1, records_per_file=(256 << 20) // 290)[0]
            starts = np.arange(f.nrec + 1, dtype=np.int64) * 290
        else:
            fs, vsz, n, rl = zipf_files(ctx, 0.5, 2 ** 31)
            f = fs[0][0]
            r = rl[fs[0][1]].cpu().numpy().astype(np.int64)
            starts = np.concatenate([[0], np.cumsum(r)])
        try:
            ctx.scan_device([(1, f.data)])
        except cask_amd.errors.Error as e:  # CASK_NO_REPAIR: an invalid speculation ends the call
            print(name, "scan:", e)
        torch.cuda.synchronize()
        nch = (f.data.numel() + 32767) // 32768
        spec = np.zeros(nch, np.uint64); ex = np.zeros(nch, np.uint64); tin = np.zeros(nch, np.uint64)
        cnt = np.zeros(nch, np.uint32)
        rc = L.cask_debug_chunks(ctx._h, spec.ctypes.data, ex.ctypes.data, tin.ctypes.data, cnt.ctypes.data, nch)
        assert rc == 0, rc
        R = 32
        bad = 0
        for t0 in range(R, nch, R):
            b0 = t0 * 32768
            want = int(starts[np.searchsorted(starts, b0)])
            got = int(tin[t0])
            if got != want:
                bad += 1
                if bad <= 10:
                    print(name, "run", t0 // R, "b0", b0, "want", want, "got", got, "got-b0", got - b0, "want-b0", want - b0)
        print(name, "runs", nch // R, "bad", bad, "counters", ctx.last_counters())


if __name__ == "__main__":
    main()

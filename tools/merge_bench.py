"""Host fold of one keydir block (cask_keydir_merge + cask_keydir_finish), timed on this machine's
threads: a synthetic block of N unique 16-B keys (kind kKept, 64 files), the shape of configs[3]'s
device-reduced open. CPU only (no GPU needed): python tools/merge_bench.py [N [LIB]]."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def block(n, nfiles=64, seed=1):
    rng = np.random.default_rng(seed)
    hdr = np.zeros(8, np.uint64)
    rec = np.zeros(n, dtype=[("pos", "<u8"), ("seq", "<u8"), ("file_id", "<u4"), ("vsz", "<u4"), ("ksz", "<u2"),
                             ("kind", "u1"), ("pad0", "u1"), ("pad1", "<u4")])
    rec["pos"] = rng.integers(0, 1 << 30, n)
    rec["seq"] = np.arange(1, n + 1)
    rec["file_id"] = rng.integers(1, nfiles + 1, n)
    rec["vsz"] = 256
    rec["ksz"] = 16
    fst = np.zeros(nfiles, dtype=[("file_id", "<u4"), ("pad", "<u4"), ("puts", "<u8"), ("put_bytes", "<u8"),
                                  ("stale", "<u8"), ("stale_bytes", "<u8")])
    fst["file_id"] = np.arange(1, nfiles + 1)
    cnt = np.bincount(rec["file_id"], minlength=nfiles + 1)[1:]
    fst["puts"] = cnt
    fst["put_bytes"] = cnt * (18 + 16 + 256)
    keys = rng.integers(0, 256, n * 16, dtype=np.uint8)
    body = rec.tobytes() + fst.tobytes() + keys.tobytes()
    total = 64 + len(body)
    total = (total + 7) // 8 * 8
    h = np.zeros(1, dtype=[("magic", "<u4"), ("version", "<u4"), ("nrec", "<u8"), ("key_bytes", "<u8"), ("nfiles", "<u4"),
                          ("pad", "<u4"), ("max_seq_p1", "<u8"), ("rows_in", "<u8"), ("bytes", "<u8"), ("pad2", "<u8")])
    h["magic"], h["version"], h["nrec"], h["key_bytes"], h["nfiles"] = 0x52444B43, 1, n, n * 16, nfiles
    h["max_seq_p1"], h["rows_in"], h["bytes"] = n + 1, n, total
    out = bytearray(h.tobytes() + body)
    out += b"\0" * (total - len(out))
    return bytes(out)


def main():
    os.environ.setdefault("CASK_TEST_HOOKS", "1")
    os.environ.setdefault("CASK_OPEN_TRACE", "1")
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    import cask_amd
    if len(sys.argv) > 2:  # an A/B build of the library
        cask_amd._lib.use_library(sys.argv[2])
    L = cask_amd.lib()
    b = block(n)
    for _ in range(2):
        db = L.cask_keydir_new()
        t0 = time.perf_counter()
        st = L.cask_keydir_merge(db, b, len(b))
        t1 = time.perf_counter()
        st2 = L.cask_keydir_finish(db)
        t2 = time.perf_counter()
        assert st == 0 and st2 == 0, (st, st2)
        print(f"{n} records: merge {1e3 * (t1 - t0):.1f} ms, finish {1e3 * (t2 - t1):.1f} ms, live {L.cask_db_len(db)}", flush=True)
        L.cask_db_close(db)


if __name__ == "__main__":
    main()

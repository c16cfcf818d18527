"""Host fold microbenchmark (no GPU needed): Cask::open over hint files only (log.rs:121-135), so
the timed work is the hint parse + the keydir fold (Index::update + Stats, cask.rs:60-90) that the
scanned path runs on the rows the device returns.

The database is configs[3]-shaped: files of 3,702,558 records of 16-B keys drawn from a key space of
20 % of the records, 10 % of keys ending in a tombstone; each file holds only its hint file (and an
empty data file, so find_data_files lists it).

  python tools/fold_bench.py --files 16 --reps 3 [--dir /dev/shm]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

RPF = 3_702_558


def splitmix(x):
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def write_db(path, nfiles, seed=0xC0FFEE):
    import xxhash
    rng = np.random.default_rng(seed)
    n = nfiles * RPF
    nkeys = n // 5
    kid = rng.integers(0, nkeys, n, dtype=np.int64)
    last = np.full(nkeys, -1, np.int64)
    np.maximum.at(last, kid, np.arange(n))
    present = last >= 0
    tomb = (rng.random(nkeys) < 0.1) & present
    vsz = np.full(n, 256, np.uint32)
    vsz[last[tomb]] = 0xFFFFFFFF
    live = int((present & ~tomb).sum())
    dt = np.dtype([("seq", "<u8"), ("ksz", "<u2"), ("vsz", "<u4"), ("pos", "<u8"), ("k0", "<u8"), ("k1", "<u8")])
    assert dt.itemsize == 38
    for i in range(nfiles):
        sl = slice(i * RPF, (i + 1) * RPF)
        h = np.zeros(RPF, dt)
        h["seq"] = np.arange(i * RPF, (i + 1) * RPF, dtype=np.uint64) + 1
        h["ksz"] = 16
        h["vsz"] = vsz[sl]
        size = np.where(vsz[sl] == 0xFFFFFFFF, 34, 290).astype(np.uint64)
        h["pos"] = np.concatenate([[0], np.cumsum(size)[:-1]]).astype(np.uint64)
        k = kid[sl].astype(np.uint64)
        h["k0"] = splitmix(k)
        h["k1"] = splitmix(k ^ np.uint64(0x5555))
        body = h.tobytes()
        fid = i + 1
        with open(os.path.join(path, f"{fid:010}.cask.hint"), "wb") as f:
            f.write(body)
            f.write(xxhash.xxh32_intdigest(body).to_bytes(4, "little"))
        open(os.path.join(path, f"{fid:010}.cask.data"), "wb").close()
    return n, live


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/dev/shm" if os.path.isdir("/dev/shm") else None)
    ap.add_argument("--lib", default="", help="an A/B build of the library (cask_amd._lib.use_library)")
    args = ap.parse_args()
    if args.lib:
        import cask_amd
        cask_amd._lib.use_library(args.lib)
    from cask_amd import CaskOptions
    work = tempfile.mkdtemp(prefix="cask_fold_", dir=args.dir)
    try:
        t0 = time.perf_counter()
        n, live = write_db(work, args.files)
        print(f"wrote {args.files} hint files ({n} records) in {time.perf_counter() - t0:.1f} s", file=sys.stderr,
              flush=True)
        best = None
        for r in range(args.reps):
            t0 = time.perf_counter()
            with CaskOptions().open(work) as db:
                el = time.perf_counter() - t0
                assert len(db) == live, (len(db), live)
                tm = db.open_timings()
            print(json.dumps({"rep": r, "open_s": el, "records": n, "mrec_per_s": n / el / 1e6, "timings_ms": tm}),
                  flush=True)
            best = el if best is None else min(best, el)
        print(json.dumps({"files": args.files, "records": n, "live": live, "best_open_s": best,
                          "mrec_per_s": n / best / 1e6}), flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()

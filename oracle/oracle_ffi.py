"""ctypes wrapper of oracle/build/libcask_oracle.so. TEST INFRASTRUCTURE ONLY.

Loaded by tests/, __graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline leg (as
the timed CPU baseline). Never used by the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libcask_oracle.so")

ROW_DTYPE = np.dtype([("pos", "<u8"), ("seq", "<u8"), ("vsz_raw", "<u4"), ("ksz", "<u2"), ("status", "u1"),
                      ("pad", "u1"), ("expected", "<u4"), ("found", "<u4")])
assert ROW_DTYPE.itemsize == 32


class CompactResult(C.Structure):
    _fields_ = [("n_compacted", C.c_uint32), ("n_new", C.c_uint32), ("n_tomb_only", C.c_uint32),
                ("file_id_seq", C.c_uint32), ("n_out", C.c_uint64), ("live_records", C.c_uint64),
                ("tombstones", C.c_uint64), ("bytes_out", C.c_uint64), ("err_kind", C.c_int32),
                ("err_file_id", C.c_uint32), ("err_pos", C.c_uint64), ("err_expected", C.c_uint32),
                ("err_found", C.c_uint32)]


class ParallelResult(C.Structure):
    _fields_ = [("records", C.c_uint64), ("live", C.c_uint64), ("max_seq", C.c_uint64), ("digest", C.c_uint64),
                ("stats_rows", C.c_uint64), ("err_kind", C.c_int32), ("err_file_id", C.c_uint32),
                ("err_pos", C.c_uint64), ("err_expected", C.c_uint32), ("err_found", C.c_uint32)]


class ReplayResult(C.Structure):
    _fields_ = [("records", C.c_uint64), ("bytes", C.c_uint64), ("max_seq", C.c_uint64), ("err_kind", C.c_int32),
                ("err_file_id", C.c_uint32), ("err_pos", C.c_uint64), ("err_expected", C.c_uint32),
                ("err_found", C.c_uint32), ("live_keys", C.c_uint64)]


_lib = None


def build():
    import subprocess
    subprocess.run(["make", "-s"], cwd=HERE, check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, u64, u32, u16 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint16
        L.orc_xxh32.restype = u32
        L.orc_xxh32.argtypes = [vp, C.c_size_t, u32]
        L.orc_entry_encode.restype = C.c_size_t
        L.orc_entry_encode.argtypes = [u64, vp, u16, vp, u32, C.c_int, vp]
        L.orc_scan_buffer.restype = C.c_int64
        L.orc_scan_buffer.argtypes = [vp, u64, vp, u64]
        L.orc_hint_encode.restype = C.c_size_t
        L.orc_hint_encode.argtypes = [u64, u16, u32, u64, vp, vp]
        L.orc_index_new.restype = vp
        L.orc_index_new.argtypes = []
        L.orc_index_free.restype = None
        L.orc_index_free.argtypes = [vp]
        L.orc_index_update.restype = None
        L.orc_index_update.argtypes = [vp, vp, u16, u32, u64, u32, u64]
        L.orc_index_len.restype = u64
        L.orc_index_len.argtypes = [vp]
        L.orc_index_export.restype = None
        L.orc_index_export.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp]
        L.orc_index_stats.restype = u64
        L.orc_index_stats.argtypes = [vp, vp, vp, vp, vp, u64]
        L.orc_replay_file_faithful.restype = C.c_int
        L.orc_replay_file_faithful.argtypes = [C.c_char_p, C.c_char_p, u32, vp, C.POINTER(ReplayResult)]
        L.orc_replay_buffer_fast.restype = C.c_int
        L.orc_replay_buffer_fast.argtypes = [vp, u64, u32, vp, C.POINTER(ReplayResult)]
        L.orc_index_get.restype = C.c_int
        L.orc_index_get.argtypes = [vp, vp, u16, vp, vp, vp, vp]
        L.orc_compact_files.restype = C.c_int
        L.orc_compact_files.argtypes = [C.c_char_p, C.c_char_p, vp, vp, u64, u32, u64, vp, vp, u64,
                                        C.POINTER(CompactResult)]
        L.orc_entry_digest.restype = u64
        L.orc_entry_digest.argtypes = [vp, u16, u32, u64, u64, u64]
        L.orc_index_digest.restype = u64
        L.orc_index_digest.argtypes = [vp]
        L.orc_replay_parallel.restype = C.c_int
        L.orc_replay_parallel.argtypes = [vp, vp, vp, u32, u32, C.POINTER(ParallelResult), vp, vp, vp, vp, u64]
        L.orc_pindex_build.restype = vp
        L.orc_pindex_build.argtypes = [vp, vp, vp, u32, u32, C.POINTER(ParallelResult), vp, vp, vp, vp, u64]
        L.orc_pindex_free.restype = None
        L.orc_pindex_free.argtypes = [vp]
        L.orc_compact_files_fn.restype = C.c_int
        L.orc_compact_files_fn.argtypes = [C.c_char_p, C.c_char_p, vp, vp, vp, u64, u32, u64, vp, vp, u64,
                                           C.POINTER(CompactResult)]
        L.orc_hint_body.restype = C.c_int64
        L.orc_hint_body.argtypes = [vp, u64, vp, u64]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data if a.size else None


def xxh32(data: bytes, seed: int = 0) -> int:
    b = np.frombuffer(bytes(data), np.uint8)
    return int(load().orc_xxh32(_ptr(b), b.size, seed))


def entry_encode(seq: int, key: bytes, value: bytes, deleted: bool = False) -> bytes:
    out = np.zeros(18 + len(key) + (0 if deleted else len(value)), np.uint8)
    k = np.frombuffer(bytes(key), np.uint8)
    v = np.frombuffer(bytes(value), np.uint8)
    n = load().orc_entry_encode(seq, _ptr(k), len(key), _ptr(v), len(value), 1 if deleted else 0, _ptr(out))
    return out[:n].tobytes()


def scan(buf) -> np.ndarray:
    """Rows of the restated Entries iterator over one data file (ROW_DTYPE)."""
    b = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else np.ascontiguousarray(buf, np.uint8)
    cap = b.size // 18 + 2
    rows = np.zeros(cap, ROW_DTYPE)
    n = load().orc_scan_buffer(_ptr(b), b.size, rows.ctypes.data, cap)
    assert n >= 0
    return rows[:n]


def hint_file_bytes(buf, rows: np.ndarray) -> bytes:
    """Hint records of every OK row + XXH32 trailer (log.rs:367-395, 449-471)."""
    b = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
    L = load()
    parts = []
    for r in rows:
        if r["status"] != 0:
            continue
        k = b[int(r["pos"]) + 18:int(r["pos"]) + 18 + int(r["ksz"])]
        out = np.zeros(22 + k.size, np.uint8)
        L.orc_hint_encode(int(r["seq"]), int(r["ksz"]), int(r["vsz_raw"]), int(r["pos"]), _ptr(np.ascontiguousarray(k)),
                          _ptr(out))
        parts.append(out.tobytes())
    body = b"".join(parts)
    return body + xxh32(body).to_bytes(4, "little")


class Index:
    """Index::update + Stats (cask.rs:60-90, stats.rs)."""

    def __init__(self):
        self.L = load()
        self.h = self.L.orc_index_new()

    def __del__(self):
        if self.h:
            self.L.orc_index_free(self.h)
            self.h = None

    def update(self, key: bytes, file_id: int, pos: int, vsz_raw: int, seq: int):
        k = np.frombuffer(bytes(key), np.uint8)
        self.L.orc_index_update(self.h, _ptr(k), len(key), file_id, pos, vsz_raw, seq)

    def fold_rows(self, buf, rows: np.ndarray, file_id: int):
        b = np.frombuffer(buf, np.uint8) if not isinstance(buf, np.ndarray) else buf
        for r in rows:
            p, k = int(r["pos"]), int(r["ksz"])
            self.update(b[p + 18:p + 18 + k].tobytes(), file_id, p, int(r["vsz_raw"]), int(r["seq"]))

    def __len__(self):
        return int(self.L.orc_index_len(self.h))

    def export(self):
        n = len(self)
        off = np.zeros(max(n, 1), np.uint64)
        kl = np.zeros(max(n, 1), np.uint16)
        fid = np.zeros(max(n, 1), np.uint32)
        pos = np.zeros(max(n, 1), np.uint64)
        size = np.zeros(max(n, 1), np.uint64)
        seq = np.zeros(max(n, 1), np.uint64)
        self.L.orc_index_export(self.h, None, _ptr(off), _ptr(kl), None, None, None, None)
        total = int(off[n - 1] + kl[n - 1]) if n else 0
        keys = np.zeros(max(total, 1), np.uint8)
        self.L.orc_index_export(self.h, _ptr(keys), _ptr(off), _ptr(kl), _ptr(fid), _ptr(pos), _ptr(size), _ptr(seq))
        kb = keys.tobytes()
        return [[kb[int(off[i]):int(off[i]) + int(kl[i])].hex(), int(fid[i]), int(pos[i]), int(size[i]), int(seq[i])]
                for i in range(n)]

    def get(self, key: bytes):
        """Index::get (cask.rs:41-43): (file_id, pos, size, seq) or None."""
        k = np.frombuffer(bytes(key), np.uint8)
        f, p, z, q = C.c_uint32(), C.c_uint64(), C.c_uint64(), C.c_uint64()
        if not self.L.orc_index_get(self.h, _ptr(k), len(key), C.byref(f), C.byref(p), C.byref(z), C.byref(q)):
            return None
        return int(f.value), int(p.value), int(z.value), int(q.value)

    def digest(self) -> int:
        return int(self.L.orc_index_digest(self.h))

    def stats(self):
        cap = 1 << 16
        a = [np.zeros(cap, np.uint32)] + [np.zeros(cap, np.uint64) for _ in range(3)]
        n = int(self.L.orc_index_stats(self.h, *[_ptr(x) for x in a], cap))
        return [[int(a[0][i]), int(a[1][i]), int(a[2][i]), int(a[3][i])] for i in range(n)]


def replay_faithful(data_path: str, hint_path: str | None, file_id: int, index: Index) -> ReplayResult:
    r = ReplayResult()
    rc = load().orc_replay_file_faithful(data_path.encode(), hint_path.encode() if hint_path else None, file_id,
                                         index.h, C.byref(r))
    assert rc == 0
    return r


def replay_fast(buf: np.ndarray, file_id: int, index: Index) -> ReplayResult:
    r = ReplayResult()
    load().orc_replay_buffer_fast(_ptr(buf), buf.size, file_id, index.h, C.byref(r))
    return r


def compact_files(src_dir: str, dst_dir: str, index: Index, files, file_id_seq: int, max_file_size: int):
    """Cask::compact_files_aux (cask.rs:451-523) restated in C: reads src_dir, writes the new files into
    dst_dir (ids file_id_seq + 1, ...), `index` unchanged. Returns (CompactResult, [(file_id, live)])."""
    f = np.ascontiguousarray(np.asarray(list(files), np.uint32))
    cap = 1 << 16
    ids = np.zeros(cap, np.uint32)
    live = np.zeros(cap, np.uint8)
    r = CompactResult()
    load().orc_compact_files(src_dir.encode(), dst_dir.encode(), index.h, _ptr(f), f.size, file_id_seq, max_file_size,
                             _ptr(ids), _ptr(live), cap, C.byref(r))
    n = min(int(r.n_out), cap)
    return r, [(int(ids[i]), bool(live[i])) for i in range(n)]


def entry_digest(key: bytes, file_id: int, pos: int, size: int, seq: int) -> int:
    k = np.frombuffer(bytes(key), np.uint8)
    return int(load().orc_entry_digest(_ptr(k), len(key), file_id, pos, size, seq))


def hint_body(buf) -> np.ndarray:
    """RecreateHints over one data file (log.rs:137-148, 449-471): the hint body, no trailer."""
    b = buf if isinstance(buf, np.ndarray) else np.frombuffer(buf, np.uint8)
    out = np.empty(b.size + 4 * (b.size // 18) + 64, np.uint8)  # a hint is 4 B longer than its >= 18-B record
    n = load().orc_hint_body(_ptr(b), b.size, _ptr(out), out.size)
    assert n >= 0
    return out[:n]


class PIndex:
    """The threaded replay's keydir kept for lookups (orc_pindex_build): liveness for compaction."""

    def __init__(self, bufs, file_ids, nthreads: int = 8):
        self.L = load()
        arrs = [b if isinstance(b, np.ndarray) else np.frombuffer(b, np.uint8) for b in bufs]
        n = len(arrs)
        ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data if a.size else None for a in arrs])
        lens = np.asarray([a.size for a in arrs] or [0], np.uint64)
        fids = np.asarray(list(file_ids) or [0], np.uint32)
        cap = 1 << 16
        sf = np.zeros(cap, np.uint32)
        se, sd, sb = (np.zeros(cap, np.uint64) for _ in range(3))
        self.result = ParallelResult()
        self.h = self.L.orc_pindex_build(ptrs, _ptr(lens), _ptr(fids), n, nthreads, C.byref(self.result), _ptr(sf),
                                         _ptr(se), _ptr(sd), _ptr(sb), cap)
        k = min(int(self.result.stats_rows), cap)
        self.stats = sorted([int(sf[i]), int(se[i]), int(sd[i]), int(sb[i])] for i in range(k))

    def close(self):
        if self.h:
            self.L.orc_pindex_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def compact_files(self, src_dir: str, dst_dir: str, files, file_id_seq: int, max_file_size: int):
        """orc_compact_files with this keydir's liveness; see compact_files."""
        f = np.ascontiguousarray(np.asarray(list(files), np.uint32))
        cap = 1 << 16
        ids = np.zeros(cap, np.uint32)
        live = np.zeros(cap, np.uint8)
        r = CompactResult()
        fn = C.cast(self.L.orc_pindex_seq, C.c_void_p)
        self.L.orc_compact_files_fn(src_dir.encode(), dst_dir.encode(), fn, self.h, _ptr(f), f.size, file_id_seq,
                                    max_file_size, _ptr(ids), _ptr(live), cap, C.byref(r))
        n = min(int(r.n_out), cap)
        return r, [(int(ids[i]), bool(live[i])) for i in range(n)]


def replay_parallel(bufs, file_ids, nthreads: int = 8):
    """Cask::open over in-memory data files (replay order) on host threads. Returns
    (ParallelResult, stats rows sorted by file id [[fid, entries, dead_entries, dead_bytes]])."""
    arrs = [b if isinstance(b, np.ndarray) else np.frombuffer(b, np.uint8) for b in bufs]
    n = len(arrs)
    ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data if a.size else None for a in arrs])
    lens = np.asarray([a.size for a in arrs] or [0], np.uint64)
    fids = np.asarray(list(file_ids) or [0], np.uint32)
    cap = 1 << 16
    sf = np.zeros(cap, np.uint32)
    se, sd, sb = (np.zeros(cap, np.uint64) for _ in range(3))
    r = ParallelResult()
    load().orc_replay_parallel(ptrs, _ptr(lens), _ptr(fids), n, nthreads, C.byref(r), _ptr(sf), _ptr(se), _ptr(sd),
                               _ptr(sb), cap)
    k = min(int(r.stats_rows), cap)
    rows = sorted([int(sf[i]), int(se[i]), int(sd[i]), int(sb[i])] for i in range(k))
    return r, rows


def keydir_digest_np(keys: np.ndarray, key_len: np.ndarray, file_id, pos, size, seq) -> int:
    """orc_entry_digest summed over keydir rows, vectorised (numpy, wrapping uint64) — the same
    function as the C oracle's, for a product export of fixed-size keys (keys: n x ksz uint8)."""
    with np.errstate(over="ignore"):
        def mix(x):
            x = x ^ (x >> np.uint64(30))
            x = x * np.uint64(0xBF58476D1CE4E5B9)
            x = x ^ (x >> np.uint64(27))
            x = x * np.uint64(0x94D049BB133111EB)
            return x ^ (x >> np.uint64(31))
        n, ksz = keys.shape
        assert (key_len == ksz).all()
        h = mix(np.full(n, 0x9E3779B97F4A7C15 ^ ksz, np.uint64))
        pad = (-ksz) % 8
        kp = np.concatenate([keys, np.zeros((n, pad), np.uint8)], axis=1) if pad else keys
        words = np.ascontiguousarray(kp).view("<u8")
        for w in range(words.shape[1]):
            h = mix(h ^ words[:, w])
        for v in (file_id, pos, size, seq):
            h = mix(h ^ np.asarray(v).astype(np.uint64))
        return int(h.sum(dtype=np.uint64))

"""Host-side mirror of the reference's public API for the replay path.

`CaskOptions` keeps the builder of cask.rs:194-331 (same names, same defaults); `open()` runs the
Cask::open replay (cask.rs:335-382) in the native engine, with every data file that lacks a valid
hint file scanned on the GPU. Only the keydir/stats/sequence the replay builds are exposed here;
`compact()` / `compact_files()` run the compaction merge (cask.rs:451-642) with the live records
verified and copied on the GPU. get/put/delete and the background sync/compaction threads are
outside this path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from . import _lib as L
from .errors import raise_status


class SyncStrategy:
    """cask.rs:209-218 (accepted for API compatibility; syncing is outside the replay path)."""
    Never = "never"
    Always = "always"

    @staticmethod
    def Interval(millis: int):
        return ("interval", int(millis))


@dataclass(frozen=True)
class IndexEntry:
    """cask.rs:20-26."""
    file_id: int
    entry_pos: int
    entry_size: int
    sequence: int


class CaskOptions:
    """cask.rs:194-331. Defaults from cask.rs:220-237."""

    def __init__(self):
        self._create = True
        self._sync = SyncStrategy.Interval(1000)
        self._max_file_size = 2 * 1024 * 1024 * 1024
        self._file_pool_size = 2048
        self._compaction = True
        self._compaction_check_frequency = 3600
        self._compaction_window = (0, 23)
        self._fragmentation_trigger = 0.6
        self._dead_bytes_trigger = 512 * 1024 * 1024
        self._fragmentation_threshold = 0.4
        self._dead_bytes_threshold = 128 * 1024 * 1024
        self._small_file_threshold = 10 * 1024 * 1024
        self._device = 0
        self._write_hints = True

    @classmethod
    def default(cls) -> "CaskOptions":
        return cls()

    def sync(self, s):
        self._sync = s
        return self

    def max_file_size(self, n: int):
        self._max_file_size = int(n)
        return self

    def file_pool_size(self, n: int):
        self._file_pool_size = int(n)
        return self

    def compaction(self, b: bool):
        self._compaction = bool(b)
        return self

    def create(self, b: bool):
        self._create = bool(b)
        return self

    def compaction_check_frequency(self, s: int):
        self._compaction_check_frequency = int(s)
        return self

    def compaction_window(self, start: int, end: int):
        self._compaction_window = (int(start), int(end))
        return self

    def fragmentation_trigger(self, f: float):
        self._fragmentation_trigger = float(f)
        return self

    def dead_bytes_trigger(self, n: int):
        self._dead_bytes_trigger = int(n)
        return self

    def fragmentation_threshold(self, f: float):
        self._fragmentation_threshold = float(f)
        return self

    def dead_bytes_threshold(self, n: int):
        self._dead_bytes_threshold = int(n)
        return self

    def small_file_threshold(self, n: int):
        self._small_file_threshold = int(n)
        return self

    # extensions of this build
    def device(self, ordinal: int):
        """GPU used for the data-file scan."""
        self._device = int(ordinal)
        return self

    def write_hints(self, b: bool):
        self._write_hints = bool(b)
        return self

    def open(self, path: str) -> "Cask":
        """cask.rs:328-330."""
        return Cask.open(path, self)


class Cask:
    """Handle to a replayed database (cask.rs:171-177)."""

    def __init__(self, handle, path: str, options: "CaskOptions | None" = None):
        self._h = handle
        self.path = path
        self.options = options or CaskOptions()

    @staticmethod
    def open(path: str, options: CaskOptions | None = None) -> "Cask":
        """Cask::open (cask.rs:335-382)."""
        o = options or CaskOptions()
        lib = L.lib()
        opts = L.Options()
        lib.cask_options_default(C.byref(opts))
        opts.create = 1 if o._create else 0
        opts.write_hints = 1 if o._write_hints else 0
        opts.max_file_size = o._max_file_size
        opts.device = o._device
        err = L.OpenError()
        h = lib.cask_db_open(path.encode(), C.byref(opts), C.byref(err))
        if not h:
            raise_status(err.status, err.file_id, err.pos, err.expected, err.found, what=path)
        return Cask(h, path, o)

    def _handle(self):
        if not self._h:
            raise ValueError("Cask is closed")
        return self._h

    def close(self):
        if self._h:
            L.lib().cask_db_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self) -> int:
        return int(L.lib().cask_db_len(self._handle()))

    @property
    def current_sequence(self) -> int:
        """cask.rs:379."""
        return int(L.lib().cask_db_current_sequence(self._handle()))

    def files(self) -> list[int]:
        """Log::files (log.rs:104-106)."""
        lib = L.lib()
        n = lib.cask_db_files(self._handle(), None, 0)
        arr = (C.c_uint32 * max(n, 1))()
        lib.cask_db_files(self._handle(), arr, n)
        return list(arr[:n])

    def get_entry(self, key: bytes) -> IndexEntry | None:
        """Index::get (cask.rs:41-43)."""
        e = L.IndexEntry()
        kb = bytes(key)
        ok = L.lib().cask_db_get_entry(self._handle(), kb, len(kb), C.byref(e))
        if ok != 1:  # (1: found; 0: not found)
            return None
        return IndexEntry(e.file_id, e.entry_pos, e.entry_size, e.sequence)

    def index(self) -> dict[bytes, IndexEntry]:
        """The whole keydir, keys in bytewise order."""
        lib = L.lib()
        n = len(self)
        total = lib.cask_db_export(self._handle(), None, 0, None, None, None, n)
        if total < 0:
            raise_status(int(total))
        kb = (C.c_uint8 * max(total, 1))()
        off = (C.c_uint64 * max(n, 1))()
        kl = (C.c_uint64 * max(n, 1))()
        ents = (L.IndexEntry * max(n, 1))()
        r = lib.cask_db_export(self._handle(), kb, total, off, kl, ents, n)
        if r < 0:
            raise_status(int(r))
        raw = bytes(kb)
        out = {}
        for i in range(n):
            e = ents[i]
            out[raw[off[i]:off[i] + kl[i]]] = IndexEntry(e.file_id, e.entry_pos, e.entry_size, e.sequence)
        return out

    def export_arrays(self):
        """The whole keydir as numpy arrays, keys in bytewise order (for keydirs too large for a
        dict): (key_bytes uint8, key_off u64, key_len u64, entries) with entries a structured array
        of file_id, entry_pos, entry_size, sequence."""
        import numpy as np
        lib = L.lib()
        n = len(self)
        total = lib.cask_db_export(self._handle(), None, 0, None, None, None, n)
        if total < 0:
            raise_status(int(total))
        kb = np.zeros(max(total, 1), np.uint8)
        off = np.zeros(max(n, 1), np.uint64)
        kl = np.zeros(max(n, 1), np.uint64)
        ents = np.zeros(max(n, 1), np.dtype([("file_id", "<u4"), ("pad", "<u4"), ("entry_pos", "<u8"),
                                             ("entry_size", "<u8"), ("sequence", "<u8")]))
        u64p = C.POINTER(C.c_uint64)
        r = lib.cask_db_export(self._handle(), kb.ctypes.data, total, off.ctypes.data_as(u64p), kl.ctypes.data_as(u64p),
                               ents.ctypes.data_as(C.POINTER(L.IndexEntry)), n)
        if r < 0:
            raise_status(int(r))
        return kb[:total], off[:n], kl[:n], ents[:n]

    def keys(self) -> list[bytes]:
        """Cask::keys (cask.rs:668-671), sorted."""
        return list(self.index().keys())

    def stats(self) -> dict[int, tuple[int, int, int]]:
        """Stats (stats.rs:6-67): file_id -> (entries, dead_entries, dead_bytes)."""
        lib = L.lib()
        n = lib.cask_db_stats(self._handle(), None, None, None, None, 0)
        fid = (C.c_uint32 * max(n, 1))()
        en = (C.c_uint64 * max(n, 1))()
        de = (C.c_uint64 * max(n, 1))()
        db = (C.c_uint64 * max(n, 1))()
        lib.cask_db_stats(self._handle(), fid, en, de, db, n)
        return {int(fid[i]): (int(en[i]), int(de[i]), int(db[i])) for i in range(n)}

    def file_stats(self) -> list[tuple[int, float, int]]:
        """Stats::file_stats (stats.rs:56-67): (file_id, dead/entries, dead_bytes)."""
        return [(f, (d / e) if e else float("nan"), b) for f, (e, d, b) in sorted(self.stats().items())]

    def _compact_opts(self) -> "L.CompactOptions":
        o = self.options
        c = L.CompactOptions()
        c.fragmentation_trigger = o._fragmentation_trigger
        c.dead_bytes_trigger = o._dead_bytes_trigger
        c.fragmentation_threshold = o._fragmentation_threshold
        c.dead_bytes_threshold = o._dead_bytes_threshold
        c.small_file_threshold = o._small_file_threshold
        return c

    @staticmethod
    def _compact_report(r: "L.CompactResult") -> dict:
        return {"compacted": int(r.n_compacted), "new_files": int(r.n_new), "tombstone_only_files": int(r.n_tomb_only),
                "live_records": int(r.live_records), "tombstones": int(r.tombstones), "bytes_in": int(r.bytes_in),
                "bytes_out": int(r.bytes_out), "hints_ms": r.ms[0], "verify_ms": r.ms[1], "gather_ms": r.ms[2],
                "write_ms": r.ms[3], "swap_ms": r.ms[4], "total_ms": r.ms_total}

    def compact_files(self, files) -> dict:
        """Cask::compact_files (cask.rs:525-560): compact the given data files (ascending, once
        each) into new ones. Returns a report of what was done; raises like the reference."""
        ids = sorted(set(int(f) for f in files))
        arr = (C.c_uint32 * max(len(ids), 1))(*ids)
        res, err = L.CompactResult(), L.OpenError()
        st = L.lib().cask_db_compact_files(self._handle(), arr, len(ids), C.byref(res), C.byref(err))
        if st != L.OK:
            raise_status(st, err.file_id, err.pos, err.expected, err.found, what=self.path)
        return self._compact_report(res)

    def compact(self) -> dict | None:
        """Cask::compact (cask.rs:563-642) with this Cask's CaskOptions thresholds. Returns the
        report, or None when no trigger fired."""
        opts = self._compact_opts()
        res, err = L.CompactResult(), L.OpenError()
        n = L.lib().cask_db_compact(self._handle(), C.byref(opts), C.byref(res), C.byref(err))
        if n < 0:
            raise_status(int(n), err.file_id, err.pos, err.expected, err.found, what=self.path)
        return self._compact_report(res) if n > 0 else None

    def open_timings(self) -> dict[str, float]:
        t = (C.c_double * 5)()
        L.lib().cask_db_open_timings(self._handle(), t)
        return {"discover_read_ms": t[0], "device_scan_ms": t[1], "hint_write_ms": t[2], "fold_ms": t[3],
                "total_ms": t[4]}

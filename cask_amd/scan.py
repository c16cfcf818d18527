"""Python face of the device scan (include/cask_scan.h).

`ScanContext.scan_device` takes data files already resident in HBM (torch uint8 CUDA tensors)
and returns rows as CUDA tensors — the replacement for `Entries`/`Entry::from_read`
(log.rs:403-429, data.rs:161-206). `scan_host` does the same for host buffers (numpy), staging
through the device. torch is used only to hold device memory; all work is in libcask_scan.so.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .errors import CapacityError, raise_status


@dataclass
class ScanFailure:
    """First failing record (cask_scan_error)."""
    kind: int
    file_id: int
    pos: int
    expected: int
    found: int
    row: int


@dataclass
class ScanResult:
    count: int
    pos: object      # torch.Tensor (device scan) or np.ndarray (host scan), length >= count
    seq: object
    vsz: object
    ksz: object
    status: object
    file_row_offset: list
    error: ScanFailure | None

    def file_rows(self, i: int) -> slice:
        return slice(self.file_row_offset[i], self.file_row_offset[i + 1])


def _err(e: L.ScanError) -> ScanFailure | None:
    if e.kind == 0:
        return None
    return ScanFailure(int(e.kind), int(e.file_id), int(e.pos), int(e.expected), int(e.found), int(e.row))


class ScanContext:
    """One per GPU (cask_ctx)."""

    def __init__(self, device: int = 0):
        self.lib = L.lib()
        st = C.c_int(0)
        self._h = self.lib.cask_ctx_create(int(device), C.byref(st))
        if not self._h:
            raise_status(st.value, what=f"cask_ctx_create(device={device})")
        self.device = device

    def close(self):
        if self._h:
            self.lib.cask_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _inputs_ready(self):
        """The context runs on its own non-blocking HIP stream, which does not wait for torch's
        stream by itself: tensors torch is still producing must be complete before the library
        reads them. The context's stream waits for torch's on the device (an event), the host does
        not block."""
        import torch
        s = torch.cuda.current_stream(self.device).cuda_stream
        raise_status(self.lib.cask_ctx_wait_stream(self._h, C.c_void_p(s or None)), what="cask_ctx_wait_stream")

    def set_stream(self, stream_ptr: int | None):
        self.lib.cask_ctx_set_stream(self._h, C.c_void_p(stream_ptr or 0))

    @property
    def stream_ptr(self) -> int:
        return int(self.lib.cask_ctx_stream(self._h) or 0)

    @staticmethod
    def chunk_bytes() -> int:
        return int(L.lib().cask_scan_chunk_bytes())

    # -- device-resident ----------------------------------------------------------------------
    @staticmethod
    def rows_bound(lengths) -> int:
        return int(sum(int(n) // 18 + 1 for n in lengths))

    def alloc_rows(self, capacity: int):
        import torch
        dev = torch.device("cuda", self.device)
        cap = max(int(capacity), 1)
        return {
            "pos": torch.empty(cap, dtype=torch.int64, device=dev),
            "seq": torch.empty(cap, dtype=torch.int64, device=dev),
            "vsz": torch.empty(cap, dtype=torch.int32, device=dev),
            "ksz": torch.empty(cap, dtype=torch.int16, device=dev),
            "status": torch.empty(cap, dtype=torch.uint8, device=dev),
        }

    def scan_device(self, files, rows: dict | None = None, raise_on_capacity: bool = True) -> ScanResult:
        """files: list of (file_id, uint8 CUDA tensor). rows: dict from alloc_rows (reused if given)."""
        return self._scan_device(self.lib.cask_scan_device, "cask_scan_device", files, rows, raise_on_capacity)

    def prepare_scan(self, files, rows: dict):
        """A repeatable cask_scan_device call on the same device-resident files and rows, its ctypes
        arguments built once (what a compiled caller of the C ABI pays per call: the call itself).
        Returns (run, timings): run() issues the scan and returns the row count (raising on any
        error); timings(out) copies the call's eight phase times (ms, last_timings' order) into a
        float array of 8."""
        n = len(files)
        views = (L.FileView * max(n, 1))()
        for i, (fid, t) in enumerate(files):
            assert t.is_cuda and t.dtype.itemsize == 1 and t.is_contiguous()
            views[i].file_id = int(fid)
            views[i].flags = L.VIEW_DEVICE
            views[i].data = t.data_ptr() if t.numel() else None
            views[i].len = t.numel()
        r = L.Rows()
        r.capacity = rows["pos"].numel()
        r.pos, r.seq = rows["pos"].data_ptr(), rows["seq"].data_ptr()
        r.vsz, r.ksz, r.status = rows["vsz"].data_ptr(), rows["ksz"].data_ptr(), rows["status"].data_ptr()
        off = (C.c_uint64 * (n + 1))()
        e = L.ScanError()
        self._inputs_ready()
        fn, h, rr, ee, lib = self.lib.cask_scan_device, self._h, C.byref(r), C.byref(e), self.lib

        def run():
            rc = fn(h, views, n, rr, off, ee)
            if rc or e.kind:
                raise_status(rc, what=f"cask_scan_device: {self.last_error()}")
                raise RuntimeError(f"scan failure {_err(e)}")
            return r.count

        def timings(out):
            lib.cask_last_timings8(h, out)

        return run, timings

    def parse_hints_device(self, bodies, rows: dict | None = None, raise_on_capacity: bool = True) -> ScanResult:
        """Hint-file bodies (trailer excluded) on the device, parsed there (cask_parse_hints_device:
        Hints::next / Hint::from_read, log.rs:437-447, data.rs:258-276). Row pos = the hint's offset in
        its body; seq, ksz, vsz as in the hint; status Ok or EOF (a body cut short)."""
        return self._scan_device(self.lib.cask_parse_hints_device, "cask_parse_hints_device", bodies, rows,
                                 raise_on_capacity)

    def _scan_device(self, fn, name, files, rows, raise_on_capacity):
        n = len(files)
        views = (L.FileView * max(n, 1))()
        for i, (fid, t) in enumerate(files):
            assert t.is_cuda and t.dtype.itemsize == 1 and t.is_contiguous()
            views[i].file_id = int(fid)
            views[i].flags = L.VIEW_DEVICE
            views[i].data = t.data_ptr() if t.numel() else None
            views[i].len = t.numel()
        if rows is None:
            rows = self.alloc_rows(self.rows_bound([t.numel() for _, t in files]))
        r = L.Rows()
        r.capacity = rows["pos"].numel()
        r.pos, r.seq = rows["pos"].data_ptr(), rows["seq"].data_ptr()
        r.vsz, r.ksz, r.status = rows["vsz"].data_ptr(), rows["ksz"].data_ptr(), rows["status"].data_ptr()
        off = (C.c_uint64 * (n + 1))()
        e = L.ScanError()
        self._inputs_ready()
        rc = fn(self._h, views, n, C.byref(r), off, C.byref(e))
        if rc == L.E_CAPACITY:
            if raise_on_capacity:
                raise CapacityError(int(r.count))
        else:
            raise_status(rc, what=f"{name}: {self.last_error()}")
        return ScanResult(int(r.count), rows["pos"], rows["seq"], rows["vsz"], rows["ksz"], rows["status"],
                          list(off), _err(e))

    # -- host-resident ------------------------------------------------------------------------
    def scan_host(self, files) -> ScanResult:
        """files: list of (file_id, bytes | np.ndarray[uint8]). Rows come back as numpy arrays."""
        n = len(files)
        bufs = [np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray, memoryview))
                else np.ascontiguousarray(b, dtype=np.uint8) for _, b in files]
        views = (L.FileView * max(n, 1))()
        for i, (fid, _) in enumerate(files):
            views[i].file_id = int(fid)
            views[i].flags = 0
            views[i].data = bufs[i].ctypes.data if bufs[i].size else None
            views[i].len = bufs[i].size
        cap = max(self.rows_bound([b.size for b in bufs]), 1)
        pos = np.empty(cap, np.uint64)
        seq = np.empty(cap, np.uint64)
        vsz = np.empty(cap, np.uint32)
        ksz = np.empty(cap, np.uint16)
        status = np.empty(cap, np.uint8)
        r = L.Rows()
        r.capacity = cap
        r.pos, r.seq, r.vsz = pos.ctypes.data, seq.ctypes.data, vsz.ctypes.data
        r.ksz, r.status = ksz.ctypes.data, status.ctypes.data
        off = (C.c_uint64 * (n + 1))()
        e = L.ScanError()
        rc = self.lib.cask_scan_host(self._h, views, n, C.byref(r), off, C.byref(e))
        raise_status(rc, what=f"cask_scan_host: {self.last_error()}")
        c = int(r.count)
        return ScanResult(c, pos[:c], seq[:c], vsz[:c], ksz[:c], status[:c], list(off), _err(e))

    # -- instrumentation ----------------------------------------------------------------------
    def scratch_bytes(self) -> int:
        """Device scratch this context holds (cask_ctx_scratch_bytes)."""
        return int(self.lib.cask_ctx_scratch_bytes(self._h))

    def last_error(self) -> str:
        v = self.lib.cask_ctx_last_error(self._h)
        return v.decode() if v else ""

    def last_timings(self) -> dict[str, float]:
        t = (C.c_float * 8)()
        self.lib.cask_last_timings8(self._h, t)
        # validate_ms: k_finish on the dense path (validation + dense rows; compact_ms is then 0),
        # the three validation launches on the repair path; chunk_scan_ms is the first pass's kernel
        # (k_scan_chunks, or k_walk_hash in walk mode, whose run searches are search_ms)
        return {"pipeline_ms": t[0], "chunk_scan_ms": t[1], "long_ms": t[2], "validate_ms": t[3],
                "repair_ms": t[4], "compact_ms": t[5], "search_ms": t[6], "chase_ms": t[7]}

    def last_counters(self) -> dict[str, int]:
        c = (C.c_uint64 * 5)()
        self.lib.cask_last_counters(self._h, c)
        return {"chunks": int(c[0]), "long_records": int(c[1]), "repaired_chunks": int(c[2]),
                "local_repair_passes": int(c[3]), "walked": int(c[4]),
                "dense_path": int(self.lib.cask_last_dense(self._h)),
                "walk_mode": int(self.lib.cask_last_walk(self._h)),
                "geometry": int(self.lib.cask_last_geometry(self._h))}

    # -- encoder ------------------------------------------------------------------------------
    def encode_synthetic(self, off, seq, ksz, vsz_raw, key_id, value_seed: int, out):
        """Batched Entry::write_bytes (data.rs:90-121) of generated keys/values (DESIGN.md
        §Synthetic data). All tensors on this device; out is a uint8 tensor."""
        n = off.numel()
        self._inputs_ready()
        rc = self.lib.cask_encode_synthetic_device(self._h, n, off.data_ptr(), seq.data_ptr(), ksz.data_ptr(),
                                                   vsz_raw.data_ptr(), key_id.data_ptr(),
                                                   int(value_seed) & 0xFFFFFFFFFFFFFFFF, out.data_ptr())
        raise_status(rc, what="cask_encode_synthetic_device")

    def encode(self, off, seq, ksz, vsz_raw, keys, key_off, vals, val_off, out):
        """Batched Entry::write_bytes of caller keys/values (device tensors)."""
        n = off.numel()
        self._inputs_ready()
        rc = self.lib.cask_encode_device(self._h, n, off.data_ptr(), seq.data_ptr(), ksz.data_ptr(),
                                         vsz_raw.data_ptr(), keys.data_ptr(), key_off.data_ptr(),
                                         vals.data_ptr(), val_off.data_ptr(), out.data_ptr())
        raise_status(rc, what="cask_encode_device")


def xxh32(data: bytes) -> int:
    """util.rs:37-41 via the native library."""
    b = bytes(data)
    return int(L.lib().cask_xxh32(b, len(b)))

"""ctypes binding of include/cask_scan.h (libcask_scan.so, built in-tree by __graft_entry__.build()).

There is no fallback: if the native library is missing, every entry point raises
NativeLibraryMissing. This is the only module that loads the shared object.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# The in-tree product build. No environment variable selects another library: diagnostic builds
# (make -C cask_amd stamps) are loaded only by tools that call use_library() explicitly, and
# bench.py refuses to time anything but this file.
LIB_PATH = os.path.join(_HERE, "libcask_scan.so")
_path = LIB_PATH

c_u8p = C.POINTER(C.c_uint8)
c_u16p = C.POINTER(C.c_uint16)
c_u32p = C.POINTER(C.c_uint32)
c_u64p = C.POINTER(C.c_uint64)


class NativeLibraryMissing(ImportError):
    pass


class FileView(C.Structure):
    _fields_ = [("file_id", C.c_uint32), ("flags", C.c_uint32), ("data", C.c_void_p), ("len", C.c_uint64)]


class Rows(C.Structure):
    _fields_ = [("capacity", C.c_uint64), ("count", C.c_uint64), ("pos", C.c_void_p), ("seq", C.c_void_p),
                ("vsz", C.c_void_p), ("ksz", C.c_void_p), ("status", C.c_void_p)]


class ScanError(C.Structure):
    _fields_ = [("kind", C.c_int32), ("file_id", C.c_uint32), ("pos", C.c_uint64), ("expected", C.c_uint32),
                ("found", C.c_uint32), ("row", C.c_uint64)]


class Options(C.Structure):
    _fields_ = [("create", C.c_int32), ("write_hints", C.c_int32), ("max_file_size", C.c_uint64),
                ("device", C.c_int32), ("reserved", C.c_int32)]


class OpenError(C.Structure):
    _fields_ = [("status", C.c_int32), ("file_id", C.c_uint32), ("pos", C.c_uint64), ("expected", C.c_uint32),
                ("found", C.c_uint32)]


class CompactOptions(C.Structure):
    _fields_ = [("fragmentation_trigger", C.c_double), ("dead_bytes_trigger", C.c_uint64),
                ("fragmentation_threshold", C.c_double), ("dead_bytes_threshold", C.c_uint64),
                ("small_file_threshold", C.c_uint64)]


class CompactResult(C.Structure):
    _fields_ = [("n_compacted", C.c_uint32), ("n_new", C.c_uint32), ("n_tomb_only", C.c_uint32),
                ("pad", C.c_uint32), ("live_records", C.c_uint64), ("tombstones", C.c_uint64),
                ("bytes_in", C.c_uint64), ("bytes_out", C.c_uint64), ("ms", C.c_double * 5),
                ("ms_total", C.c_double)]


class IndexEntry(C.Structure):
    _fields_ = [("file_id", C.c_uint32), ("pad", C.c_uint32), ("entry_pos", C.c_uint64),
                ("entry_size", C.c_uint64), ("sequence", C.c_uint64)]


VIEW_DEVICE = 1
ROW_OK, ROW_CHECKSUM, ROW_EOF = 0, 1, 2

# cask_status
OK = 0
E_CHECKSUM = -1
E_EOF = -2
E_IO = -3
E_INVALID_PATH = -4
E_INVALID_FILE_ID = -5
E_INVALID_ARG = -10
E_DEVICE = -11
E_CAPACITY = -12
E_NOMEM = -13
E_LOCKED = -14

# (name, restype, argtypes) for every symbol declared in include/cask_scan.h
SIGNATURES = [
    ("cask_ctx_create", C.c_void_p, [C.c_int, C.POINTER(C.c_int)]),
    ("cask_ctx_destroy", None, [C.c_void_p]),
    ("cask_ctx_set_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("cask_ctx_stream", C.c_void_p, [C.c_void_p]),
    ("cask_ctx_wait_stream", C.c_int, [C.c_void_p, C.c_void_p]),
    ("cask_ctx_device", C.c_int, [C.c_void_p]),
    ("cask_ctx_last_error", C.c_char_p, [C.c_void_p]),
    ("cask_scan_chunk_bytes", C.c_uint32, []),
    ("cask_rows_bound", C.c_uint64, [C.POINTER(FileView), C.c_uint32]),
    ("cask_parse_hints_device", C.c_int, [C.c_void_p, C.POINTER(FileView), C.c_uint32, C.POINTER(Rows), c_u64p,
                                   C.POINTER(ScanError)]),
    ("cask_scan_device", C.c_int, [C.c_void_p, C.POINTER(FileView), C.c_uint32, C.POINTER(Rows), c_u64p,
                                   C.POINTER(ScanError)]),
    ("cask_scan_host", C.c_int, [C.c_void_p, C.POINTER(FileView), C.c_uint32, C.POINTER(Rows), c_u64p,
                                 C.POINTER(ScanError)]),
    ("cask_last_timings", C.c_int, [C.c_void_p, C.POINTER(C.c_float)]),
    ("cask_last_timings8", C.c_int, [C.c_void_p, C.POINTER(C.c_float)]),
    ("cask_last_counters", C.c_int, [C.c_void_p, c_u64p]),
    ("cask_last_walk", C.c_int, [C.c_void_p]),
    ("cask_last_geometry", C.c_int, [C.c_void_p]),
    ("cask_last_dense", C.c_int, [C.c_void_p]),
    ("cask_encode_synthetic_device", C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p,
                                               C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    ("cask_log_write", C.c_int64, [C.c_char_p, C.c_uint32, C.c_uint64, C.c_int, C.c_int, C.c_uint64, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_uint64]),
    ("cask_encode_device", C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    ("cask_xxh32", C.c_uint32, [C.c_void_p, C.c_uint64]),
    ("cask_read_entries_device", C.c_int, [C.c_void_p, C.c_void_p, c_u64p, C.c_uint32, c_u32p, c_u64p, C.c_uint64,
                                           c_u64p, c_u8p, c_u32p, c_u32p]),
    ("cask_options_default", None, [C.POINTER(Options)]),
    ("cask_db_open", C.c_void_p, [C.c_char_p, C.POINTER(Options), C.POINTER(OpenError)]),
    ("cask_db_close", None, [C.c_void_p]),
    ("cask_db_len", C.c_uint64, [C.c_void_p]),
    ("cask_db_get_entry", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(IndexEntry)]),
    ("cask_db_export", C.c_int64, [C.c_void_p, C.c_void_p, C.c_uint64, c_u64p, c_u64p, C.POINTER(IndexEntry),
                                   C.c_uint64]),
    ("cask_db_stats", C.c_uint64, [C.c_void_p, c_u32p, c_u64p, c_u64p, c_u64p, C.c_uint64]),
    ("cask_db_current_sequence", C.c_uint64, [C.c_void_p]),
    ("cask_db_files", C.c_uint64, [C.c_void_p, c_u32p, C.c_uint64]),
    ("cask_db_open_timings", C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    ("cask_compact_options_default", None, [C.POINTER(CompactOptions)]),
    ("cask_db_compact_files", C.c_int, [C.c_void_p, c_u32p, C.c_uint64, C.POINTER(CompactResult),
                                        C.POINTER(OpenError)]),
    ("cask_db_compact", C.c_int64, [C.c_void_p, C.POINTER(CompactOptions), C.POINTER(CompactResult),
                                    C.POINTER(OpenError)]),
    ("cask_shard_keydir_hints", C.c_int, [C.c_void_p, C.POINTER(FileView), C.c_uint32, C.POINTER(Rows), c_u64p,
                                    C.POINTER(C.c_void_p), c_u64p]),
    ("cask_shard_keydir", C.c_int, [C.c_void_p, C.POINTER(FileView), C.c_uint32, C.POINTER(Rows), c_u64p,
                                    C.POINTER(C.c_void_p), c_u64p]),
    ("cask_copy", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64]),
    ("cask_debug_inject", C.c_int, [C.c_void_p, C.c_uint32]),
    ("cask_ctx_scratch_bytes", C.c_uint64, [C.c_void_p]),
    ("cask_rccl_unique_id", C.c_int, [C.c_void_p]),
    ("cask_rccl_comm_init", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    ("cask_rccl_comm_destroy", C.c_int, [C.c_void_p]),
    ("cask_keydir_gather_rccl", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p,
                                          c_u64p, c_u64p]),
    ("cask_hints_device", C.c_int, [C.c_void_p, C.POINTER(FileView), C.c_uint32, C.POINTER(Rows), c_u64p,
                                    C.c_void_p, C.c_uint64, c_u64p]),
    ("cask_keydir_exchange_rccl", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                            c_u64p, c_u64p]),
    ("cask_keydir_owner", C.c_uint32, [C.c_void_p, C.c_uint64, C.c_uint32]),
    ("cask_keydir_partition", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.POINTER(C.c_void_p),
                                        c_u64p]),
    ("cask_keydir_partition_host", C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_uint64, c_u64p]),
    ("cask_keydir_terms", C.c_int64, [C.c_void_p, C.c_void_p, C.c_uint64]),
    ("cask_keydir_finish_terms", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    ("cask_keydir_new", C.c_void_p, []),
    ("cask_keydir_merge", C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64]),
    ("cask_keydir_merge_many", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_uint32]),
    ("cask_keydir_finish", C.c_int, [C.c_void_p]),
    ("cask_db_open_multi", C.c_void_p, [C.c_char_p, C.POINTER(Options), C.POINTER(C.c_int), C.c_int,
                                        C.POINTER(OpenError)]),
]

_lib = None


def use_library(path: str) -> None:
    """Tools only: load `path` (a diagnostic build) instead of the product library. Must run
    before the first lib() call; symbols the build lacks are left unbound."""
    global _path
    if _lib is not None:
        raise RuntimeError("libcask_scan.so is already loaded")
    _path = os.path.abspath(path)


def loaded_path() -> str:
    """Path of the shared object lib() loaded (or will load)."""
    return _path


def lib():
    """Load libcask_scan.so once and bind every signature. Raises if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(_path):
            raise NativeLibraryMissing(
                f"{_path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        # torch (device-memory plumbing) bundles its own libamdhip64.so.7; whichever copy loads
        # first serves the whole process. Load torch's first so torch and this library share one
        # HIP runtime; loading ours first leaves torch with "No HIP GPUs are available".
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(_path)
        for name, res, args in SIGNATURES:
            if _path != LIB_PATH and not hasattr(L, name):
                continue  # a diagnostic or older build (tools' A/B timing): bind what it has
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib

"""cask_amd — MI355X-native data-file scan for Cask (andresilva/cask v0.7.1).

The replay/compaction hot path of the reference (record decode + XXH32 verify, log.rs/data.rs,
driven from Cask::open in cask.rs) runs as hand-written HIP kernels for gfx950 behind the C ABI in
include/cask_scan.h. This package is the Python face of that library:

* `CaskOptions().open(path)` — the reference's replay entry point (cask.rs:328) on the native engine;
* `ScanContext` — the device scan over HBM-resident data files (torch tensors) or host buffers;
* `cask_amd.errors` — the reference's Error enum (errors.rs).
"""
from . import errors
from ._lib import LIB_PATH, NativeLibraryMissing, lib
from .cask import Cask, CaskOptions, IndexEntry, SyncStrategy
from .scan import ScanContext, ScanFailure, ScanResult, xxh32

ROW_OK, ROW_CHECKSUM, ROW_EOF = 0, 1, 2

__all__ = ["Cask", "CaskOptions", "IndexEntry", "SyncStrategy", "ScanContext", "ScanResult", "ScanFailure",
           "errors", "lib", "LIB_PATH", "NativeLibraryMissing", "xxh32", "ROW_OK", "ROW_CHECKSUM", "ROW_EOF"]

"""Bulk write path: a batch of entries through one LogWriter that is then dropped.

Mirrors LogWriter::write's rollover (log.rs:282-306) with EntryWriter / HintWriter (log.rs:317-395):
the record bytes (Entry::write_bytes, data.rs:90-121) are encoded and XXH32-checksummed on the GPU
(cask_log_write -> cask_encode_device); data files and hint files are written by the native engine.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .errors import raise_status

ENTRY_TOMBSTONE = 0xFFFFFFFF  # data.rs:12
MAX_KEY_SIZE = 0xFFFF  # data.rs:13
MAX_VALUE_SIZE = 0xFFFFFFFE  # data.rs:14


def log_write(path: str, entries, max_file_size: int, first_file_id: int = 1, write_hints: bool = True,
              device: int = 0) -> list[int]:
    """Write `entries` — (sequence, key, value) with value None for a deletion (Entry::deleted,
    data.rs:51-61) — in order into data files first_file_id, first_file_id + 1, ... of `path`.
    Returns the file ids written. Key/value limits are Entry::new's (data.rs:27-49)."""
    entries = list(entries)
    n = len(entries)
    seq = np.empty(n, dtype=np.uint64)
    ksz = np.empty(n, dtype=np.uint16)
    vsz = np.empty(n, dtype=np.uint32)
    key_off = np.empty(n, dtype=np.uint64)
    val_off = np.empty(n, dtype=np.uint64)
    keys, vals = bytearray(), bytearray()
    for i, (s, k, v) in enumerate(entries):
        if len(k) > MAX_KEY_SIZE:
            raise ValueError("InvalidKeySize")
        if v is not None and len(v) > MAX_VALUE_SIZE:
            raise ValueError("InvalidValueSize")
        seq[i] = s
        ksz[i] = len(k)
        key_off[i] = len(keys)
        keys += k
        val_off[i] = len(vals)
        if v is None:
            vsz[i] = ENTRY_TOMBSTONE
        else:
            vsz[i] = len(v)
            vals += v
    kb = np.frombuffer(bytes(keys) or b"\0", dtype=np.uint8)
    vb = np.frombuffer(bytes(vals) or b"\0", dtype=np.uint8)
    ids = np.zeros(max(n, 1), dtype=np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)
    rc = L.lib().cask_log_write(path.encode(), first_file_id, max_file_size, int(bool(write_hints)), device, n,
                                p(seq), p(ksz), p(vsz), p(kb), p(key_off), p(vb), p(val_off), p(ids), ids.size)
    if rc < 0:
        raise_status(int(rc), what="cask_log_write")
    return [int(x) for x in ids[:rc]]

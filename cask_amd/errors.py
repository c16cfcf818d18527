"""Error types mirroring the reference's `cask::errors::Error` (src/errors.rs:12-25)."""
from __future__ import annotations

from . import _lib as L


class Error(Exception):
    """errors.rs:12 — base of everything a Cask operation can return."""


class Io(Error):
    """Error::Io (errors.rs:14)."""


class UnexpectedEof(Io):
    """Error::Io(UnexpectedEof): a record or hint cut short (data.rs:163,172,181; data.rs:259-265)."""

    def __init__(self, file_id: int = 0, pos: int = 0):
        super().__init__(f"IO error: failed to fill whole buffer (file {file_id}, pos {pos})")
        self.file_id, self.pos = file_id, pos


class InvalidChecksum(Error):
    """Error::InvalidChecksum { expected, found } (errors.rs:22, data.rs:193-198)."""

    def __init__(self, expected: int, found: int, file_id: int = 0, pos: int = 0):
        super().__init__(f"Invalid checksum, expected: {expected}, found: {found}")
        self.expected, self.found, self.file_id, self.pos = expected, found, file_id, pos


class InvalidPath(Error):
    """Error::InvalidPath (errors.rs:24)."""


class InvalidFileId(Error):
    """Error::InvalidFileId (errors.rs:16)."""


class Locked(Io):
    """flock on cask.lock failed (log.rs:58-59): the database is open in another process."""


class DeviceError(Error):
    """HIP runtime / device failure in the scan."""


class CapacityError(Error):
    """The caller's row buffers were too small; `needed` rows are required."""

    def __init__(self, needed: int):
        super().__init__(f"row capacity too small: {needed} rows needed")
        self.needed = needed


def raise_status(status: int, file_id: int = 0, pos: int = 0, expected: int = 0, found: int = 0,
                 what: str = ""):
    if status == L.OK:
        return
    if status == L.E_CHECKSUM:
        raise InvalidChecksum(expected, found, file_id, pos)
    if status == L.E_EOF:
        raise UnexpectedEof(file_id, pos)
    if status == L.E_INVALID_PATH:
        raise InvalidPath(what)
    if status == L.E_INVALID_FILE_ID:
        raise InvalidFileId(file_id)
    if status == L.E_LOCKED:
        raise Locked(what)
    if status == L.E_IO:
        e = Io(f"{what or 'io error'} (file {file_id})" if file_id else (what or "io error"))
        e.file_id = file_id  # (the file the failing call named, when it names one)
        raise e
    if status in (L.E_DEVICE, L.E_NOMEM):
        raise DeviceError(f"device failure ({status}) {what}")
    raise Error(f"cask status {status} {what}")

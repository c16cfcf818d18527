"""cask_ref.py — pure-Python restatement of Cask's replay/compaction path. TEST INFRASTRUCTURE ONLY.

Used by tests/ (and tests/golden/make_golden.py) as the checker that generates and re-derives
golden fixtures. It is written independently of oracle/cask_oracle.c so the two cross-check
each other. Never imported by the product (cask_amd/) or by bench.py's timed path.

Reference: andresilva/cask v0.7.1 (Rust, not buildable here: no rustc/cargo). Every function
cites the reference lines it restates. XXH32 comes from python-xxhash (libxxhash 0.8.2), the
reference implementation of the algorithm the absent `twox-hash` crate implements
(Cargo.toml:18; util.rs:8,14,37-41).
"""
from __future__ import annotations

import os
import re
import stat
import struct
from dataclasses import dataclass, field

import xxhash

ENTRY_STATIC_SIZE = 18          # data.rs:11
ENTRY_TOMBSTONE = 0xFFFFFFFF    # data.rs:12
MAX_VALUE_SIZE = 0xFFFFFFFE     # data.rs:13
MAX_KEY_SIZE = 0xFFFF           # data.rs:14
DATA_FILE_EXTENSION = "cask.data"  # log.rs:20
HINT_FILE_EXTENSION = "cask.hint"  # log.rs:21

ROW_OK, ROW_CHECKSUM, ROW_EOF = 0, 1, 2


def xxhash32(buf: bytes) -> int:
    """util.rs:37-41 — XXH32 seed 0."""
    return xxhash.xxh32_intdigest(buf, seed=0)


class XxHash32:
    """util.rs:10-23 — streaming hasher, seed 0."""

    def __init__(self):
        self._h = xxhash.xxh32(seed=0)

    def update(self, b: bytes):
        self._h.update(b)

    def get(self) -> int:
        return self._h.intdigest()


# ----------------------------------------------------------------------------- record codec
@dataclass
class Entry:
    """data.rs:18-24."""
    key: bytes
    value: bytes
    sequence: int
    deleted: bool = False

    def size(self) -> int:  # data.rs:63-65
        return ENTRY_STATIC_SIZE + len(self.key) + len(self.value)

    def to_bytes(self) -> bytes:
        """data.rs:68-88 (one-shot checksum over bytes[4..])."""
        tail = struct.pack("<QH", self.sequence, len(self.key))
        if self.deleted:
            tail += struct.pack("<I", ENTRY_TOMBSTONE) + self.key
        else:
            tail += struct.pack("<I", len(self.value)) + self.key + self.value
        return struct.pack("<I", xxhash32(tail)) + tail

    def write_bytes(self) -> bytes:
        """data.rs:90-121 (streaming checksum: header tail, key, value)."""
        hdr = struct.pack("<QHI", self.sequence, len(self.key),
                          ENTRY_TOMBSTONE if self.deleted else len(self.value))
        h = XxHash32()
        h.update(hdr)
        h.update(self.key)
        h.update(self.value)
        out = struct.pack("<I", h.get()) + hdr + self.key
        if not self.deleted:
            out += self.value
        return out


def entry_new(sequence: int, key: bytes, value: bytes) -> Entry:
    """data.rs:27-49 (size limits)."""
    if len(key) > MAX_KEY_SIZE:
        raise ValueError("InvalidKeySize")
    if len(value) > MAX_VALUE_SIZE:
        raise ValueError("InvalidValueSize")
    return Entry(bytes(key), bytes(value), sequence, False)


def entry_deleted(sequence: int, key: bytes) -> Entry:
    """data.rs:51-61."""
    return Entry(bytes(key), b"", sequence, True)


@dataclass
class Row:
    """One Entries::next item (log.rs:403-429) in the scan's row form."""
    pos: int
    seq: int = 0
    ksz: int = 0
    vsz_raw: int = 0
    status: int = ROW_OK
    expected: int = 0
    found: int = 0
    key: bytes = b""

    @property
    def deleted(self) -> bool:
        return self.vsz_raw == ENTRY_TOMBSTONE

    @property
    def value_size(self) -> int:  # Hint::from -> e.value.len() (data.rs:228-236)
        return 0 if self.deleted else self.vsz_raw

    @property
    def entry_size(self) -> int:  # data.rs:238-240
        return ENTRY_STATIC_SIZE + self.ksz + self.value_size


def scan_entries(buf: bytes) -> list[Row]:
    """Entries over Take<File> (log.rs:108-119, 397-430) + Entry::from_read (data.rs:161-206).

    read_exact(header) -> read_exact(key) -> read_exact(value) unless tombstone; a short read is
    Io(UnexpectedEof) and drains the Take limit (iteration ends). Otherwise XXH32 over
    header[4..18] ‖ key ‖ value decides Ok / InvalidChecksum{expected, found}. The position
    advances by bytes consumed, so a checksum failure does not stop the iterator.
    """
    rows: list[Row] = []
    pos = 0
    n = len(buf)
    while pos < n:  # limit == 0 -> None
        rem = n - pos
        if rem < ENTRY_STATIC_SIZE:
            rows.append(Row(pos=pos, status=ROW_EOF))
            break
        stored, seq, ksz, vsz = struct.unpack_from("<IQHI", buf, pos)
        vsz_eff = 0 if vsz == ENTRY_TOMBSTONE else vsz
        if rem < ENTRY_STATIC_SIZE + ksz or rem < ENTRY_STATIC_SIZE + ksz + vsz_eff:
            rows.append(Row(pos=pos, seq=seq, ksz=ksz, vsz_raw=vsz, status=ROW_EOF, expected=stored))
            break
        end = pos + ENTRY_STATIC_SIZE + ksz + vsz_eff
        found = xxhash32(buf[pos + 4:end])
        key = bytes(buf[pos + ENTRY_STATIC_SIZE:pos + ENTRY_STATIC_SIZE + ksz])
        rows.append(Row(pos=pos, seq=seq, ksz=ksz, vsz_raw=vsz,
                        status=ROW_OK if found == stored else ROW_CHECKSUM,
                        expected=stored, found=found, key=key))
        pos = end
    return rows


def hint_bytes(seq: int, key: bytes, value_size: int, deleted: bool, entry_pos: int) -> bytes:
    """Hint::write_bytes (data.rs:242-256)."""
    return struct.pack("<QHIQ", seq, len(key), ENTRY_TOMBSTONE if deleted else value_size,
                       entry_pos) + key


def hint_file_bytes(rows: list[Row]) -> bytes:
    """What RecreateHints + HintWriter leave on disk (log.rs:367-395, 449-471): every Ok row's
    hint (the drain in RecreateHints::drop keeps writing after an error), then the u32 LE
    XXH32 trailer of all hint bytes."""
    body = b"".join(hint_bytes(r.seq, r.key, r.value_size, r.deleted, r.pos)
                    for r in rows if r.status == ROW_OK)
    return body + struct.pack("<I", xxhash32(body))


def parse_hints(body: bytes):
    """Hints::next / Hint::from_read (log.rs:437-447; data.rs:258-276) over the file minus the
    4-byte trailer. Yields Row-like hints, or raises EOFError on a short read."""
    pos = 0
    n = len(body)
    while pos < n:
        if n - pos < 22:
            raise EOFError("hint")
        seq, ksz, vsz, epos = struct.unpack_from("<QHIQ", body, pos)
        if n - pos - 22 < ksz:
            raise EOFError("hint key")
        key = bytes(body[pos + 22:pos + 22 + ksz])
        pos += 22 + ksz
        yield Row(pos=epos, seq=seq, ksz=ksz, vsz_raw=vsz, key=key)


def hint_offsets(body: bytes):
    """Hints::next over a body (log.rs:437-447; Hint::from_read, data.rs:258-276) in the device
    parser's row form: (offset of the hint in the body, seq, ksz, value_size raw, status) per record,
    the last one ROW_EOF if the body cuts it short (then iteration stops, as `hint?` does)."""
    out, pos, n = [], 0, len(body)
    while pos < n:
        if n - pos < 22:
            out.append((pos, 0, 0, 0, ROW_EOF))
            break
        seq, ksz, vsz, _ = struct.unpack_from("<QHIQ", body, pos)
        if n - pos - 22 < ksz:
            out.append((pos, seq, ksz, vsz, ROW_EOF))
            break
        out.append((pos, seq, ksz, vsz, ROW_OK))
        pos += 22 + ksz
    return out


def is_valid_hint_bytes(buf: bytes) -> bool:
    """is_valid_hint_file (log.rs:512-539)."""
    return len(buf) >= 4 and xxhash32(buf[:-4]) == struct.unpack("<I", buf[-4:])[0]


# ----------------------------------------------------------------------------- keydir + stats
@dataclass
class IndexEntry:
    """cask.rs:20-26."""
    file_id: int
    entry_pos: int
    entry_size: int
    sequence: int


class Stats:
    """stats.rs:6-67."""

    def __init__(self):
        self.map: dict[int, list[int]] = {}  # file_id -> [entries, dead_entries, dead_bytes]

    def add_entry(self, e: IndexEntry):  # stats.rs:23-36
        if e.file_id in self.map:
            self.map[e.file_id][0] += 1
        else:
            self.map[e.file_id] = [1, 0, 0]

    def remove_entry(self, e: IndexEntry):  # stats.rs:38-48 (missing row: warn only)
        s = self.map.get(e.file_id)
        if s is not None:
            s[1] += 1
            s[2] += e.entry_size

    def remove_files(self, files):  # stats.rs:50-54
        for f in files:
            self.map.pop(f, None)


class Index:
    """cask.rs:28-95."""

    def __init__(self):
        self.map: dict[bytes, IndexEntry] = {}
        self.stats = Stats()

    def insert(self, key: bytes, ie: IndexEntry):  # cask.rs:45-51
        self.stats.add_entry(ie)
        old = self.map.get(key)
        self.map[key] = ie
        if old is not None:
            self.stats.remove_entry(old)

    def remove(self, key: bytes):  # cask.rs:53-58
        old = self.map.pop(key, None)
        if old is not None:
            self.stats.remove_entry(old)
        return old

    def update(self, hint: Row, file_id: int):  # cask.rs:60-90
        ie = IndexEntry(file_id, hint.pos, hint.entry_size, hint.seq)
        o = self.map.get(hint.key)
        if o is not None:
            if o.sequence <= hint.seq:
                self.stats.remove_entry(o)
                if hint.deleted:
                    del self.map[hint.key]
                else:
                    self.stats.add_entry(ie)
                    self.map[hint.key] = ie
            else:
                self.stats.add_entry(ie)
                self.stats.remove_entry(ie)
        elif not hint.deleted:
            self.stats.add_entry(ie)
            self.map[hint.key] = ie


# ----------------------------------------------------------------------------- replay
_DATA_RE = re.compile(r"(\d+).cask.data$")  # log.rs:486-489 (unescaped '.', unanchored start)


def find_data_files(path: str) -> list[int]:
    """log.rs:483-510."""
    out = []
    for name in os.listdir(path):
        full = os.path.join(path, name)
        # DirEntry::metadata does not traverse symlinks on Unix: only regular files count
        if not stat.S_ISREG(os.lstat(full).st_mode):
            continue
        m = _DATA_RE.search(name)
        if m:
            v = int(m.group(1))
            if v <= 0xFFFFFFFF:  # parse::<u32>() fails on overflow -> skipped
                out.append(v)
    return sorted(out)


def data_file_path(path: str, file_id: int) -> str:  # log.rs:473-476
    return os.path.join(path, f"{file_id:010}.{DATA_FILE_EXTENSION}")


def hint_file_path(path: str, file_id: int) -> str:  # log.rs:478-481
    return os.path.join(path, f"{file_id:010}.{HINT_FILE_EXTENSION}")


class CaskError(Exception):
    def __init__(self, kind: str, file_id: int = 0, pos: int = 0, expected: int = 0, found: int = 0):
        super().__init__(kind)
        self.kind, self.file_id, self.pos, self.expected, self.found = kind, file_id, pos, expected, found


@dataclass
class ReplayResult:
    index: Index
    sequence: int              # max over all hints (cask.rs:350-352)
    files: list[int] = field(default_factory=list)
    error: CaskError | None = None
    file_id_seq: int = 0       # Log::file_id_seq: the last data file id at open (log.rs:63-69)

    @property
    def current_sequence(self) -> int:  # cask.rs:379
        return self.sequence + 1


def replay(path: str, write_hints: bool = True) -> ReplayResult:
    """Cask::open replay (cask.rs:335-382): ascending file ids; a valid hint file is trusted
    (log.rs:121-135), else the data file is scanned and its hint file recreated
    (log.rs:137-148, 449-471). The first Err aborts open(); hint files already written stay."""
    index = Index()
    res = ReplayResult(index=index, sequence=0, files=find_data_files(path))
    res.file_id_seq = res.files[-1] if res.files else 0
    for file_id in res.files:
        hp = hint_file_path(path, file_id)
        hb = None
        if os.path.isfile(hp):
            with open(hp, "rb") as f:
                hb = f.read()
        if hb is not None and is_valid_hint_bytes(hb):
            try:
                for h in parse_hints(hb[:-4]):
                    res.sequence = max(res.sequence, h.seq)
                    index.update(h, file_id)
            except EOFError:
                res.error = CaskError("eof", file_id=file_id)
                return res
            continue
        with open(data_file_path(path, file_id), "rb") as f:
            buf = f.read()
        rows = scan_entries(buf)
        if write_hints:
            with open(hp, "wb") as f:
                f.write(hint_file_bytes(rows))
        for r in rows:
            if r.status != ROW_OK:
                kind = "checksum" if r.status == ROW_CHECKSUM else "eof"
                res.error = CaskError(kind, file_id, r.pos, r.expected, r.found)
                return res
            res.sequence = max(res.sequence, r.seq)
            index.update(r, file_id)
    return res


def write_log(path: str, entries: list[Entry], max_file_size: int, first_file_id: int = 1,
              write_hints: bool = True) -> list[int]:
    """LogWriter::write rollover (log.rs:282-306) + EntryWriter/HintWriter (log.rs:317-395):
    a new file when there is no writer or pos + size > max_file_size. Returns file ids."""
    os.makedirs(path, exist_ok=True)
    files: list[int] = []
    cur = None
    pos = 0
    hints: list[bytes] = []

    def close():
        if cur is not None:
            with open(data_file_path(path, cur[0]), "wb") as f:
                f.write(b"".join(cur[1]))
            if write_hints:
                body = b"".join(hints)
                with open(hint_file_path(path, cur[0]), "wb") as f:
                    f.write(body + struct.pack("<I", xxhash32(body)))

    file_id = first_file_id - 1
    for e in entries:
        if cur is None or pos + e.size() > max_file_size:
            close()
            file_id += 1
            cur = (file_id, [])
            files.append(file_id)
            pos = 0
            hints = []
        cur[1].append(e.write_bytes())
        hints.append(hint_bytes(e.sequence, e.key, len(e.value), e.deleted, pos))
        pos += e.size()
    close()
    return files


# ----------------------------------------------------------------------------- compaction
def read_entry(path: str, file_id: int, entry_pos: int) -> Entry:
    """Log::read_entry (log.rs:150-166) = seek + Entry::from_read (data.rs:161-206): a short read
    is Io(UnexpectedEof), a hash mismatch InvalidChecksum{expected: stored, found: computed}."""
    with open(data_file_path(path, file_id), "rb") as f:
        f.seek(entry_pos)
        hdr = f.read(ENTRY_STATIC_SIZE)
        if len(hdr) < ENTRY_STATIC_SIZE:
            raise CaskError("eof", file_id, entry_pos)
        stored, seq, ksz, vsz = struct.unpack("<IQHI", hdr)
        deleted = vsz == ENTRY_TOMBSTONE
        key = f.read(ksz)
        value = b"" if deleted else f.read(vsz)
        if len(key) < ksz or len(value) < (0 if deleted else vsz):
            raise CaskError("eof", file_id, entry_pos)
    found = xxhash32(hdr[4:] + key + value)
    if found != stored:
        raise CaskError("checksum", file_id, entry_pos, stored, found)
    return Entry(key, value, seq, deleted)


class LogWriter:
    """LogWriter::write rollover (log.rs:245-306) with EntryWriter + HintWriter (log.rs:317-395):
    a new file (id = file_id_seq.increment(), util.rs:62-64) when there is no writer or
    pos + entry.size() > max_file_size. Files are flushed on close (the writers' Drop)."""

    def __init__(self, path: str, max_file_size: int, file_id_seq: int):
        self.path, self.max_file_size, self.file_id_seq = path, max_file_size, file_id_seq
        self.cur = None  # [file_id, [record bytes], [hint bytes], pos]

    def _flush(self):
        if self.cur is not None:
            fid, recs, hints, _ = self.cur
            with open(data_file_path(self.path, fid), "wb") as f:
                f.write(b"".join(recs))
            body = b"".join(hints)
            with open(hint_file_path(self.path, fid), "wb") as f:
                f.write(body + struct.pack("<I", xxhash32(body)))

    def write(self, e: Entry):
        """Returns ("new", file_id) or ("ok", entry_pos) like LogWrite (log.rs:260-263)."""
        new = self.cur is None or self.cur[3] + e.size() > self.max_file_size
        if new:
            self._flush()
            self.file_id_seq += 1
            self.cur = [self.file_id_seq, [], [], 0]
        pos = self.cur[3]
        self.cur[1].append(e.write_bytes())
        self.cur[2].append(hint_bytes(e.sequence, e.key, len(e.value), e.deleted, pos))
        self.cur[3] += e.size()
        return ("new", self.cur[0]) if new else ("ok", pos)

    def close(self):
        self._flush()
        self.cur = None


def _valid_hints(path: str, file_id: int):
    """Log::hints (log.rs:121-135): the hint rows if the hint file is valid, else None."""
    hp = hint_file_path(path, file_id)
    if not os.path.isfile(hp):
        return None
    with open(hp, "rb") as f:
        hb = f.read()
    return hb[:-4] if is_valid_hint_bytes(hb) else None


def compact_files(path: str, db: ReplayResult, files, max_file_size: int):
    """Cask::compact_files (cask.rs:525-560) over compact_files_aux (cask.rs:451-523). Mutates db
    (index, stats, files, file_id_seq). Per file in the given order: hints of files with a valid
    hint file (others are skipped and stay), live = index[key].sequence == hint.sequence, then
    read_entry + LogWriter.write of each live entry. The tombstones of keys absent from the index
    (highest sequence per key) are written last; the reference iterates a HashMap there, the
    restatement uses first-seen order (the engine's documented choice). Files created only by
    tombstone writes are not in new_files (cask.rs:518-520). Raises CaskError on the first
    failure, leaving what was written so far (as the reference does)."""
    compacted, new_files = [], []
    deletes: dict[bytes, int] = {}
    w = LogWriter(path, max_file_size, db.file_id_seq)
    try:
        for fid in files:
            body = _valid_hints(path, fid)
            if body is None:
                continue
            inserts = []
            try:
                hints = list(parse_hints(body))
            except EOFError:
                raise CaskError("eof", fid)
            for h in hints:
                ie = db.index.map.get(h.key)
                if h.deleted:
                    if ie is None and deletes.get(h.key, -1) < h.seq:
                        deletes[h.key] = h.seq
                elif ie is not None and ie.sequence == h.seq:
                    inserts.append(h)
            for h in inserts:
                kind, v = w.write(read_entry(path, fid, h.pos))
                if kind == "new":
                    new_files.append(v)
            compacted.append(fid)
        for key, seq in deletes.items():
            w.write(entry_deleted(seq, key))
    finally:
        w.close()
        db.file_id_seq = w.file_id_seq
    for fid in new_files:
        for h in parse_hints(_valid_hints(path, fid)):
            db.index.update(h, fid)
    db.index.stats.remove_files(compacted)
    for fid in compacted:  # Log::swap_files (log.rs:198-217)
        db.files.remove(fid)
        os.remove(data_file_path(path, fid))
        try:
            os.remove(hint_file_path(path, fid))
        except FileNotFoundError:
            pass
    db.files = sorted(db.files + new_files)
    return compacted, new_files


def compact_select(path: str, db: ReplayResult, fragmentation_trigger=0.6, dead_bytes_trigger=512 << 20,
                   fragmentation_threshold=0.4, dead_bytes_threshold=128 << 20,
                   small_file_threshold=10 << 20):
    """Cask::compact's file choice (cask.rs:563-642), stats rows visited in ascending file id
    (the reference visits a HashMap; with trigger >= threshold the chosen set is the same).
    Returns (triggered, sorted files)."""
    files: set[int] = set()
    triggered = False
    for fid in sorted(db.index.stats.map):
        e, d, b = db.index.stats.map[fid]
        frag = d / e
        if not triggered:
            if frag >= fragmentation_trigger:
                triggered = True
                files.add(fid)
            elif b >= dead_bytes_trigger and fid not in files:
                triggered = True
                files.add(fid)
        if frag >= fragmentation_threshold and fid not in files:
            files.add(fid)
        elif b >= dead_bytes_threshold and fid not in files:
            files.add(fid)
        if fid not in files:
            try:
                if os.path.getsize(data_file_path(path, fid)) <= small_file_threshold:
                    files.add(fid)
            except OSError:
                pass
    return triggered, sorted(files)

"""cask_shard.py — restatement of the shard keydir block (cask_amd/csrc/k_keydir.hip,
keydir_format.h) and of rank 0's fold (engine.cpp cask_keydir_merge / cask_keydir_finish).
TEST INFRASTRUCTURE ONLY: the gloo tests build blocks with it on the CPU, the GPU tests compare the
device's blocks with it byte for byte, and the property tests check the whole scheme against the
reference's in-order fold (Index::update, cask.rs:60-90; Stats, stats.rs:23-48) restated in
cask_ref.py. Never imported by the product.
"""
from __future__ import annotations

import struct

import cask_ref as R

M64 = (1 << 64) - 1
MAGIC, VERSION = 0x52444B43, 1
KEPT, COND, RAW = 0, 1, 2
HDR = struct.Struct("<IIQQIIQQQQ")   # 64 B
REC = struct.Struct("<QQIIHBBI")     # 32 B
FST = struct.Struct("<IIQQQQ")       # 40 B


def _mix64(z: int) -> int:
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def key_hash(k: bytes) -> int:
    """k_keydir.hip key_hash."""
    n = len(k)
    h = 0x9E3779B97F4A7C15 ^ ((n * 0xD6E8FEB86659FD93) & M64)
    i = 0
    while i + 8 <= n:
        h = _mix64(h ^ int.from_bytes(k[i:i + 8], "little"))
        i += 8
    t = int.from_bytes(k[i:], "little")
    return _mix64(h ^ t ^ 0xA0761D6478BD642F)


def shard_block(file_ids: list[int], rows: list[tuple[int, "R.Row"]]) -> bytes:
    """The keydir block of a shard: `file_ids` its data files in order, `rows` its Ok rows in
    replay order as (file_id, Row with key)."""
    fidx = {f: i for i, f in enumerate(file_ids)}
    n = len(rows)
    fst = [[0, 0, 0, 0] for _ in file_ids]
    for fid, r in rows:
        if not r.deleted:
            fst[fidx[fid]][0] += 1
            fst[fidx[fid]][1] += R.ENTRY_STATIC_SIZE + r.ksz + r.vsz_raw
    order = sorted(range(n), key=lambda d: (key_hash(rows[d][1].key), d))
    kind = [0] * n
    tval = [0] * n
    i = 0
    while i < n:
        h = key_hash(rows[order[i]][1].key)
        j = i
        while j < n and key_hash(rows[order[j]][1].key) == h:
            j += 1
        seg = order[i:j]
        if any(rows[d][1].key != rows[seg[0]][1].key for d in seg):
            for p in range(i, j):
                kind[p] = 4
        else:
            later = 0
            for p in range(j - 1, i - 1, -1):  # suffix-strict maxima
                q = rows[order[p]][1].seq + 1
                kind[p] = 1 if q > later else 0
                later = max(later, q)
            L = A = C = 0
            for p in range(i, j):
                fid, r = rows[order[p]]
                q = r.seq + 1
                if not r.deleted:
                    A, C = max(A, q), max(C, q)
                    continue
                if C > q:
                    fst[fidx[fid]][2] += 1
                    fst[fidx[fid]][3] += R.ENTRY_STATIC_SIZE + r.ksz
                else:
                    kind[p] |= 2
                    tval[p] = L if A > q else max(L, q)
                if A > q:
                    C = C if C > q else 0
                else:
                    L, C = max(L, q), 0
        i = j
    recs, keys = [], []

    def emit(fid, r, k, seq):
        recs.append(REC.pack(r.pos, seq, fid, r.vsz_raw, r.ksz, k, 0, 0))
        keys.append(r.key)

    for p in range(n):
        fid, r = rows[order[p]]
        kd = kind[p]
        if kd & 4:
            emit(fid, r, RAW, r.seq)
            continue
        if kd & 2:
            emit(fid, r, COND, tval[p])
        if kd & 1:
            emit(fid, r, KEPT, r.seq)
    fbytes = b"".join(FST.pack(f, 0, *fst[i]) for i, f in enumerate(file_ids))
    kb = b"".join(keys)
    body = b"".join(recs) + fbytes + kb
    total = (HDR.size + len(body) + 7) & ~7
    maxp1 = max((r.seq for _, r in rows), default=-1) + 1
    hdr = HDR.pack(MAGIC, VERSION, len(recs), len(kb), len(file_ids), 0, maxp1, n, total, 0)
    return (hdr + body).ljust(total, b"\0")


def parse_block(b: bytes):
    (magic, ver, nrec, kb, nfiles, _, maxp1, rows_in, total, _) = HDR.unpack_from(b, 0)
    assert magic == MAGIC and ver == VERSION
    recs = [REC.unpack_from(b, HDR.size + REC.size * i) for i in range(nrec)]
    fat = HDR.size + REC.size * nrec
    fst = [FST.unpack_from(b, fat + FST.size * i) for i in range(nfiles)]
    kat = fat + FST.size * nfiles
    out, ko = [], kat
    for (pos, seq, fid, vsz, ksz, kind, _, _) in recs:
        out.append((kind, fid, pos, seq, vsz, ksz, bytes(b[ko:ko + ksz])))
        ko += ksz
    return out, fst, maxp1


def fold_blocks(blocks: list[bytes]):
    """Restatement of cask_keydir_merge over the blocks in order, then cask_keydir_finish.
    Returns (keydir {key: (file_id, pos, size, seq)}, stats {file: (entries, dead, dead_bytes)},
    max sequence or -1)."""
    kd = {}
    terms = {}
    maxs = -1

    def stale(fid, ksz):
        t = terms.setdefault(fid, [0, 0, 0, 0])
        t[2] += 1
        t[3] += R.ENTRY_STATIC_SIZE + ksz

    def update(k, fid, pos, vsz, seq):  # Index::update's keydir effect
        dele = vsz == R.ENTRY_TOMBSTONE
        if k in kd:
            if kd[k][3] <= seq:
                if dele:
                    del kd[k]
                else:
                    kd[k] = (fid, pos, R.ENTRY_STATIC_SIZE + len(k) + vsz, seq)
        elif not dele:
            kd[k] = (fid, pos, R.ENTRY_STATIC_SIZE + len(k) + vsz, seq)

    for b in blocks:
        recs, fst, maxp1 = parse_block(b)
        for (kind, fid, pos, seq, vsz, ksz, k) in recs:
            if kind == COND and ((kd[k][3] + 1) if k in kd else 0) > seq:
                stale(fid, ksz)
        for (kind, fid, pos, seq, vsz, ksz, k) in recs:
            if kind == COND:
                continue
            if kind == RAW and vsz == R.ENTRY_TOMBSTONE and k in kd and kd[k][3] > seq:
                stale(fid, ksz)
            update(k, fid, pos, vsz, seq)
        for (fid, _, puts, pb, st, sb) in fst:
            t = terms.setdefault(fid, [0, 0, 0, 0])
            t[0] += puts
            t[1] += pb
            t[2] += st
            t[3] += sb
        maxs = max(maxs, maxp1 - 1)
    live = {}
    for k, (fid, pos, size, seq) in kd.items():
        l = live.setdefault(fid, [0, 0])
        l[0] += 1
        l[1] += size
    stats = {}
    for fid, (puts, pb, st, sb) in terms.items():
        if puts or st:
            le, lb = live.get(fid, (0, 0))
            stats[fid] = (puts + st, puts - le + st, pb - lb + sb)
    return kd, stats, maxs


def key_owner(k: bytes, nparts: int) -> int:
    """keydir_format.h key_owner: the high 32 bits of the key hash scaled to [0, nparts)."""
    return ((key_hash(k) >> 32) * nparts) >> 32


def partition_block(b: bytes, nparts: int) -> list[bytes]:
    """Restatement of the key-hash partition (keydir_format.h; k_keydir.hip kd_partition, engine.cpp
    cask_keydir_partition_host): part o = the records whose key's owner is o, in block order, their
    keys, and the stats table (counts in part 0 only)."""
    (magic, ver, nrec, kb, nfiles, _, maxp1, rows_in, total, _) = HDR.unpack_from(b, 0)
    assert magic == MAGIC and ver == VERSION
    fat = HDR.size + REC.size * nrec
    kat = fat + FST.size * nfiles
    fst = [FST.unpack_from(b, fat + FST.size * i) for i in range(nfiles)]
    recs = [[] for _ in range(nparts)]
    keys = [[] for _ in range(nparts)]
    ko = kat
    for i in range(nrec):
        raw = b[HDR.size + REC.size * i:HDR.size + REC.size * (i + 1)]
        ksz = REC.unpack(raw)[4]
        k = bytes(b[ko:ko + ksz])
        ko += ksz
        o = key_owner(k, nparts)
        recs[o].append(bytes(raw))
        keys[o].append(k)
    out = []
    for o in range(nparts):
        fb = b"".join(FST.pack(f, 0, *((p, pb, s, sb) if o == 0 else (0, 0, 0, 0))) for (f, _, p, pb, s, sb) in fst)
        kbytes = b"".join(keys[o])
        body = b"".join(recs[o]) + fb + kbytes
        size = (HDR.size + len(body) + 7) & ~7
        hdr = HDR.pack(MAGIC, VERSION, len(recs[o]), len(kbytes), nfiles, 0, maxp1, rows_in if o == 0 else 0, size, 0)
        out.append((hdr + body).ljust(size, b"\0"))
    return out

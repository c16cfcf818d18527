"""Parity of the HIP scan (through the C ABI) with the CPU oracle. Needs an MI355X.

Bit-exact comparisons on the golden fixtures and on seeded inputs the oracle finishes in seconds
(uniform, variable, long records, many/empty files, adversarial values, corruption, truncation,
all-zero data); size-independent properties at BASELINE configs[1] size (8 x 1,073,741,820 B).
"""
import json
import os
import random
import shutil

import numpy as np
import pytest

from conftest import GOLDEN, golden_cases

import cask_ref as R
import oracle_ffi as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["auto", "walk", "wide"])
def scan_mode(request, monkeypatch):
    """Every test here runs three times: the mode the library picks (k_scan_chunks for these mostly
    short records — with the short 1,008-B halo when the file heads hold short records — and the
    walk for the long-record cases), the walk mode forced (k_walk_search, k_walk_chase, k_run_hash),
    and the chunk scan forced
    with the wide 4,080-B halo (there host-resident inputs and rows also go through the pinned
    staging ring, CASK_STAGE_MIN=0)."""
    if request.param == "auto":
        monkeypatch.delenv("CASK_SCAN_MODE", raising=False)
    else:
        monkeypatch.setenv("CASK_SCAN_MODE", request.param)
    if request.param == "wide":  # host-resident scans staged through the pinned ring on threads
        monkeypatch.setenv("CASK_STAGE_MIN", "0")
    return request.param


def _expected(case):
    with open(os.path.join(GOLDEN, case, "expected.json")) as f:
        return json.load(f)


def _file_bytes(case, fid):
    with open(R.data_file_path(os.path.join(GOLDEN, case), fid), "rb") as f:
        return f.read()


def rows_list(res, sl):
    return [[int(res.pos[i]), int(res.seq[i]) & 0xFFFFFFFFFFFFFFFF, int(res.ksz[i]) & 0xFFFF, int(res.vsz[i]) & 0xFFFFFFFF, int(res.status[i])]
            for i in range(sl.start, sl.stop)]


def oracle_rows(buf):
    rows = O.scan(buf)
    return [[int(r["pos"]), int(r["seq"]), int(r["ksz"]), int(r["vsz_raw"]), int(r["status"])] for r in rows], rows


def check_against_oracle(ctx, bufs, device=False):
    """Scan `bufs` (list of bytes) in one call; compare every row and the first error."""
    files = list(enumerate(bufs, start=1))
    if device:
        import torch
        tens = [(fid, torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()) for fid, b in files]
        res = ctx.scan_device(tens)
        res.pos, res.seq, res.vsz, res.ksz, res.status = [t[:res.count].cpu().numpy() for t in
                                                          (res.pos, res.seq, res.vsz, res.ksz, res.status)]
    else:
        res = ctx.scan_host(files)
    first_err = None
    total = 0
    for i, (fid, b) in enumerate(files):
        want, orows = oracle_rows(b)
        got = rows_list(res, res.file_rows(i))
        assert len(got) == len(want), (fid, len(got), len(want))
        if got != want:
            bad = next(j for j in range(len(got)) if got[j] != want[j])
            raise AssertionError(f"file {fid} row {bad}: got {got[bad]} want {want[bad]}")
        total += len(want)
        if first_err is None:
            for r in orows:
                if int(r["status"]) != 0:
                    first_err = (int(r["status"]), fid, int(r["pos"]), int(r["expected"]),
                                 int(r["found"]) if int(r["status"]) == 1 else 0)
                    break
    assert res.count == total
    if first_err is None:
        assert res.error is None
    else:
        e = res.error
        assert e is not None
        assert (e.kind, e.file_id, e.pos, e.expected, e.found) == first_err
    return res


# ------------------------------------------------------------------------------------- golden
@pytest.mark.parametrize("case", golden_cases())
def test_golden_rows_host(gpu_ctx, case):
    exp = _expected(case)
    bufs = [_file_bytes(case, fe["file_id"]) for fe in exp["files"]]
    files = [(fe["file_id"], b) for fe, b in zip(exp["files"], bufs)]
    res = gpu_ctx.scan_host(files)
    for i, fe in enumerate(exp["files"]):
        assert rows_list(res, res.file_rows(i)) == [r[:5] for r in fe["rows"]], fe["file_id"]
    rep = exp["replay"]["error"]
    if rep is not None and not case.startswith("hints"):
        assert res.error is not None
        assert res.error.file_id == rep["file_id"] and res.error.pos == rep["pos"]
        if rep["kind"] == "checksum":
            assert (res.error.kind, res.error.expected, res.error.found) == (1, rep["expected"], rep["found"])
        else:
            assert res.error.kind == 2


@pytest.mark.parametrize("case", golden_cases())
def test_golden_rows_device(gpu_ctx, case):
    exp = _expected(case)
    bufs = [_file_bytes(case, fe["file_id"]) for fe in exp["files"]]
    check_against_oracle(gpu_ctx, bufs, device=True)


@pytest.mark.parametrize("fold", ["devfold", "fold", "sharded_fold"])
@pytest.mark.parametrize("case", golden_cases())
def test_golden_engine_open(native, case, tmp_path, monkeypatch, fold):
    """Cask::open on the fixture directory: keydir, stats, sequence or error, hint files — with the
    keydir reduced on the device and merged (the default when every file is scanned), and with the
    host fold (CASK_OPEN_DEVFOLD=0) on one thread and sharded by key hash over threads
    (CASK_PAR_FOLD_MIN=0 forces it); the last two with every data file a pipeline batch of its own
    (read, scanned and folded in turn)."""
    from cask_amd import CaskOptions, errors
    par_fold = fold != "fold"
    monkeypatch.setenv("CASK_OPEN_DEVFOLD", "1" if fold == "devfold" else "0")
    monkeypatch.setenv("CASK_PAR_FOLD_MIN", "0" if par_fold else str(1 << 62))
    if par_fold:  # and the hint bodies' copy to the host staged through the pinned ring
        monkeypatch.setenv("CASK_STAGE_MIN", "0")
        monkeypatch.setenv("CASK_OPEN_BATCH", "1")
    exp = _expected(case)
    rep = exp["replay"]
    d = tmp_path / case
    shutil.copytree(os.path.join(GOLDEN, case), d)
    os.remove(d / "expected.json")
    if rep["error"] is None:
        with CaskOptions().open(str(d)) as db:
            got = sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence] for k, e in db.index().items())
            assert got == rep["keydir"]
            assert sorted([f, *s] for f, s in db.stats().items()) == rep["stats"]
            assert db.current_sequence == rep["current_sequence"]
    else:
        want = errors.InvalidChecksum if rep["error"]["kind"] == "checksum" else errors.UnexpectedEof
        with pytest.raises(want) as ei:
            CaskOptions().open(str(d))
        assert ei.value.file_id == rep["error"]["file_id"] and ei.value.pos == rep["error"]["pos"]
        if rep["error"]["kind"] == "checksum":
            assert (ei.value.expected, ei.value.found) == (rep["error"]["expected"], rep["error"]["found"])
    for fid, hx in rep["hint_files_after"].items():
        with open(R.hint_file_path(str(d), int(fid)), "rb") as f:
            assert f.read().hex() == hx, fid


# ------------------------------------------------------------------------------ seeded inputs
def make_records(rng, n, ksz_fn, vsz_fn, seq0=1, tomb_p=0.0):
    out = []
    for i in range(n):
        k = rng.randbytes(ksz_fn(rng))
        if rng.random() < tomb_p:
            out.append(R.entry_deleted(seq0 + i, k).write_bytes())
        else:
            out.append(R.entry_new(seq0 + i, k, rng.randbytes(vsz_fn(rng))).write_bytes())
    return b"".join(out)


@pytest.mark.parametrize("batch", [None, "1"], ids=["batches", "file_batches"])
def test_sharded_fold_matches_single_thread(native, tmp_path, monkeypatch, batch):
    """Many files of overwrites, stale and live tombstones and out-of-order sequences: the sharded
    fold and the device-reduced block merged on the host must give the single-thread fold's keydir,
    stats and sequence (Index::update, Stats); the device path also with every file a batch of its
    own (its rows gathered batch after batch into one block)."""
    if batch:
        monkeypatch.setenv("CASK_OPEN_BATCH", batch)
    from cask_amd import CaskOptions
    rng = random.Random(53)
    keys = [rng.randbytes(rng.randrange(0, 24)) for _ in range(700)]
    d = tmp_path / "db"
    d.mkdir()
    seq = 1
    for fid in range(1, 7):
        recs = []
        for _ in range(2500):
            k = rng.choice(keys)
            s = seq if rng.random() < 0.9 else max(1, seq - rng.randrange(1, 3000))  # some stale sequences
            seq += 1
            if rng.random() < 0.15:
                recs.append(R.entry_deleted(s, k).write_bytes())
            else:
                recs.append(R.entry_new(s, k, rng.randbytes(rng.randrange(0, 300))).write_bytes())
        with open(R.data_file_path(str(d), fid), "wb") as f:
            f.write(b"".join(recs))
    got = []
    for par, devfold in ((False, "0"), (True, "0"), (False, "1")):
        for h in d.glob("*.cask.hint"):
            h.unlink()  # every open takes the scan path
        monkeypatch.setenv("CASK_PAR_FOLD_MIN", "0" if par else str(1 << 62))
        monkeypatch.setenv("CASK_OPEN_DEVFOLD", devfold)
        with CaskOptions().open(str(d)) as db:
            got.append((sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence] for k, e in db.index().items()),
                        sorted([f, *st] for f, st in db.stats().items()), db.current_sequence))
    assert got[0] == got[1] == got[2]
    assert len(got[0][0]) > 100


def test_devfold_forced_hash_collisions(native, tmp_path, monkeypatch):
    """The device-reduced keydir where different keys share a key-hash segment (CASK_KD_HASH_BITS
    groups rows by 4 bits of the hash, then by none): k_kd_segs must tell the keys apart — short
    keys by their gathered 16 bytes, longer ones sharing those 16 bytes by the rest from the files —
    and send such segments whole (kRaw); the merged keydir, stats and sequence equal the host
    fold's, as with the full hash."""
    from cask_amd import CaskOptions
    rng = random.Random(71)
    prefixes = [rng.randbytes(16) for _ in range(4)]
    keys = [rng.randbytes(rng.randrange(0, 17)) for _ in range(150)]
    keys += [rng.choice(prefixes) + rng.randbytes(rng.randrange(1, 30)) for _ in range(150)]
    keys += [p[:rng.randrange(0, 17)] for p in prefixes]
    d = tmp_path / "db"
    d.mkdir()
    seq = 1
    for fid in range(1, 4):
        recs = []
        for _ in range(3000):
            k = rng.choice(keys)
            s = seq if rng.random() < 0.9 else max(1, seq - rng.randrange(1, 2000))
            seq += 1
            if rng.random() < 0.15:
                recs.append(R.entry_deleted(s, k).write_bytes())
            else:
                recs.append(R.entry_new(s, k, rng.randbytes(rng.randrange(0, 200))).write_bytes())
        with open(R.data_file_path(str(d), fid), "wb") as f:
            f.write(b"".join(recs))
    got = []
    for devfold, bits in (("0", None), ("1", None), ("1", "4"), ("1", "0")):
        for h in d.glob("*.cask.hint"):
            h.unlink()
        monkeypatch.setenv("CASK_OPEN_DEVFOLD", devfold)
        if bits is None:
            monkeypatch.delenv("CASK_KD_HASH_BITS", raising=False)
        else:
            monkeypatch.setenv("CASK_KD_HASH_BITS", bits)
        with CaskOptions().open(str(d)) as db:
            got.append((sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence] for k, e in db.index().items()),
                        sorted([f, *st] for f, st in db.stats().items()), db.current_sequence))
    assert got[0] == got[1] == got[2] == got[3]
    assert len(got[0][0]) > 200


def test_uniform_290(gpu_ctx):
    rng = random.Random(1)
    buf = make_records(rng, 20000, lambda r: 16, lambda r: 256)
    res = check_against_oracle(gpu_ctx, [buf])
    cnt = gpu_ctx.last_counters()
    assert cnt["repaired_chunks"] == 0 and cnt["dense_path"] == 1, cnt


def test_short_halo_records_crossing_the_window(gpu_ctx):
    """Short records at the file heads pick the 1,008-B halo; records of 1-4 KiB later in the file
    then cross the window's end and go to k_long_hash (some corrupted), row for row."""
    rng = random.Random(11)
    head = make_records(rng, 300, lambda r: 16, lambda r: 100)
    tail = bytearray(make_records(rng, 2000, lambda r: r.randrange(0, 30),
                                  lambda r: r.randrange(0, 4000), tomb_p=0.05, seq0=301))
    for _ in range(6):
        tail[rng.randrange(len(tail))] ^= 1 << rng.randrange(8)
    check_against_oracle(gpu_ctx, [head + bytes(tail)], device=True)
    cnt = gpu_ctx.last_counters()
    if os.environ.get("CASK_SCAN_MODE") is None:
        assert cnt["geometry"] == 3 and cnt["long_records"] > 0, cnt


def test_repeated_calls_alternating_file_sets(gpu_ctx):
    """The file table and the call blocks stay on the device between calls (a call over the same
    files as the last one copies nothing before its first kernel; k_finish clears the next call's
    block): calls alternating between a clean set, a set with a checksum error and a set that
    takes the repair path, each set's device buffers reused, must each give the oracle's rows."""
    import torch
    rng = random.Random(17)
    clean = [make_records(rng, 3000, lambda r: 16, lambda r: 256, seq0=1 + 3000 * i) for i in range(3)]
    bad = bytearray(make_records(rng, 2500, lambda r: r.randrange(1, 20), lambda r: r.randrange(0, 900)))
    bad[len(bad) // 2] ^= 0x40
    inner = [R.entry_new(10_000 + i, rng.randbytes(8), rng.randbytes(rng.randrange(0, 40))).write_bytes()
             for i in range(64)]
    adv = b"".join(R.entry_new(i + 1, b"outer%d" % i, b"".join(rng.choice(inner) for _ in range(rng.randrange(1, 30))))
                   .write_bytes() for i in range(2000))
    sets = {"clean": clean, "bad": [clean[0], bytes(bad)], "adv": [adv, clean[1]]}
    dev = {k: [(i + 1, torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()) for i, b in enumerate(v)]
           for k, v in sets.items()}
    want = {k: [O.scan(b) for b in v] for k, v in sets.items()}
    for k in ["clean", "clean", "bad", "clean", "adv", "adv", "clean", "bad", "bad", "clean", "clean"]:
        res = gpu_ctx.scan_device(dev[k])
        assert res.count == sum(len(w) for w in want[k]), k
        for i, w in enumerate(want[k]):
            sl = res.file_rows(i)
            assert np.array_equal(res.pos[sl].cpu().numpy().astype(np.uint64), w["pos"]), (k, i)
            assert np.array_equal(res.seq[sl].cpu().numpy().astype(np.uint64), w["seq"]), (k, i)
            assert np.array_equal(res.status[sl].cpu().numpy(), w["status"].astype(np.uint8)), (k, i)
            assert np.array_equal(res.vsz[sl].cpu().numpy().astype(np.uint32), w["vsz_raw"].astype(np.uint32)), (k, i)
            assert np.array_equal(res.ksz[sl].cpu().numpy().astype(np.uint16), w["ksz"].astype(np.uint16)), (k, i)
        assert (res.error is None) == (k != "bad"), k


def test_uniform_82_device(gpu_ctx):
    rng = random.Random(2)
    check_against_oracle(gpu_ctx, [make_records(rng, 60000, lambda r: 16, lambda r: 48)], device=True)


def test_variable_sizes_with_long_records(gpu_ctx):
    rng = random.Random(3)

    def vsz(r):
        x = r.random()
        if x < 0.5:
            return r.randrange(0, 64)
        if x < 0.9:
            return r.randrange(64, 4096)
        return r.randrange(4096, 70000)
    buf = make_records(rng, 3000, lambda r: r.randrange(0, 40), vsz, tomb_p=0.1)
    check_against_oracle(gpu_ctx, [buf])
    cnt = gpu_ctx.last_counters()
    assert cnt["long_records"] > 0 or cnt["walk_mode"] >= 1, cnt  # k_long_hash, or the walk hashed them


def _zipf_vsz(rng, s=1.1, kmax=4096):
    """vsz = 16·k, k ~ Zipf(s) truncated to [1, kmax] (BASELINE configs[2] shape)."""
    w = [k ** -s for k in range(1, kmax + 1)]
    tot = sum(w)
    cdf, acc = [], 0.0
    for x in w:
        acc += x / tot
        cdf.append(acc)
    import bisect

    def f(r):
        return 16 * (min(bisect.bisect_left(cdf, r.random()), kmax - 1) + 1)
    return f


@pytest.mark.parametrize("seed", [41, 42])
def test_zipf_sizes_long_records(gpu_ctx, seed):
    """configs[2] record shape (16 B keys, Zipf value sizes up to 64 KiB): most bytes sit in
    records longer than the window, whose starts the speculative search cannot verify; the local
    repair (exact re-scans from T[c]) must settle them without the serial walk."""
    rng = random.Random(seed)
    buf = make_records(rng, 4000, lambda r: 16, _zipf_vsz(rng), tomb_p=0.02)
    check_against_oracle(gpu_ctx, [buf, buf[: len(buf) // 3]], device=True)
    cnt = gpu_ctx.last_counters()
    assert cnt["long_records"] > 0 or cnt["walk_mode"] >= 1, cnt
    assert cnt["walked"] == 0, cnt


@pytest.mark.parametrize("seqs", ["rising", "shuffled", "jumps", "corrupt"])
def test_walk_search_long_stretches(gpu_ctx, seqs):
    """k_walk_search where a run's first short record lies behind stretches of 4-8 records of ~64 KiB
    (>= 30 windows of 8 KiB): the probe follows the long candidates' chains header to header to the
    first short record and hashes it (k_walk.hip, phase 3). Its chains must raise the sequence by at
    most 2^32 per hop: with rising sequences it takes that path; with the sequences shuffled, or
    jumping by 2^33 at every stretch, it must fall back to the windows; with a byte flipped in some
    of the short records behind the stretches (their checksums fail) it must move on to a later
    candidate. Rows and the first error equal the oracle's row for row (24 MiB: many 1-MiB runs
    start inside a stretch)."""
    rng = random.Random(0x5EA)
    recs, seq, bad = [], 1, []
    seqlist = list(range(1, 4000))
    if seqs == "shuffled":
        rng.shuffle(seqlist)
    total = 0
    while total < 24 << 20:
        for _ in range(rng.randrange(4, 9)):
            s = seqlist[len(recs)] if seqs == "shuffled" else seq
            recs.append(R.entry_new(s, rng.randbytes(16), rng.randbytes(rng.randrange(60000, 65536))).write_bytes())
            seq += 1
            total += len(recs[-1])
        if seqs == "jumps":
            seq += 1 << 33
        for j in range(rng.randrange(1, 4)):
            s = seqlist[len(recs)] if seqs == "shuffled" else seq
            r = bytearray(R.entry_new(s, rng.randbytes(16), rng.randbytes(rng.randrange(0, 200))).write_bytes())
            if seqs == "corrupt" and j == 0 and rng.random() < 0.3:
                r[len(r) - 1 if len(r) > 34 else 20] ^= 0x40
                bad.append(len(recs))
            recs.append(bytes(r))
            seq += 1
            total += len(recs[-1])
    assert seqs != "corrupt" or bad
    buf = b"".join(recs)
    check_against_oracle(gpu_ctx, [buf, buf[: len(buf) // 2 + 12345]], device=True)
    cnt = gpu_ctx.last_counters()
    if os.environ.get("CASK_SCAN_MODE") in (None, "walk") and seqs != "corrupt":
        assert cnt["walk_mode"] >= 1 and cnt["walked"] == 0, cnt


def test_walk_slot_rows_overflow_redo(gpu_ctx):
    """A walk-mode call sizes its slot rows for kWalkSlotCap (128) records per 32-KiB chunk: a log of
    long records with a burst of ~600 tiny ones inside one chunk overflows them, and the call is
    redone with full slot rows — same rows as the oracle either way; the Zipf log alone keeps the
    small slots (its scratch is a fraction of its bytes)."""
    import torch
    rng = random.Random(77)
    head = make_records(rng, 300, lambda r: 16, _zipf_vsz(rng))
    burst = make_records(rng, 600, lambda r: 4, lambda r: 20, seq0=301)  # 42-B records
    tail = make_records(rng, 300, lambda r: 16, _zipf_vsz(rng), seq0=901)
    check_against_oracle(gpu_ctx, [head + burst + tail], device=True)
    if os.environ.get("CASK_SCAN_MODE") in (None, "walk"):
        zipf = make_records(rng, 3000, lambda r: 16, _zipf_vsz(rng), tomb_p=0.02)
        ctx2 = type(gpu_ctx)(0)  # a fresh context: its scratch is this call's alone
        t = torch.from_numpy(np.frombuffer(zipf, np.uint8).copy()).cuda()
        res = ctx2.scan_device([(1, t)])
        assert res.error is None
        if ctx2.last_counters()["walk_mode"] == 1:
            nch = (len(zipf) + 32767) // 32768
            assert ctx2.scratch_bytes() < 8192 * nch + (8 << 20), (ctx2.scratch_bytes(), nch)


@pytest.mark.parametrize("corrupt", [False, True])
def test_mixed_modes_in_one_call(gpu_ctx, corrupt):
    """One call over a file of fixed 290-B records (configs[1] shape), a file of Zipf-length records
    (configs[2] shape) and a file with a short-record head and a long-record body: the library picks
    the mode per region of each file (chunk mode for the short records, walk mode for the long ones,
    walk_mode == 2), and the rows equal the oracle's row for row — with a flipped byte in the short
    and in the long regions too."""
    rng = random.Random(61)
    a = bytearray(make_records(rng, 29000, lambda r: 16, lambda r: 256))
    b = bytearray(make_records(rng, 5000, lambda r: 16, _zipf_vsz(rng), seq0=100_000, tomb_p=0.02))
    head = make_records(rng, 25000, lambda r: 16, lambda r: r.randrange(40, 160), seq0=200_000)
    body = make_records(rng, 2600, lambda r: 16, _zipf_vsz(rng), seq0=300_000)
    c = bytearray(head + body)
    if corrupt:
        a[len(a) // 2] ^= 0x08
        c[len(c) - len(body) // 3] ^= 0x80
    check_against_oracle(gpu_ctx, [bytes(a), bytes(b), bytes(c)], device=True)
    cnt = gpu_ctx.last_counters()
    if os.environ.get("CASK_SCAN_MODE") is None:
        assert cnt["walk_mode"] == 2, cnt


def test_zipf_sizes_corrupt(gpu_ctx):
    rng = random.Random(43)
    buf = bytearray(make_records(rng, 3000, lambda r: 16, _zipf_vsz(rng)))
    for _ in range(3):
        buf[rng.randrange(len(buf))] ^= 1 << rng.randrange(8)
    check_against_oracle(gpu_ctx, [bytes(buf)], device=True)


def test_zipf_many_failures_on_a_caller_stream(gpu_ctx):
    """Walk mode with k_finish beside the hash: many checksum failures spread over many chunks (the
    statuses k_hash_fix sets after both), one record cut short at the end, the scan on a stream the
    caller owns (the side stream must order itself after it and the caller's stream after the
    side stream) — rows and the first error against the oracle, twice, the second call reusing the
    device buffers."""
    import torch
    rng = random.Random(53)
    buf = bytearray(make_records(rng, 6000, lambda r: 16, _zipf_vsz(rng), tomb_p=0.02))
    for _ in range(150):
        buf[rng.randrange(len(buf))] ^= 1 << rng.randrange(8)
    short = bytes(buf[: len(buf) - 7])  # the last record cut short: an UnexpectedEof row
    s = torch.cuda.Stream()
    old = gpu_ctx.stream_ptr
    gpu_ctx.set_stream(s.cuda_stream)
    try:
        for _ in range(2):
            check_against_oracle(gpu_ctx, [bytes(buf), short], device=True)
    finally:
        gpu_ctx.set_stream(old)


def test_long_record_hash_every_length_residue(gpu_ctx):
    """Records past ScanArgs::big (2 KiB) are hashed from HBM by quads of lanes (k_long_hash): every
    hashed length mod 64 (full 4-stripe blocks, 1-3 trailing stripes, 0-15 tail bytes), with value
    bytes flipped in a third of them, must give the oracle's statuses row for row."""
    rng = random.Random(47)
    recs, seq = [], 1
    for vsz in list(range(2020, 2150)) + [rng.randrange(4096, 70000) for _ in range(12)]:
        rec = bytearray(R.entry_new(seq, rng.randbytes(16), rng.randbytes(vsz)).write_bytes())
        if rng.random() < 0.33:
            rec[18 + 16 + rng.randrange(vsz)] ^= 1 << rng.randrange(8)
        recs.append(bytes(rec))
        seq += 1
    buf = b"".join(recs)
    res = check_against_oracle(gpu_ctx, [buf, buf[: len(buf) // 2]], device=True)
    cnt = gpu_ctx.last_counters()
    assert cnt["long_records"] > 0 or cnt["walk_mode"] >= 1, cnt
    assert res.error is not None


def test_line_rounds_every_offset_and_length(gpu_ctx):
    """k_run_hash reads a record in rounds of whole 128-B lines from the line of its body's first
    byte and funnels the body out of them (walk mode): bodies starting at every offset in a line
    (each residue mod 128 many times), body lengths around the 16-B stripe, 64-B block, 128-B line and
    1-KiB round boundaries, stored checksums that start in the line before the body's, a third of
    the records corrupted in the body, the stored checksum or the tail, and files ending inside the
    last record's 16-B tail granule — row for row as the oracle."""
    rng = random.Random(71)
    lens = [14, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 1007, 1008, 1009, 1023, 1024, 1025,
            1039, 1040, 1041, 2047, 2048, 2049, 3071, 3072, 3073, 4095, 4096, 4097]
    files, seq = [], 1
    for f in range(3):
        recs = []
        for _ in range(900):
            body = rng.choice(lens) if rng.random() < 0.7 else rng.randrange(14, 9000)
            ksz = rng.randrange(0, 24)
            vsz = max(0, body - 14 - ksz)  # body = 14 + ksz + vsz (header past the checksum + key + value)
            rec = bytearray(R.entry_new(seq, rng.randbytes(ksz), rng.randbytes(vsz)).write_bytes())
            seq += 1
            x = rng.random()
            if x < 0.11:
                rec[4 + rng.randrange(len(rec) - 4)] ^= 1 << rng.randrange(8)  # body
            elif x < 0.22:
                rec[rng.randrange(4)] ^= 0x01  # stored checksum
            elif x < 0.33:
                rec[-1 - rng.randrange(min(15, len(rec) - 1))] ^= 0x80  # the tail bytes
            recs.append(bytes(rec))
        files.append(b"".join(recs))
    # the last file cut inside its last record's tail: an UnexpectedEof row at the end
    files.append(files[0][: len(files[0]) - 7])
    res = check_against_oracle(gpu_ctx, files, device=True)
    assert res.error is not None
    starts = np.concatenate([O.scan(b)["pos"] for b in files[:3]]).astype(np.int64)
    assert len(set(((starts + 4) % 128).tolist())) == 128  # every body offset in a line was exercised


def test_records_past_walk_hash_limit(gpu_ctx):
    """Records over 2 MiB (the chunk scan leaves them to k_long_hash; k_walk_hash hashes them in
    stride, past their run's end) between short ones, one corrupted."""
    rng = random.Random(48)
    recs = []
    for i, vsz in enumerate([40, 2_500_000, 17, 2_200_000, 3000, 2_097_200, 9]):
        rec = bytearray(R.entry_new(i + 1, rng.randbytes(16), rng.randbytes(vsz)).write_bytes())
        if i == 3:
            rec[18 + 16 + 777_777] ^= 0x10
        recs.append(bytes(rec))
    check_against_oracle(gpu_ctx, [b"".join(recs)], device=True)
    cnt = gpu_ctx.last_counters()
    assert cnt["long_records"] >= 3 or cnt["walk_mode"] >= 1, cnt


def test_many_files_empty_and_tiny(gpu_ctx):
    rng = random.Random(4)
    bufs = []
    for i in range(40):
        kind = i % 5
        if kind == 0:
            bufs.append(b"")
        elif kind == 1:
            bufs.append(rng.randbytes(rng.randrange(1, 18)))  # shorter than a header: EOF row
        else:
            bufs.append(make_records(rng, rng.randrange(1, 400), lambda r: r.randrange(1, 20),
                                     lambda r: r.randrange(0, 600)))
    check_against_oracle(gpu_ctx, bufs)


def test_adversarial_embedded_records_repair(gpu_ctx):
    """Values made of valid serialized records defeat the speculative boundary search; the
    validate pass must catch it and the exact walk must repair it."""
    rng = random.Random(5)
    inner = [R.entry_new(10_000 + i, rng.randbytes(8), rng.randbytes(rng.randrange(0, 40))).write_bytes()
             for i in range(64)]
    out = []
    for i in range(3000):
        v = b"".join(rng.choice(inner) for _ in range(rng.randrange(1, 30)))
        out.append(R.entry_new(i + 1, b"outer%d" % i, v).write_bytes())
    check_against_oracle(gpu_ctx, [b"".join(out)])
    cnt = gpu_ctx.last_counters()
    if not cnt["walk_mode"]:  # the walk's search may pick the true starts here
        assert cnt["repaired_chunks"] > 0 and cnt["dense_path"] == 0, cnt


def test_adversarial_repair_by_walk_only(gpu_ctx):
    """The same input with the local repair disabled: the exact boundary walk alone repairs it."""
    rng = random.Random(5)
    inner = [R.entry_new(10_000 + i, rng.randbytes(8), rng.randbytes(rng.randrange(0, 40))).write_bytes()
             for i in range(64)]
    out = [R.entry_new(i + 1, b"outer%d" % i, b"".join(rng.choice(inner) for _ in range(rng.randrange(1, 30))))
           .write_bytes() for i in range(3000)]
    os.environ["CASK_LOCAL_REPAIRS"] = "0"
    try:
        check_against_oracle(gpu_ctx, [b"".join(out)])
        cnt = gpu_ctx.last_counters()
        assert cnt["walked"] == 1 or (cnt["walk_mode"] and cnt["dense_path"]), cnt
    finally:
        del os.environ["CASK_LOCAL_REPAIRS"]


def test_all_zero_file(gpu_ctx):
    """Zero bytes parse as 18-byte records that all fail their checksum."""
    res = check_against_oracle(gpu_ctx, [bytes(300_000)])
    assert res.error.kind == 1 and res.error.pos == 0


@pytest.mark.parametrize("seed", [6, 7, 8])
def test_random_corruption(gpu_ctx, seed):
    rng = random.Random(seed)
    base = bytearray(make_records(rng, 30000, lambda r: r.randrange(4, 24), lambda r: r.randrange(0, 300)))
    for _ in range(5):
        p = rng.randrange(len(base))
        base[p] ^= 1 << rng.randrange(8)
    check_against_oracle(gpu_ctx, [bytes(base)])


@pytest.mark.parametrize("seed", [9, 10])
def test_truncation(gpu_ctx, seed):
    rng = random.Random(seed)
    base = make_records(rng, 5000, lambda r: 16, lambda r: r.randrange(0, 500))
    cut = rng.randrange(len(base) // 2, len(base))
    check_against_oracle(gpu_ctx, [base[:cut], base])


def test_engine_scan_path_large(native, tmp_path):
    """Cask::open with no hint files over a multi-file DB: GPU scan + hint recreation + fold vs
    the Python restatement of the replay."""
    from cask_amd import CaskOptions
    rng = random.Random(12)
    keys = [rng.randbytes(rng.randrange(1, 30)) for _ in range(3000)]
    ents = []
    for i in range(40000):
        k = rng.choice(keys)
        if rng.random() < 0.1:
            ents.append(R.entry_deleted(i + 1, k))
        else:
            ents.append(R.entry_new(i + 1, k, rng.randbytes(rng.randrange(0, 200))))
    path = str(tmp_path / "db")
    R.write_log(path, ents, max_file_size=1 << 20, write_hints=False)
    ref_dir = str(tmp_path / "ref")
    shutil.copytree(path, ref_dir)
    py = R.replay(ref_dir)
    with CaskOptions().open(path) as db:
        assert db.current_sequence == py.current_sequence
        assert db.stats() == {f: tuple(s) for f, s in py.index.stats.map.items()}
        got = db.index()
        assert len(got) == len(py.index.map)
        for k, v in py.index.map.items():
            e = got[k]
            assert (e.file_id, e.entry_pos, e.entry_size, e.sequence) == (v.file_id, v.entry_pos, v.entry_size,
                                                                           v.sequence)
    for fid in R.find_data_files(path):
        with open(R.hint_file_path(path, fid), "rb") as a, open(R.hint_file_path(ref_dir, fid), "rb") as b:
            assert a.read() == b.read()


# ------------------------------------------------------------------------------------ encoder
def _splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def test_encoder_matches_oracle(gpu_ctx):
    import torch
    rng = np.random.default_rng(13)
    n = 5000
    ksz = rng.integers(0, 40, n).astype(np.int16)
    vsz = rng.integers(0, 2000, n).astype(np.int64)
    vsz[rng.random(n) < 0.1] = 0xFFFFFFFF
    veff = np.where(vsz == 0xFFFFFFFF, 0, vsz)
    rl = 18 + ksz.astype(np.int64) + veff
    off = np.cumsum(rl) - rl
    seq = np.arange(n, dtype=np.int64) * 3 + 7
    kid = rng.integers(0, 1 << 40, n).astype(np.int64)
    dev = torch.device("cuda")
    out = torch.empty(int(rl.sum()), dtype=torch.uint8, device=dev)
    t = lambda a, dt: torch.from_numpy(a.astype(dt)).to(dev)
    gpu_ctx.encode_synthetic(t(off, np.int64), t(seq, np.int64), t(ksz, np.int16),
                             t(vsz.astype(np.uint32).view(np.int32), np.int32), t(kid, np.int64), 0xABCDEF, out)
    buf = out.cpu().numpy().tobytes()
    rows = O.scan(buf)
    assert len(rows) == n and (rows["status"] == 0).all()
    assert (rows["pos"] == off.astype(np.uint64)).all() and (rows["seq"] == seq.astype(np.uint64)).all()
    assert (rows["ksz"] == ksz.astype(np.uint16)).all()
    assert (rows["vsz_raw"] == vsz.astype(np.uint32)).all()
    # key bytes follow the documented generator: word i of key id k = splitmix64((k << 16) | i)
    for r in range(0, n, 97):
        k = int(ksz[r])
        want = b"".join(_splitmix64(((int(kid[r]) << 16) | i) & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")
                        for i in range((k + 7) // 8))[:k]
        assert buf[int(off[r]) + 18:int(off[r]) + 18 + k] == want


# ------------------------------------------------------------------------- full-size properties
def test_cfg2_full_size_properties(gpu_ctx):
    """BASELINE configs[1] at full size: 8 x 3,702,558 records of 290 B. Every row verifies, rows
    are exactly the encoded layout, and every file's rows (all 29.6 M, through the regular-chunk
    expansion) equal the C oracle's scan of the file row for row, all five fields."""
    import torch
    from cask_amd.workloads import CFG2_RECORDS_PER_FILE, cfg2_files
    files = cfg2_files(gpu_ctx)
    res = gpu_ctx.scan_device([(f.file_id, f.data) for f in files])
    n = CFG2_RECORDS_PER_FILE
    assert res.count == 8 * n and res.error is None
    assert int((res.status[:res.count] != 0).sum().item()) == 0
    idx = torch.arange(n, device=res.pos.device, dtype=torch.int64)
    for i, f in enumerate(files):
        sl = res.file_rows(i)
        assert sl.stop - sl.start == n
        assert torch.equal(res.pos[sl], idx * 290)
        assert torch.equal(res.seq[sl], idx + f.seq0)
    assert int((res.ksz[:res.count] != 16).sum().item()) == 0
    assert int((res.vsz[:res.count] != 256).sum().item()) == 0
    cnt = gpu_ctx.last_counters()
    assert cnt["repaired_chunks"] == 0 and cnt["dense_path"] == 1, cnt
    assert cnt["geometry"] == {"auto": 3, "wide": 0, "walk": -1}[os.environ.get("CASK_SCAN_MODE", "auto")], cnt
    # every file against the C oracle's scan of its bytes, all five row fields
    for i, f in enumerate(files):
        host = f.data.cpu().numpy()
        want = O.scan(host)
        sl = res.file_rows(i)
        m = len(want)
        assert m == n and (want["status"] == 0).all()
        assert np.array_equal(want["pos"], res.pos[sl].cpu().numpy().astype(np.uint64))
        assert np.array_equal(want["seq"], res.seq[sl].cpu().numpy().astype(np.uint64))
        assert np.array_equal(want["ksz"].astype(np.uint16), res.ksz[sl].cpu().numpy().view(np.uint16))
        assert np.array_equal(want["vsz_raw"].astype(np.uint32), res.vsz[sl].cpu().numpy().view(np.uint32))
        assert np.array_equal(want["status"].astype(np.uint8), res.status[sl].cpu().numpy())
        del host, want


def test_zipf_head_and_tail_units(gpu_ctx):
    """configs[2] record shape at 4.5 GiB in 2-GiB files: over 4,000 walk runs, so k_run_hash hands out
    whole runs first and then the last two grids' worth of runs in pieces, each piece twice (its records
    of at least 24 KiB, marked by k_walk_chase, then its shorter ones). Bit flips in the bodies of
    records all over both parts; every row of every file and the call's first error as the C oracle's
    scan of the same bytes."""
    import torch
    from cask_amd.workloads import zipf_files
    fs, _, n, rl = zipf_files(gpu_ctx, 4.5, 2 ** 31)
    rl_h = rl[:n].cpu().numpy()
    rng = np.random.default_rng(5)
    hosts = []
    for f, idx in fs:
        i0, i1 = int(idx[0]), int(idx[-1]) + 1
        off = np.concatenate([[0], np.cumsum(rl_h[i0:i1])[:-1]])
        host = f.data.cpu().numpy().copy()
        for r in rng.choice(i1 - i0, size=16, replace=False):
            b = int(off[r]) + 18 + int(rng.integers(int(rl_h[i0 + r]) - 18))
            host[b] ^= np.uint8(1 << int(rng.integers(8)))
        f.data.copy_(torch.from_numpy(host))
        hosts.append(host)
    res = gpu_ctx.scan_device([(f.file_id, f.data) for f, _ in fs])
    first_err = None
    for i, ((f, _), host) in enumerate(zip(fs, hosts)):
        want = O.scan(host)
        sl = res.file_rows(i)
        assert sl.stop - sl.start == len(want)
        assert np.array_equal(want["pos"], res.pos[sl].cpu().numpy().astype(np.uint64))
        assert np.array_equal(want["seq"], res.seq[sl].cpu().numpy().astype(np.uint64))
        assert np.array_equal(want["ksz"].astype(np.uint16), res.ksz[sl].cpu().numpy().view(np.uint16))
        assert np.array_equal(want["vsz_raw"].astype(np.uint32), res.vsz[sl].cpu().numpy().view(np.uint32))
        assert np.array_equal(want["status"].astype(np.uint8), res.status[sl].cpu().numpy())
        assert int((want["status"] != 0).sum()) == 16
        if first_err is None:
            r = want[np.flatnonzero(want["status"] != 0)[0]]
            first_err = (int(r["status"]), f.file_id, int(r["pos"]), int(r["expected"]), int(r["found"]))
    e = res.error
    assert (e.kind, e.file_id, e.pos, e.expected, e.found) == first_err

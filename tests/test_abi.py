"""The C-ABI library on the CPU: it loads, exports every symbol include/cask_scan.h declares, and the
host-side parts of the engine that never touch the GPU (hint fast path, fold, stats, path/lock/
file-discovery semantics) match the reference restatement. No compute call needs a GPU here."""
import json
import os
import re
import shutil
import struct

import pytest

from conftest import GOLDEN, ROOT

import cask_ref as R


def header_functions():
    with open(os.path.join(ROOT, "include", "cask_scan.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(cask_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_exports_every_declared_symbol(native):
    import cask_amd._lib as L
    declared = header_functions()
    assert len(declared) >= 20
    bound = {n for n, _, _ in L.SIGNATURES}
    assert set(declared) == bound, set(declared) ^ bound
    for name in declared:
        assert hasattr(native, name), name


def test_stream_ceiling_utility_loads():
    """bench.py's read-only stream ceiling (cask_amd/libcask_stream.so, built by build()): it loads,
    exports its one entry point and rejects bad arguments before touching a device."""
    import ctypes as C
    p = os.path.join(ROOT, "cask_amd", "libcask_stream.so")
    if not os.path.exists(p):
        pytest.skip("libcask_stream.so not built")
    lib = C.CDLL(p)
    fn = lib.cask_stream_read
    fn.restype = C.c_int
    g = C.c_double()
    assert fn(None, None, 0, 1, 0, 0, C.byref(g), None) != 0
    bufs, lens = (C.c_void_p * 1)(), (C.c_uint64 * 1)(16)
    assert fn(bufs, lens, 65, 1, 0, 0, C.byref(g), None) != 0  # more buffers than it takes
    assert fn(bufs, lens, 1, 0, 0, 0, C.byref(g), None) != 0   # no passes


def test_host_xxh32_kat(native):
    import cask_amd
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        kat = json.load(f)
    for spec, want in kat["xxh32"]:
        data = bytes((i * 7 + 3) & 0xFF for i in range(int(spec.split(":")[1]))) if spec.startswith("pattern:") \
            else bytes.fromhex(spec)
        assert cask_amd.xxh32(data) == want


def test_defaults(native):
    import ctypes as C
    import cask_amd._lib as L
    o = L.Options()
    native.cask_options_default(C.byref(o))
    assert o.create == 1 and o.write_hints == 1 and o.max_file_size == 2 * 1024 ** 3  # cask.rs:223-225
    assert native.cask_scan_chunk_bytes() == 32768
    fv = (L.FileView * 2)()
    fv[0].len, fv[1].len = 18 * 10, 17
    assert native.cask_rows_bound(fv, 2) == 11 + 1


def test_no_gpu_means_loud_failure(native):
    """The product path has no CPU fallback: a scan without a GPU raises."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from cask_amd import ScanContext, errors
    with pytest.raises(errors.DeviceError):
        ScanContext(0)


def _copy_case(case, tmp_path):
    d = tmp_path / case
    shutil.copytree(os.path.join(GOLDEN, case), d)
    os.remove(d / "expected.json")
    return str(d)


def test_engine_hint_path_matches_fixture(native, tmp_path):
    """hints_valid: every file has a valid hint file, so Cask::open never scans (log.rs:357-362)."""
    from cask_amd import CaskOptions
    with open(os.path.join(GOLDEN, "hints_valid", "expected.json")) as f:
        rep = json.load(f)["replay"]
    path = _copy_case("hints_valid", tmp_path)
    with CaskOptions().open(path) as db:
        got = sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence] for k, e in db.index().items())
        assert got == rep["keydir"]
        assert sorted([f, *s] for f, s in db.stats().items()) == rep["stats"]
        assert db.current_sequence == rep["current_sequence"]
        assert db.files() == R.find_data_files(path)
        assert db.keys() == sorted(bytes.fromhex(k[0]) for k in rep["keydir"])


def _write_db_with_hints(path, groups):
    """groups: list of entry lists, one data file each, all with valid hint files."""
    os.makedirs(path, exist_ok=True)
    fid = 0
    for ents in groups:
        fid += 1
        R.write_log(path + f"/_tmp{fid}", ents, 1 << 30, first_file_id=fid)
        for ext in ("cask.data", "cask.hint"):
            shutil.move(path + f"/_tmp{fid}/{fid:010}.{ext}", path + f"/{fid:010}.{ext}")
        shutil.rmtree(path + f"/_tmp{fid}")


def test_engine_fold_edge_cases_via_hints(native, tmp_path):
    """Index::update semantics (cask.rs:60-90) through the hint path: stale tombstone, resurrection,
    equal-sequence duplicates across files, tombstone of an absent key."""
    from cask_amd import CaskOptions
    K = b"key-A"
    groups = [
        [R.entry_new(10, K, b"v10"), R.entry_new(5, b"B", b"v5")],
        [R.entry_deleted(3, K), R.entry_deleted(7, b"B"), R.entry_deleted(99, b"nobody")],
        [R.entry_new(6, b"B", b"v6"), R.entry_new(10, K, b"v10-copy"), R.entry_new(8, b"C", b"x")],
        [R.entry_new(8, b"C", b"y"), R.entry_deleted(8, b"C")],
    ]
    path = str(tmp_path / "db")
    _write_db_with_hints(path, groups)
    py = R.replay(path, write_hints=False)
    with CaskOptions().open(path) as db:
        assert sorted([k.hex(), e.file_id, e.entry_pos, e.entry_size, e.sequence] for k, e in db.index().items()) == \
            sorted([k.hex(), v.file_id, v.entry_pos, v.entry_size, v.sequence] for k, v in py.index.map.items())
        assert db.stats() == {f: tuple(s) for f, s in py.index.stats.map.items()}
        assert db.current_sequence == py.current_sequence


def test_open_removes_files_a_compaction_left_behind(native, tmp_path):
    """A compaction renames the compacted files to `*.cask.data.gone` / `*.cask.hint.gone` and
    unlinks them on the db's reclaim thread; if the process ends first they stay on disk. The next
    open removes them (holding the lock), and they never count as data files (log.rs:483-510)."""
    from cask_amd import CaskOptions
    path = str(tmp_path / "db")
    _write_db_with_hints(path, [[R.entry_new(1, b"k", b"v")]])
    left = [path + "/0000000007.cask.data.gone", path + "/0000000007.cask.hint.gone"]
    for f in left:
        with open(f, "wb") as fh:
            fh.write(b"x" * 4096)
    with CaskOptions().open(path) as db:
        assert db.current_sequence == 2 and len(db) == 1
    assert not any(os.path.exists(f) for f in left)
    assert sorted(os.listdir(path)) == ["0000000001.cask.data", "0000000001.cask.hint", "cask.lock"]


def test_engine_truncated_hint_body_is_eof(native, tmp_path):
    """A hint file whose trailer is valid but whose last hint is cut short: Hint::from_read fails
    with UnexpectedEof and open() returns it (data.rs:258-265, cask.rs:360)."""
    from cask_amd import CaskOptions, errors
    path = str(tmp_path / "db")
    _write_db_with_hints(path, [[R.entry_new(1, b"k1", b"v"), R.entry_new(2, b"k2", b"v")]])
    hp = R.hint_file_path(path, 1)
    with open(hp, "rb") as f:
        body = f.read()[:-4]
    body = body[:-1]  # cut the last key byte
    with open(hp, "wb") as f:
        f.write(body + struct.pack("<I", R.xxhash32(body)))
    with pytest.raises(errors.UnexpectedEof):
        CaskOptions().open(path)


def test_engine_paths_and_lock(native, tmp_path):
    from cask_amd import CaskOptions, errors
    missing = str(tmp_path / "missing")
    with pytest.raises(errors.InvalidPath):  # log.rs:52-55
        CaskOptions().create(False).open(missing)
    afile = tmp_path / "afile"
    afile.write_bytes(b"x")
    with pytest.raises(errors.InvalidPath):  # log.rs:47-48
        CaskOptions().open(str(afile))
    db = CaskOptions().open(missing)  # create=true makes the directory (log.rs:49-50)
    assert os.path.isdir(missing) and os.path.exists(os.path.join(missing, "cask.lock"))
    assert len(db) == 0 and db.current_sequence == 1  # empty DB: sequence 0 + 1 (cask.rs:379)
    with pytest.raises(errors.Locked):  # try_lock_exclusive (log.rs:59)
        CaskOptions().open(missing)
    db.close()
    CaskOptions().open(missing).close()


def test_engine_file_discovery(native, tmp_path):
    """find_data_files (log.rs:483-510): regex (\\d+).cask.data$ unanchored with unescaped dots,
    regular files only, u32 parse (overflow skipped), ascending order."""
    from cask_amd import CaskOptions
    path = tmp_path / "db"
    path.mkdir()
    empty_hint = struct.pack("<I", R.xxhash32(b""))
    names = ["0000000003.cask.data", "12.cask.data", "x7ycask.data", "5xcaskydata",
             "0000000009.cask.data.bak", "99999999999.cask.data", "4.CASK.data"]
    for n in names:
        (path / n).write_bytes(b"")
    (path / "6.cask.data").mkdir()
    os.symlink(str(path / "12.cask.data"), str(path / "13.cask.data"))
    want = R.find_data_files(str(path))
    assert want == [3, 5, 7, 12]
    for fid in want:
        (path / f"{fid:010}.cask.hint").write_bytes(empty_hint)
    with CaskOptions().open(str(path)) as db:
        assert db.files() == want
        assert len(db) == 0


_LIMIT_CHILD = r"""
import ctypes as C, resource, sys
sys.path.insert(0, sys.argv[3])
import cask_amd._lib as L
lib = L.lib()
vm = int([l for l in open("/proc/self/status") if l.startswith("VmSize")][0].split()[1]) * 1024
lim = vm + (int(sys.argv[2]) << 20)
resource.setrlimit(resource.RLIMIT_AS, (lim, lim))
err = L.OpenError()
h = lib.cask_db_open(sys.argv[1].encode(), None, C.byref(err))
print("RESULT", 1 if h else 0, err.status, flush=True)
"""


def test_open_out_of_memory_returns_status(native, tmp_path):
    """No C++ exception crosses the C ABI (cask_scan.h): open() of a database whose hint file is
    larger than the memory the process has left (RLIMIT_AS in a child process) returns
    CASK_E_NOMEM — the std::bad_alloc of the hint read, on a worker thread, reaches the entry
    point's handler — instead of terminating the process."""
    import subprocess
    import sys
    import numpy as np
    path = str(tmp_path / "db")
    os.makedirs(path)
    open(R.data_file_path(path, 1), "wb").close()
    n = 3 << 20  # 3 Mi hint records of 38 B: a 114-MB hint file
    rec = np.zeros((n, 38), np.uint8)
    rec[:, 0:8] = np.arange(1, n + 1, dtype="<u8").view(np.uint8).reshape(n, 8)
    rec[:, 8] = 16  # ksz
    rec[:, 22:30] = np.arange(n, dtype="<u8").view(np.uint8).reshape(n, 8)  # keys
    body = rec.tobytes()
    with open(R.hint_file_path(path, 1), "wb") as f:
        f.write(body + R.xxhash32(body).to_bytes(4, "little"))
    out = subprocess.run([sys.executable, "-c", _LIMIT_CHILD, path, "64", ROOT], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    res = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
    assert res == ["RESULT 0 -13"], (out.stdout, out.stderr[-2000:])
    # and with the memory it needs, the same database opens
    out = subprocess.run([sys.executable, "-c", _LIMIT_CHILD, path, "4096", ROOT], capture_output=True, text=True,
                         timeout=300)
    assert [l for l in out.stdout.splitlines() if l.startswith("RESULT")] == ["RESULT 1 0"], out.stderr[-2000:]

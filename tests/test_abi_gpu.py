"""The C ABI's error contract on the GPU (include/cask_scan.h: no C++ exception crosses it; every
entry point returns a cask_status). Needs an MI355X.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from test_shard_gpu import _files, _make_db

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INJ_THROW = 8

_HOST_SCAN_CHILD = r"""
import ctypes as C, resource, sys
sys.path.insert(0, sys.argv[2])
import cask_amd._lib as L
lib = L.lib()
st = C.c_int()
ctx = lib.cask_ctx_create(0, C.byref(st))
assert ctx, st.value
n = int(sys.argv[3])  # views of empty files: the library's per-file host tables are 8-32 B each
views = (L.FileView * n)()
for v in (views[0], views[n - 1]):
    v.file_id = 1
cap = n + 16
rows = L.Rows()
arrs = [(C.c_uint64 * cap)(), (C.c_uint64 * cap)(), (C.c_uint32 * cap)(), (C.c_uint16 * cap)(), (C.c_uint8 * cap)()]
rows.capacity = cap
rows.pos, rows.seq, rows.vsz, rows.ksz, rows.status = [C.addressof(a) for a in arrs]
off = (C.c_uint64 * (n + 1))()
err = L.ScanError()
small = (L.FileView * 1)()
assert lib.cask_scan_host(ctx, small, 1, C.byref(rows), off, C.byref(err)) == 0  # warm: the device is up
vm = int([l for l in open("/proc/self/status") if l.startswith("VmSize")][0].split()[1]) * 1024
lim = vm + (int(sys.argv[1]) << 20)
resource.setrlimit(resource.RLIMIT_AS, (lim, lim))
rc = lib.cask_scan_host(ctx, views, n, C.byref(rows), off, C.byref(err))
rc2 = lib.cask_scan_host(ctx, small, 1, C.byref(rows), off, C.byref(err))  # the context still works
print("RESULT", rc, rc2, flush=True)
"""


def test_scan_host_out_of_memory_returns_status(native):
    """cask_scan_host over more files than the process has memory left for (RLIMIT_AS lowered in a
    child process once the device is initialised): the std::bad_alloc of the host-side file tables
    comes back as CASK_E_NOMEM instead of terminating the process, and the context scans again
    afterwards."""
    out = subprocess.run([sys.executable, "-c", _HOST_SCAN_CHILD, "8", ROOT, str(1 << 20)], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert [l for l in out.stdout.splitlines() if l.startswith("RESULT")] == ["RESULT -13 0"], out.stdout


def test_exception_in_entry_point_returns_nomem(gpu_ctx, tmp_path):
    """No C++ exception crosses the C ABI (cask_scan.h): a std::bad_alloc thrown inside each
    context entry point (the cask_debug_inject hook) comes back as CASK_E_NOMEM, and the context
    works afterwards."""
    import torch
    import cask_amd
    lib = cask_amd.lib()
    path = str(tmp_path / "db")
    _make_db(path, 80, nfiles=2)
    files = _files(path)
    tens = [(fid, torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()) for fid, b in files]
    from cask_amd.errors import DeviceError
    for call in (lambda: gpu_ctx.scan_device(tens),
                 lambda: gpu_ctx.scan_host([(fid, np.frombuffer(b, np.uint8)) for fid, b in files])):
        assert lib.cask_debug_inject(gpu_ctx._h, INJ_THROW) == 0
        with pytest.raises(DeviceError, match=r"\(-13\)"):  # CASK_E_NOMEM
            call()
        res = call()  # the hook is taken: the same call now succeeds
        assert res.error is None and res.count > 0

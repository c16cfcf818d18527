"""The hint-file parse on the device (cask_parse_hints_device: Hints::next / Hint::from_read,
log.rs:437-447, data.rs:258-276) against the restatement's walk of the same bodies (hint_offsets):
every record's offset, sequence, key size, raw value size and status, and the first failure."""
import os
import random

import numpy as np
import pytest

from conftest import GOLDEN, golden_cases

import cask_ref as R

pytestmark = pytest.mark.gpu


def _check(ctx, bodies):
    import torch
    files = [(i + 1, torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda() if b else
              torch.empty(0, dtype=torch.uint8, device="cuda")) for i, b in enumerate(bodies)]
    res = ctx.parse_hints_device(files)
    got_all = [t[:res.count].cpu().numpy() for t in (res.pos, res.seq, res.ksz, res.vsz, res.status)]
    first = None
    total = 0
    for i, b in enumerate(bodies):
        want = R.hint_offsets(b)
        sl = res.file_rows(i)
        got = [(int(got_all[0][r]), int(got_all[1][r]) & 0xFFFFFFFFFFFFFFFF, int(got_all[2][r]) & 0xFFFF,
                int(got_all[3][r]) & 0xFFFFFFFF, int(got_all[4][r])) for r in range(sl.start, sl.stop)]
        assert got == want, (i, next((j, g, w) for j, (g, w) in enumerate(zip(got, want)) if g != w)
                             if len(got) == len(want) else (len(got), len(want)))
        total += len(want)
        if first is None and want and want[-1][4] != R.ROW_OK:
            first = (R.ROW_EOF, i + 1, want[-1][0])
    assert res.count == total
    if first is None:
        assert res.error is None
    else:
        e = res.error
        assert (e.kind, e.file_id, e.pos, e.expected, e.found) == (*first, 0, 0)
    return res


def _bodies_of(path):
    out = []
    for f in R.find_data_files(path):
        hp = R.hint_file_path(path, f)
        if os.path.exists(hp):
            out.append(open(hp, "rb").read()[:-4])
    return out


def test_golden_hint_bodies(gpu_ctx):
    bodies = []
    for case in golden_cases():
        bodies += _bodies_of(os.path.join(GOLDEN, case))
    assert len(bodies) >= 5
    _check(gpu_ctx, bodies)


def _entries(rng, n, kmax=40, vmax=400, del_p=0.15, big_key_p=0.0):
    ents = []
    for i in range(n):
        k = rng.randbytes(60000 if rng.random() < big_key_p else rng.randrange(0, kmax))
        if rng.random() < del_p:
            ents.append(R.entry_deleted(i + 1, k))
        else:
            ents.append(R.entry_new(i + 1, k, rng.randbytes(rng.randrange(0, vmax))))
    return ents


@pytest.mark.parametrize("seed,kmax,mfs", [(1, 16, 1 << 20), (2, 40, 64 << 10), (3, 200, 1 << 22), (4, 1, 8 << 10)])
def test_written_hint_bodies(gpu_ctx, tmp_path, seed, kmax, mfs):
    """Hint files as the writer leaves them, many records per chunk of body."""
    rng = random.Random(seed)
    path = str(tmp_path / "db")
    R.write_log(path, _entries(rng, 40000, kmax=kmax), max_file_size=mfs)
    _check(gpu_ctx, _bodies_of(path))


def test_gaps_long_keys_truncation_empty(gpu_ctx, tmp_path):
    """Bodies with hints missing (RecreateHints skips corrupt records: the entry positions jump),
    60,000-byte keys (longer than the search window: the repair path), cut short mid-record, and
    empty."""
    rng = random.Random(7)
    path = str(tmp_path / "db")
    R.write_log(path, _entries(rng, 12000, big_key_p=0.002), max_file_size=1 << 30)
    body = _bodies_of(path)[0]
    recs = R.hint_offsets(body)
    spans = [(p, (recs[i + 1][0] if i + 1 < len(recs) else len(body))) for i, (p, *_r) in enumerate(recs)]
    gappy = b"".join(body[a:b] for i, (a, b) in enumerate(spans) if i % 7 != 3)
    cut = body[: len(body) - 5]
    cut2 = body[: spans[len(spans) // 2][0] + 10]
    _check(gpu_ctx, [body, gappy, b"", cut, cut2, body[:21]])


def test_many_small_bodies(gpu_ctx, tmp_path):
    rng = random.Random(8)
    path = str(tmp_path / "db")
    R.write_log(path, _entries(rng, 6000), max_file_size=4 << 10)
    bodies = _bodies_of(path)
    assert len(bodies) > 100
    _check(gpu_ctx, bodies)

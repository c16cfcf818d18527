"""Synthetic Cask data files for the BASELINE.json configs, generated on the GPU.

Records are laid out exactly as LogWriter would write them (log.rs:282-306: a new file when
pos + size > max_file_size) and encoded by the batched Entry::write_bytes kernel
(cask_encode_synthetic_device). Key/value bytes come from the splitmix64 generator documented in
DESIGN.md §Synthetic data (no datasets are available offline).
"""
from __future__ import annotations

from dataclasses import dataclass

from .scan import ScanContext

CFG2_RECORDS_PER_FILE = 3_702_558      # floor(2^30 / 290)
CFG2_FILES = 8
CFG2_KSZ, CFG2_VSZ = 16, 256


@dataclass
class DataFile:
    file_id: int
    data: object          # torch uint8 CUDA tensor, exactly the file bytes
    nrec: int
    seq0: int             # first sequence number in the file


def _torch():
    import torch
    return torch


def fixed_file(ctx: ScanContext, file_id: int, nrec: int, ksz: int, vsz: int, seq0: int, key_id0: int,
               value_seed: int, device=None) -> DataFile:
    """One data file of `nrec` fixed-size records: seq = seq0.., key ids = key_id0.. (unique)."""
    torch = _torch()
    dev = device or torch.device("cuda", ctx.device)
    rl = 18 + ksz + vsz
    out = torch.empty(nrec * rl, dtype=torch.uint8, device=dev)
    idx = torch.arange(nrec, dtype=torch.int64, device=dev)
    off = idx * rl
    seq = idx + seq0
    ks = torch.full((nrec,), ksz, dtype=torch.int16, device=dev)
    vs = torch.full((nrec,), vsz, dtype=torch.int32, device=dev)
    kid = idx + key_id0
    ctx.encode_synthetic(off, seq, ks, vs, kid, value_seed, out)
    del off, seq, ks, vs, kid, idx
    return DataFile(file_id, out, nrec, seq0)


def cfg2_files(ctx: ScanContext, nfiles: int = CFG2_FILES, records_per_file: int = CFG2_RECORDS_PER_FILE,
               first_file_id: int = 1, seed: int = 0xC0FFEE) -> list[DataFile]:
    """BASELINE configs[1]: 8 GiB across 8 data files, 16 B keys / 256 B values, unique keys."""
    files = []
    for i in range(nfiles):
        fid = first_file_id + i
        seq0 = 1 + (fid - 1) * records_per_file
        files.append(fixed_file(ctx, fid, records_per_file, CFG2_KSZ, CFG2_VSZ, seq0, seq0, seed + fid))
    return files


def variable_file(ctx: ScanContext, file_id: int, ksz, vsz_raw, seq, key_id, value_seed: int) -> DataFile:
    """One data file from per-record size/sequence/key tensors (device, int16/int32/int64/int64)."""
    torch = _torch()
    veff = torch.where(vsz_raw == -1, torch.zeros_like(vsz_raw), vsz_raw).to(torch.int64)
    rl = 18 + ksz.to(torch.int64) + veff
    off = torch.cumsum(rl, 0) - rl
    total = int(rl.sum().item()) if rl.numel() else 0
    out = torch.empty(total, dtype=torch.uint8, device=ksz.device)
    if rl.numel():
        ctx.encode_synthetic(off, seq, ksz, vsz_raw, key_id, value_seed, out)
    return DataFile(file_id, out, int(rl.numel()), int(seq[0].item()) if seq.numel() else 0)


def zipf_sizes(n: int, s: float = 1.1, kmax: int = 4096, seed: int = 0x5A1F, device=None):
    """vsz = 16·k, k ~ Zipf(s) truncated to [1, kmax] (BASELINE configs[2])."""
    torch = _torch()
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    k = torch.arange(1, kmax + 1, dtype=torch.float64, device=device)
    pmf = k.pow(-s)
    cdf = torch.cumsum(pmf / pmf.sum(), 0)
    u = torch.rand(n, generator=g, dtype=torch.float64, device=device)
    kk = torch.searchsorted(cdf, u).clamp_(max=kmax - 1) + 1
    return (kk * 16).to(torch.int32)


def zipf_files(ctx: ScanContext, total_gib: float = 32.0, max_file: int = 2 ** 31, seed: int = 0x5A1F,
               first_file_id: int = 1, first_seq: int = 1, first_key: int = 0):
    """BASELINE configs[2]: ~total_gib GiB of records with 16 B keys and Zipf(1.1) value sizes
    (16 B .. 64 KiB), sequences first_seq.., key ids first_key.. (unique), in files rolled over as
    LogWriter does (a new file when pos + size > max_file_size, log.rs:282-306), file ids
    first_file_id... Returns ([(DataFile, record indices)], vsz, n, record lengths) — the
    generator's own view, for checking rows (record i has sequence first_seq + i)."""
    torch = _torch()
    dev = torch.device("cuda", ctx.device)
    target = int(total_gib * 2 ** 30)
    n = int(target / (34 + 5085) * 1.05) + 1024
    vsz = zipf_sizes(n, seed=seed, device=dev)
    rl = 34 + vsz.to(torch.int64)
    cum = torch.cumsum(rl, 0)
    n = int(torch.searchsorted(cum, torch.tensor([target], device=dev, dtype=torch.int64)).item())
    files, base, r0 = [], 0, 0
    while r0 < n:  # greedy rollover: a new file when pos + size > max_file_size
        r1 = int(torch.searchsorted(cum, torch.tensor([base + max_file], device=dev, dtype=torch.int64),
                                    right=True).item())
        r1 = min(max(r1, r0 + 1), n)
        idx = torch.arange(r0, r1, dtype=torch.int64, device=dev)
        ks = torch.full((r1 - r0,), 16, dtype=torch.int16, device=dev)
        f = variable_file(ctx, first_file_id + len(files), ks, vsz[r0:r1].clone(), idx + first_seq,
                          idx + first_key, seed + len(files))
        files.append((f, idx))
        base = int(cum[r1 - 1].item())
        r0 = r1
    del cum
    torch.cuda.synchronize(dev)
    return files, vsz, n, rl

#!/usr/bin/env python3
"""Headline benchmark: device-resident Cask data-file scan (decode + XXH32 verify + row emit).

Metric (BASELINE.json): GiB/s of log bytes checksum-verified + decoded, device-resident. A step is
one pass of the scan (cask_scan_device: Entries::next + Entry::from_read, log.rs:403-429,
data.rs:161-206) over one batch of data files already resident in HBM.

  N = 1   BASELINE configs[2], the largest single-GPU configuration: 32 GiB of records with 16-B
          keys and Zipf(1.1) value sizes 16 B .. 64 KiB, rolled over into files of at most 2 GiB
          (the reference's default max_file_size, cask.rs:225; LogWriter rollover, log.rs:282-306).
  N > 1   BASELINE configs[4]: 256 GiB across 256 data files over 8 GPUs, i.e. one shard of
          32 x 1 GiB files per rank (the same record distribution as configs[2], so per-GPU work is
          the same at every N: weak scaling). Data files shard with no collective; after the timed
          loop each rank reduces its rows to a keydir block and the blocks meet on rank 0 over RCCL
          through the library's C ABI (cask_keydir_gather_rccl), timed separately.

Rank 0 prints one JSON line with the roofline of the dominant kernel (k_run_hash on these shapes,
HIP events inside the library on the stream it launches on) and, at N = 1, the CPU baseline (the
oracle's reference-faithful replay of a bounded sample of the same files, timed on this host).
Secondary numbers (configs[1], host-resident end to end) go in extra keys, never in `value`.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...      (driver, N>1)

Every CASK_* variable in the environment is printed in the line; the library's tuning knobs are
refused unless --allow-tuning is given (never for a headline).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md (8.0 TB/s spec)
CFG2_GIB, CFG2_MAX_FILE = 32.0, 2 ** 31
CFG4_FILES_PER_RANK, CFG4_FILE = 32, 2 ** 30
CFG2_MAX_RECORD = 18 + 16 + 16 * 4096  # the longest configs[2] record (16-B key, value of 16 x 4,096 B)
SEQ_STRIDE = 1 << 40  # a rank's first sequence / key id (ranks' ranges disjoint and in rank order)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (a step is ~8 ms: 50 steps keep host hiccups out of the number and still take 0.4 s)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-files", type=int, default=2, help="configs[2] files timed by the CPU baseline")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-resident (H2D+D2H) measurement")
    ap.add_argument("--no-cfg1", action="store_true", help="skip the secondary configs[1] measurement")
    ap.add_argument("--no-cold", action="store_true",
                    help="skip cold_call_ms (its calls over one file are small launches of the same kernels: "
                         "a profiled run without them has per-kernel averages over the full-size steps only)")
    ap.add_argument("--no-shard-n1", action="store_true",
                    help="N=1: skip configs4_shard_n1 (the N>1 lines' per-GPU shard timed on one GPU)")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the keydir gather + fold after the loop")
    ap.add_argument("--no-cfg5", action="store_true",
                    help="N>1: skip the cfg5 shard (290-B records) scan + key-hash partitioned keydir")
    ap.add_argument("--dist-backend", default="nccl",
                    help="rehearsal only: gloo (blocks gathered through host memory)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on cuda:0 (a one-GPU box)")
    ap.add_argument("--secondary-timeout", type=float, default=300.0,
                    help="N>1: seconds the multi-rank secondary measurements may take after the timed loop "
                         "before rank 0 prints the line without them (a stalled collective cannot hide the metric)")
    ap.add_argument("--allow-tuning", action="store_true",
                    help="run with CASK_* tuning variables set (diagnostics; the line says so)")
    return ap.parse_args()


def cask_env(allow: bool) -> dict:
    env = {k: v for k, v in sorted(os.environ.items()) if k.startswith("CASK_")}
    if env and not allow:
        raise SystemExit(f"bench.py: refusing to time with library tuning variables set: {env} "
                         f"(unset them, or pass --allow-tuning for a diagnostic run)")
    return env


def cpu_baseline(files, nfiles: int, cfg: str):
    """The oracle's reference-faithful replay (read(2) per header/key/value, 5 write(2) per hint,
    Index::update fold; 1 thread as in cask.rs:348) over `nfiles` of the workload's files, written
    to memory-backed files first (the page cache of a real replay)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi as O
    O.load()
    tmp = tempfile.mkdtemp(prefix="cask_cpu_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    paths = []
    total = 0
    try:
        for f in files[:nfiles]:
            p = os.path.join(tmp, f"{f.file_id:010}.cask.data")
            f.data.cpu().numpy().tofile(p)
            paths.append((f.file_id, p))
            total += f.data.numel()
        ix = O.Index()
        t0 = time.perf_counter()
        recs = 0
        for fid, p in paths:
            r = O.replay_faithful(p, p.replace(".cask.data", ".cask.hint"), fid, ix)
            assert r.err_kind == 0, r.err_kind
            recs += r.records
        dt = time.perf_counter() - t0
        # fast restatement (context only, BASELINE.md's "fast CPU scan" row): a tight in-memory loop
        # over the first file on 1 core, and the oracle's threaded replay (scan + XXH32 on threads by
        # file piece, keydir folded on threads by key partition) over the same sample on the host
        # cores this process may use (at most 16: the box's CPU share per GPU)
        buf = np.fromfile(paths[0][1], dtype=np.uint8)
        ix2 = O.Index()
        t1 = time.perf_counter()
        O.replay_fast(buf, paths[0][0], ix2)
        dt_fast = time.perf_counter() - t1
        del ix, ix2, buf
        # N cores: the sample cut at record boundaries into one independent data file per thread (a
        # file's records are a chain walked in order, cask.rs:348 / log.rs:403-429: one thread per
        # file, as the GPU path gives one lane per run), each piece with its own file id
        ncores = max(1, min(16, len(os.sched_getaffinity(0))))
        per = -(-ncores // len(paths))
        hosts, hids = [], []
        for fid, p in paths:
            b = np.fromfile(p, dtype=np.uint8)
            starts = O.scan(b)["pos"].astype(np.int64)
            cuts = [0] + [int(starts[np.searchsorted(starts, b.size * k // per)]) for k in range(1, per)] + [b.size]
            for k in range(per):
                if cuts[k + 1] > cuts[k]:
                    hosts.append(b[cuts[k]:cuts[k + 1]])
                    hids.append(len(hids) + 1)
        t2 = time.perf_counter()
        pr, _ = O.replay_parallel(hosts, hids, ncores)
        dt_par = time.perf_counter() - t2
        assert pr.err_kind == 0 and pr.records == recs, (pr.err_kind, pr.records, recs)
        npieces = len(hosts)
        del hosts
    finally:
        for name in os.listdir(tmp):
            os.remove(os.path.join(tmp, name))
        os.rmdir(tmp)
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": total / dt / 2 ** 30, "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"{nfiles} of the {len(files)} {cfg} files ({total} B, {recs} records) in memory-backed "
                  f"files (warm page cache); oracle/cask_oracle.c orc_replay_file_faithful = Cask::open's scan "
                  f"path without hint files (3 read(2) + 5 write(2) + fold per record)",
        "seconds": dt, "host_cpu": cpu, "nproc": os.cpu_count(),
        "fast_restatement_gibps_1core": files[0].data.numel() / dt_fast / 2 ** 30,
        "fast_restatement_gibps_Ncores": total / dt_par / 2 ** 30, "fast_restatement_cores": ncores,
        "fast_restatement_Ncores_sample": (f"the same {total} B cut at record boundaries into {npieces} data "
                                           f"files, replayed on {ncores} threads (the box's CPU share per GPU; "
                                           f"nproc {os.cpu_count()} is not this process's to use)"),
    }


def stream_ceiling(torch, dev, views, passes: int = 5):
    """The measured read-only stream ceiling over the same resident files:
    cask_amd/libcask_stream.so reads every byte once per pass (plain and nontemporal loads, the
    better of the two), HIP events around `passes` launches. None when the utility is not built."""
    p = os.path.join(ROOT, "cask_amd", "libcask_stream.so")
    if not os.path.exists(p):
        return None
    lib = C.CDLL(p)
    fn = lib.cask_stream_read
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_uint64), C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                   C.POINTER(C.c_double), C.POINTER(C.c_double)]
    n = len(views)
    bufs = (C.c_void_p * n)(*[t.data_ptr() for _, t in views])
    lens = (C.c_uint64 * n)(*[t.numel() for _, t in views])
    torch.cuda.synchronize(dev)
    out = {}
    for nt in (0, 1):
        g, ms = C.c_double(), C.c_double()
        rc = fn(bufs, lens, n, passes, nt, dev.index, C.byref(g), C.byref(ms))
        if rc != 0:
            return {"error": f"cask_stream_read: HIP error {rc}"}
        out["nontemporal" if nt else "plain"] = {"gbps": g.value, "ms_per_pass": ms.value}
    best = max(v["gbps"] for v in out.values())
    return {"gbps": best, "frac_of_8TBps": best / HBM_PEAK_GBPS, "bytes_per_pass": int(sum(lens)),
            "passes": passes, "kernel": "k_stream_read (cask_amd/csrc/stream_ceiling.hip)", **out}


def load_traffic(kernel: str):
    """Per-launch HBM bytes of `kernel` from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py); null when absent."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    k = d.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return k.get("hbm_bytes_per_launch"), k.get("source")


def check_rows(torch, rows, res, files, vsz, rl, first_seq):
    """Parity gate before timing: every record found, in order, at its offset, with its sequence,
    sizes and a passing checksum (the generator's own view of the files)."""
    n = res.count
    dev = rows["seq"].device
    assert res.error is None
    assert int((rows["status"][:n] != 0).sum().item()) == 0
    seq = rows["seq"][:n].to(torch.int64)
    assert bool((seq == torch.arange(first_seq, first_seq + n, device=dev)).all())
    assert bool((rows["vsz"][:n].to(torch.int64) == vsz[:n].to(torch.int64)).all())
    assert bool((rows["ksz"][:n].to(torch.int64) == 16).all())
    for i, (_, idx) in enumerate(files):
        rlf = rl[idx]
        want = torch.cumsum(rlf, 0) - rlf
        assert bool((rows["pos"][res.file_row_offset[i]:res.file_row_offset[i + 1]].to(torch.int64) == want).all()), i


def time_loop(torch, dev, run, timings, steps, barrier, dist, backend):
    tbuf = [(C.c_float * 8)() for _ in range(steps)]
    barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        run()
        timings(tbuf[i])
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    return elapsed, [[float(x) for x in t] for t in tbuf]


def secondary(extra: dict, key: str, fn):
    """A measurement reported beside the metric: its result goes to extra[key]; an exception does not
    end the run — it is reported as extra[key + "_error"] and the caller goes on (restoring whatever
    it dropped for the measurement's memory) to print the line."""
    try:
        extra[key] = fn()
        return True
    except Exception as e:  # noqa: BLE001 - reported in the line
        extra[key + "_error"] = f"{type(e).__name__}: {e}"[:300]
        return False


def cfg1_secondary(ctx, torch, dev, steps):
    """configs[1] (8 x 1 GiB of fixed 290-B records): the regular-chunk path, for reference."""
    from cask_amd.workloads import cfg2_files
    fs = cfg2_files(ctx)
    torch.cuda.synchronize(dev)
    views = [(f.file_id, f.data) for f in fs]
    n = sum(f.nrec for f in fs)
    rows = ctx.alloc_rows(n)
    res = ctx.scan_device(views, rows)
    assert res.count == n and res.error is None
    assert int((rows["status"][:n] != 0).sum().item()) == 0
    run, timings = ctx.prepare_scan(views, rows)
    for _ in range(3):
        run()
    el, tt = time_loop(torch, dev, run, timings, steps, lambda: torch.cuda.synchronize(dev), None, "nccl")
    nb = sum(f.data.numel() for f in fs)
    k = sum(t[1] for t in tt) / len(tt)
    out = {"gibps": nb * steps / el / 2 ** 30, "ms_per_step": el * 1e3 / steps, "kernel": "k_scan_chunks",
           "kernel_ms_avg": k, "kernel_frac_of_8TBps": nb / (k * 1e-3) / 1e9 / HBM_PEAK_GBPS, "bytes": nb}
    del fs, views, rows
    torch.cuda.empty_cache()
    return out


def cfg4_shard_n1_secondary(ctx, torch, dev, steps):
    """N = 1, reported beside the metric: the exact per-rank workload of the N > 1 lines (rank 0's
    configs[4] shard: 32 data files of up to 1 GiB, configs[2]'s record distribution, the same
    generator seed, file ids and sequences), timed on this one GPU the same way — so that a 1 -> N
    efficiency computed from this point has no file-shape term (configs[2] at N = 1 is 17 files of
    2 GiB)."""
    from cask_amd.workloads import zipf_files
    files, vsz, n, rl = zipf_files(ctx, CFG4_FILES_PER_RANK * (CFG4_FILE - CFG2_MAX_RECORD) / 2 ** 30, CFG4_FILE,
                                   seed=0x5A1F, first_file_id=1, first_seq=1, first_key=0)
    assert len(files) == CFG4_FILES_PER_RANK, (len(files), CFG4_FILES_PER_RANK)
    torch.cuda.synchronize(dev)
    views = [(f.file_id, f.data) for f, _ in files]
    rows = ctx.alloc_rows(n + 16)
    res = ctx.scan_device(views, rows)
    assert res.count == n, (res.count, n)
    check_rows(torch, rows, res, files, vsz, rl, 1)
    run, timings = ctx.prepare_scan(views, rows)
    for _ in range(3):
        run()
    el, tt = time_loop(torch, dev, run, timings, steps, lambda: torch.cuda.synchronize(dev), None, "nccl")
    nb = sum(f.data.numel() for f, _ in files)
    k = sum(t[1] for t in tt) / len(tt)
    out = {"workload": "configs[4] shard of rank 0: 32 x 1 GiB data files, configs[2]'s record distribution "
                       "(the N > 1 lines' per-GPU workload, timed at N = 1)",
           "files": len(files), "records": n, "bytes": nb,
           "gibps": nb * steps / el / 2 ** 30, "ms_per_step": el * 1e3 / steps, "steps": steps,
           "kernel": "k_run_hash", "kernel_ms_avg": k, "kernel_frac_of_8TBps": nb / (k * 1e-3) / 1e9 / HBM_PEAK_GBPS}
    del files, vsz, rl, views, rows, res
    torch.cuda.empty_cache()
    return out


def cfg5_shard_secondary(ctx, torch, dev, rank, world, dist, backend, same_device, steps, barrier):
    """N > 1, reported beside the metric: this rank's shard of SURVEY §8d's cfg5 — 32 data files of
    3,702,558 fixed 290-B records (16-B unique keys, 256-B values; 1,073,741,820 B each), file ids
    rank*32+1.., 118.5 M records per rank — scanned device-resident (its own GiB/s), then the keydir
    of the whole job built by the key-hash partition (SURVEY §8e's huge-keyspace path, no rank holds
    more than its owners' share): each rank's block on its GPU, split on the device by key owner,
    part o to rank o (cask_keydir_exchange_rccl over RCCL; a gloo rehearsal through torch.distributed),
    each rank's fold of the keys it owns and the Stats from every owner's terms. Checked: the owners'
    live keys add up to every record of every rank, each rank's Stats are {file: (records, 0, 0)} for
    all 32 x N files, and the sequence is the job's. Also the end-to-end rate of the first 2 files
    of the shard from pageable host memory (H2D, scan, rows D2H)."""
    from cask_amd.keydir import KeydirFold, partition_device, shard_keydir
    from cask_amd.workloads import CFG2_KSZ, CFG2_RECORDS_PER_FILE as RPF, CFG2_VSZ, fixed_file
    out = {"workload": "cfg5 shard: 32 x 1,073,741,820 B of 290-B records per rank (SURVEY 8d cfg5 / configs[4])"}
    nf = CFG4_FILES_PER_RANK
    files = []
    for i in range(nf):
        fid = rank * nf + i + 1
        seq0 = 1 + (fid - 1) * RPF
        files.append(fixed_file(ctx, fid, RPF, CFG2_KSZ, CFG2_VSZ, seq0, seq0, 0xC0FFEE + fid))
    torch.cuda.synchronize(dev)
    views = [(f.file_id, f.data) for f in files]
    n = nf * RPF
    nbytes = sum(f.data.numel() for f in files)
    rows = ctx.alloc_rows(n + 16)
    res = ctx.scan_device(views, rows)
    assert res.error is None and res.count == n
    assert int((rows["status"][:n] != 0).sum().item()) == 0
    run, timings = ctx.prepare_scan(views, rows)
    run()
    el, _ = time_loop(torch, dev, run, timings, steps, barrier, dist, backend)
    out["scan_gibps_all_ranks"] = nbytes * world * steps / el / 2 ** 30
    out["scan_ms_per_step"] = el * 1e3 / steps
    res = ctx.scan_device(views, rows)
    barrier()
    t0 = time.perf_counter()
    blk = shard_keydir(ctx, views, rows, res.count, res.file_row_offset)
    barrier()
    t1 = time.perf_counter()
    out["block_ms"] = (t1 - t0) * 1e3
    out["block_bytes_per_rank"] = int(blk.numel())
    del rows, res
    if backend == "nccl" and not same_device:
        from cask_amd.distributed import exchange_fold_rccl, rccl_comm_from_dist
        comm = rccl_comm_from_dist(dev.index)
        barrier()
        t1 = time.perf_counter()
        db, sent, got = exchange_fold_rccl(ctx, comm, blk)
        barrier()
        t2 = time.perf_counter()
        comm.close()
        out["exchange"] = "cask_keydir_exchange_rccl (device partition, grouped send/recv over xGMI, owner folds, terms all-gather)"
    else:  # rehearsal: the same parts through torch.distributed point-to-point
        from cask_amd.distributed import all_gather_bytes, exchange_parts
        barrier()
        t1 = time.perf_counter()
        parts = [p.cpu() for p in partition_device(ctx, blk, world)]
        sent = sum(int(p.numel()) for i, p in enumerate(parts) if i != rank)
        recv = exchange_parts(parts)
        got = sum(int(p.numel()) for p in recv)
        fold = KeydirFold()
        fold.merge_all(recv)
        terms = all_gather_bytes(torch.from_numpy(fold.terms()))
        db = fold.finish_terms(b"".join(t.numpy().tobytes() for t in terms))
        del parts, recv
        barrier()
        t2 = time.perf_counter()
        out["exchange"] = f"torch.distributed {backend} rehearsal (device partition, parts through host memory)"
    out["exchange_fold_ms"] = (t2 - t1) * 1e3
    out["sent_bytes_per_rank"] = int(sent)
    out["received_bytes_per_rank"] = int(got)
    mine = len(db)
    tn = torch.tensor([mine], dtype=torch.int64, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(tn)
    stats_ok = db.stats() == {f: (RPF, 0, 0) for f in range(1, nf * world + 1)}
    ok = torch.tensor([1 if stats_ok and db.current_sequence == nf * world * RPF + 1 else 0], dtype=torch.int64,
                      device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    out["live_keys_this_rank"] = mine
    out["live_keys_all_ranks"] = int(tn.item())
    out["keydir_ok"] = int(tn.item()) == nf * world * RPF and int(ok.item()) == 1
    db.close()
    del blk
    if rank == 0:  # end to end: the first 2 files from pageable host memory
        host = [(f.file_id, f.data.cpu().numpy()) for f in files[:2]]
        ctx.scan_host(host[:1])
        te = time.perf_counter()
        hr = ctx.scan_host(host)
        e2e = time.perf_counter() - te
        assert hr.count == 2 * RPF and hr.error is None
        out["e2e_host_scan_gibps"] = sum(b.size for _, b in host) / e2e / 2 ** 30
        del host, hr
    del files, views
    torch.cuda.empty_cache()
    return out


def main():
    args = parse()
    env = cask_env(args.allow_tuning)
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if args.same_device:
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":  # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)

    import hashlib
    import cask_amd
    from cask_amd import ScanContext
    from cask_amd.workloads import zipf_files
    # only the in-tree product build is ever timed (no environment variable selects another)
    lib_path = cask_amd._lib.loaded_path()
    if lib_path != cask_amd.LIB_PATH:
        raise SystemExit(f"bench.py times only {cask_amd.LIB_PATH}, not {lib_path}")
    with open(lib_path, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()

    ctx = ScanContext(dev.index)
    if world == 1:
        cfg = "configs[2]"
        first_seq, first_key, first_fid = 1, 0, 1
        files, vsz, n, rl = zipf_files(ctx, CFG2_GIB, CFG2_MAX_FILE)
    else:  # one rank's shard of configs[4]: 32 x 1 GiB, file ids rank*32+1.., sequences after rank-1's
        cfg = "configs[4]"
        first_seq, first_key, first_fid = 1 + rank * SEQ_STRIDE, rank * SEQ_STRIDE, 1 + rank * CFG4_FILES_PER_RANK
        # (each file fills to within one record of CFG4_FILE, so a shard of 32 x (CFG4_FILE - the
        # longest record) bytes is exactly 32 files: a 33rd would take the next rank's first file id)
        files, vsz, n, rl = zipf_files(ctx, CFG4_FILES_PER_RANK * (CFG4_FILE - CFG2_MAX_RECORD) / 2 ** 30, CFG4_FILE,
                                       seed=0x5A1F + rank, first_file_id=first_fid, first_seq=first_seq,
                                       first_key=first_key)
        assert len(files) == CFG4_FILES_PER_RANK, (len(files), CFG4_FILES_PER_RANK)
    torch.cuda.synchronize(dev)
    views = [(f.file_id, f.data) for f, _ in files]
    bytes_per_step = sum(f.data.numel() for f, _ in files)
    nfiles = len(views)
    rows = ctx.alloc_rows(n + 16)

    # correctness gate before timing (every rank): rows equal the generator's records
    res = ctx.scan_device(views, rows)
    assert res.count == n, (res.count, n)
    check_rows(torch, rows, res, files, vsz, rl, first_seq)
    counters = ctx.last_counters()

    run, timings = ctx.prepare_scan(views, rows)
    for _ in range(args.warmup):
        run()

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # the timed loop issues the same C call a compiled caller would (arguments built once); each
    # step's phase times (HIP events inside the library) are copied out of the context after it
    elapsed, tt = time_loop(torch, dev, run, timings, args.steps, barrier, dist, args.dist_backend)
    ms_per_step = elapsed * 1e3 / args.steps
    # The first call over a file set (a real Cask::open scans each set once, cask.rs:346-382): the
    # timed steps reuse the context's per-set state — the region probe (k_probe_regions) and the file
    # table already on the device — so a call over another set in between makes the next full call
    # pay both again. Reported beside `value`, never in it.
    cold = []
    for _ in range(0 if args.no_cold else 3):
        ctx.scan_device(views[:1], rows)
        torch.cuda.synchronize(dev)
        t_c = time.perf_counter()
        run()
        torch.cuda.synchronize(dev)
        cold.append((time.perf_counter() - t_c) * 1e3)
    bytes_all = bytes_per_step * world
    if dist is not None:  # every rank's bytes (the shards differ by less than a record each)
        tb_ = torch.tensor([bytes_per_step], dtype=torch.int64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tb_)
        bytes_all = int(tb_.item())
    value = bytes_all * args.steps / elapsed / 2 ** 30

    walk = int(counters.get("walk_mode") or 0)
    # (a call that ran both modes times k_run_hash and k_scan_chunks as one span: cask_scan.h)
    kname = {0: "k_scan_chunks", 1: "k_run_hash"}.get(walk, "k_run_hash+k_scan_chunks")
    k_avg = sum(t[1] for t in tt) / len(tt)
    achieved = bytes_per_step / (k_avg * 1e-3) / 1e9  # algorithmic GB/s of the dominant kernel
    traffic, traffic_src = load_traffic(kname)
    # the read-only stream ceiling over the same bytes, beside the roofline (not in `value`)
    ceiling = stream_ceiling(torch, dev, views) if rank == 0 else None
    names = ["pipeline_ms", "hash_or_chunk_scan_ms", "long_ms", "validate_ms", "repair_ms", "compact_ms",
             "search_ms", "chase_ms"]
    breakdown = {nm: sum(t[i] for t in tt) / len(tt) for i, nm in enumerate(names)}
    extra = {"pipeline_breakdown_ms": breakdown,
             # SURVEY §8d's definition: device time from the first to the last kernel of a step
             # (HIP events), per GPU; `value` above is the wall clock, host gap included
             "device_gibps_per_gpu": bytes_per_step / (breakdown["pipeline_ms"] * 1e-3) / 2 ** 30,
             "cold_call_ms": sorted(cold)[len(cold) // 2] if cold else None,
             # device scratch the context holds for this workload (chunk table, slot rows, call
             # blocks, repair state), beside the log bytes it scans
             "scratch_bytes": ctx.scratch_bytes(),
             "scratch_bytes_per_log_byte": ctx.scratch_bytes() / bytes_per_step,
             "step_note": ("every timed step is one cask_scan_device call over the same resident files: the "
                           "region probe and the device file table are cached on the context across steps; "
                           "cold_call_ms is the median of 3 calls made right after a call over another file "
                           "set (probe + table upload + scan), against ms_per_step warm")}

    # the line, built now: the secondary measurements below only add keys to `extra`, and a watchdog on
    # rank 0 prints it without them if they stall (a collective that never returns)
    line = None
    if rank == 0:
        if world == 1:
            workload = ("configs[2]: 32 GiB, 16-B keys, Zipf(1.1) value sizes 16 B-64 KiB, files of <= 2 GiB "
                        "(LogWriter rollover at the default max_file_size), 1-GPU device-resident scan")
        else:
            workload = (f"configs[4]: 32 x 1 GiB data files per GPU ({world} GPUs, {32 * world} files), "
                        f"configs[2]'s record distribution, unique keys, device-resident scan per rank")
        line = {
            "metric": "GiB/s of log bytes CRC-verified+decoded, device-resident, at 1/2/4/8 GPUs",
            "value": value,
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (device-generated records: splitmix64 keys/values, XXH32 seed 0 checksums)",
            "config": {
                "workload": workload,
                "files_per_gpu": nfiles,
                "records_per_gpu": n,
                "mean_record_bytes": bytes_per_step / n,
                "bytes_per_gpu": bytes_per_step,
                "chunk_bytes": ctx.chunk_bytes(),
                "checksum": "XXH32 seed 0 (the reference's twox-hash, not CRC32: SURVEY.md §0)",
                "parallelism": f"file-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kname,
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel_ms_avg": k_avg,
                "timer": ("mean over the K timed steps of HIP events recorded around the kernel on the "
                          "scan's stream (cask_last_timings8); rocprofv3's figures for the same kernel "
                          "are under profiles/ (kernel_stats.csv: mean and median per launch)"),
                "algorithmic_bytes_per_launch": bytes_per_step,
                "stream_ceiling": ceiling,
                "frac_of_stream_ceiling": (achieved / ceiling["gbps"]) if ceiling and "gbps" in ceiling else None,
            },
            "cpu_baseline": None,  # (rank 0 at N = 1: filled in below)
            "counters": counters,
            "cask_env": env,
            "library": {"path": os.path.relpath(lib_path, ROOT), "sha256": lib_sha},
        }
    printed = threading.Lock()
    done = []

    def emit(extra_now, note=None):
        with printed:
            if done or line is None:
                return
            done.append(1)
            out = dict(line)
            out.update(extra_now)
            if note:
                out["secondary_timeout"] = note
            print(json.dumps(out), flush=True)

    watchdog = None
    if rank == 0 and dist is not None:
        def fire():
            emit(dict(extra), f"the multi-rank secondary measurements did not finish within {args.secondary_timeout:.0f} s; "
                              f"the line was printed without the ones still running")
            # a partial run: the line is out (the timed metric is complete), but the exit status says
            # that a secondary measurement hung, and the other ranks are still blocked in it
            os._exit(3)
        watchdog = threading.Timer(args.secondary_timeout, fire)
        watchdog.daemon = True
        watchdog.start()

    # N>1: this rank's keydir block and the blocks' gather + rank-0 fold over RCCL through the C ABI
    # (cask_keydir_gather_rccl), reported apart from the metric; a failure is reported, not fatal
    if dist is not None and not args.no_gather:
        try:
            from cask_amd.keydir import shard_keydir
            # every rank's record count (ranks' Zipf draws differ): all of them are live keys
            tn = torch.tensor([n], dtype=torch.int64, device=dev if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(tn)
            n_all = int(tn.item())
            res = ctx.scan_device(views, rows)
            barrier()
            tb = time.perf_counter()
            blk = shard_keydir(ctx, views, rows, res.count, res.file_row_offset)
            barrier()
            tg = time.perf_counter()
            if args.dist_backend == "nccl" and not args.same_device:
                from cask_amd.distributed import gather_fold_rccl, rccl_comm_from_dist
                comm = rccl_comm_from_dist(dev.index)
                barrier()
                tg = time.perf_counter()
                db, got, mx = gather_fold_rccl(ctx, comm, blk, root=0)
                barrier()
                te = time.perf_counter()
                comm.close()
                extra["keydir_gather"] = "cask_keydir_gather_rccl (RCCL over xGMI, C ABI; fold on rank 0 included)"
            else:  # rehearsal: torch.distributed point-to-point, then the fold
                from cask_amd.distributed import allreduce_max_seq, gather_blocks
                from cask_amd.keydir import KeydirFold
                got_b = gather_blocks(blk if args.dist_backend == "nccl" else blk.cpu(), dst=0)
                mx = allreduce_max_seq(first_seq + n - 1, dev if args.dist_backend == "nccl" else "cpu")
                db, got = None, sum(int(b.numel()) for b in got_b) if got_b else int(blk.numel())
                if rank == 0:
                    fold = KeydirFold()
                    fold.merge_all([b.cpu() for b in got_b])
                    db = fold.finish()
                barrier()
                te = time.perf_counter()
                extra["keydir_gather"] = f"torch.distributed {args.dist_backend} rehearsal"
            extra["keydir_block_ms"] = (tg - tb) * 1e3
            extra["keydir_gather_fold_ms"] = (te - tg) * 1e3
            extra["keydir_block_bytes_per_rank"] = int(blk.numel())
            extra["keydir_max_seq"] = int(mx)
            if rank == 0:
                extra["keydir_gathered_bytes"] = int(got)
                extra["keydir_live_keys"] = len(db)
                # unique keys: every record of every rank is live
                extra["keydir_records_all_ranks"] = n_all
                extra["keydir_ok"] = len(db) == n_all and db.current_sequence == int(mx) + 1
                db.close()
            del blk
        except Exception as e:  # noqa: BLE001 - reported in the line
            extra["keydir_gather_error"] = f"{type(e).__name__}: {e}"[:300]

    # N>1: SURVEY's cfg5 shard per rank and the key-hash partitioned keydir (reported beside the metric)
    if dist is not None and not args.no_cfg5:
        # (the workload is kept by `zf` whatever happens inside; only the generator's views are dropped
        # for the shard's memory, and the rows are rebuilt after it, failed or not)
        zf = (files, vsz, rl)
        res = None
        files = vsz = rl = None
        rows = None
        torch.cuda.empty_cache()
        secondary(extra, "cfg5_shard", lambda: cfg5_shard_secondary(
            ctx, torch, dev, rank, world, dist, args.dist_backend, args.same_device, max(3, min(args.steps, 10)), barrier))
        files, vsz, rl = zf
        try:
            res = ctx.scan_device(views, ctx.alloc_rows(n + 16))
        except Exception as e:  # noqa: BLE001 - reported in the line
            res = None
            extra["rescan_error"] = f"{type(e).__name__}: {e}"[:300]

    # end-to-end: host-resident files -> H2D -> scan -> rows D2H (cask_scan_host), first 2 files
    if rank == 0 and not args.no_e2e and res is not None:
        host = [(f.file_id, f.data.cpu().numpy()) for f, _ in files[:2]]
        ctx.scan_host(host[:1])
        te = time.perf_counter()
        hr = ctx.scan_host(host)
        e2e = time.perf_counter() - te
        assert hr.count == res.file_row_offset[2] - res.file_row_offset[0]
        extra["e2e_host_scan_gibps"] = sum(b.size for _, b in host) / e2e / 2 ** 30
        extra["e2e_note"] = (f"cask_scan_host over the first 2 {cfg} files: pageable host buffers -> H2D -> "
                             f"scan -> 5 row arrays D2H, 1 GPU")
        del host, hr

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline([f for f, _ in files], max(1, min(args.cpu_sample_files, len(files))), cfg)
        line["cpu_baseline"] = cpu

    if rank == 0 and world == 1 and not (args.no_cfg1 and args.no_shard_n1):
        res = None
        rows = views = None
        files = vsz = rl = None
        run = timings = None
        torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_shard_n1:
        secondary(extra, "configs4_shard_n1", lambda: cfg4_shard_n1_secondary(ctx, torch, dev, args.steps))
    if rank == 0 and world == 1 and not args.no_cfg1:
        extra["configs1_secondary"] = cfg1_secondary(ctx, torch, dev, max(10, args.steps))

    if watchdog is not None:
        watchdog.cancel()
    if rank == 0:
        emit(extra)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

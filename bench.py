#!/usr/bin/env python3
"""Headline benchmark: device-resident Cask data-file scan (decode + XXH32 verify + row emit).

Metric (BASELINE.json): GiB/s of log bytes checksum-verified + decoded, device-resident. A step is
one pass of the scan over one batch: BASELINE configs[1] per GPU (8 data files x 1,073,741,820 B,
3,702,558 records of 16 B key + 256 B value each), already resident in HBM. With N GPUs each rank
scans its own 8 files (weak scaling; data files shard with no collective). Rank 0 prints one JSON
line with the roofline of the dominant kernel (k_scan_chunks, HIP events inside the library) and
the CPU baseline (the oracle's reference-faithful replay, timed on this host, rank 0, N=1 only).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...      (driver, N>1)
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md (8.0 TB/s spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # (a step is ~1.7 ms: 100 steps keep host hiccups out of the number and still take 0.2 s)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--files", type=int, default=8, help="data files per GPU (configs[1]: 8)")
    ap.add_argument("--records-per-file", type=int, default=3_702_558)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-files", type=int, default=1, help="files timed by the CPU baseline")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-resident (H2D+D2H) measurement")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--dist-backend", default="nccl",
                    help="rehearsal only: gloo (blocks gathered through host memory)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank on cuda:0 (a one-GPU box)")
    ap.add_argument("--no-segmented", action="store_true",
                    help="skip the segmented-output measurement (profiling runs: dense-path launches only)")
    return ap.parse_args()


def cpu_baseline(files, nfiles: int):
    """The oracle's reference-faithful replay (read(2) per header/key/value, 5 write(2) per hint,
    Index::update fold; 1 thread as in cask.rs:348) over `nfiles` of the workload's files."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ffi as O
    O.load()
    tmp = tempfile.mkdtemp(prefix="cask_cpu_")
    paths = []
    total = 0
    for f in files[:nfiles]:
        p = os.path.join(tmp, f"{f.file_id:010}.cask.data")
        f.data.cpu().numpy().tofile(p)
        paths.append((f.file_id, p))
        total += f.data.numel()
    # warm the page cache, as the reference's replay would read files already on disk
    for _, p in paths:
        with open(p, "rb") as fh:
            while fh.read(1 << 24):
                pass
    ix = O.Index()
    t0 = time.perf_counter()
    recs = 0
    for fid, p in paths:
        r = O.replay_faithful(p, p.replace(".cask.data", ".cask.hint"), fid, ix)
        assert r.err_kind == 0, r.err_kind
        recs += r.records
    dt = time.perf_counter() - t0
    # fast restatement (context only): mmap-style tight loop, 1 core
    buf = np.fromfile(paths[0][1], dtype=np.uint8)
    ix2 = O.Index()
    t1 = time.perf_counter()
    O.replay_fast(buf, paths[0][0], ix2)
    dt_fast = time.perf_counter() - t1
    del ix, ix2
    for _, p in paths:
        os.remove(p)
        h = p.replace(".cask.data", ".cask.hint")
        if os.path.exists(h):
            os.remove(h)
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
        "sample": f"{nfiles} of the {len(files)} configs[1] files ({total} B, {recs} records) on disk, warm page "
                  f"cache; oracle/cask_oracle.c orc_replay_file_faithful = Cask::open scan path without hint "
                  f"files (3 read(2) + 5 write(2) + fold per record)",
        "seconds": dt, "host_cpu": cpu, "nproc": os.cpu_count(),
        "fast_restatement_gibps_1core": buf.size / dt_fast / 2 ** 30,
    }


def load_traffic():
    """Per-launch HBM bytes of k_scan_chunks from the committed rocprofv3 PMC pass (see
    profiles/README.md); null when absent."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    return d.get("hbm_bytes_per_launch"), d.get("source")


def main():
    args = parse()
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
    from cask_amd.workloads import CFG2_KSZ, CFG2_VSZ, fixed_file
    # only the in-tree product build is ever timed (no environment variable selects another)
    lib_path = cask_amd._lib.loaded_path()
    if lib_path != cask_amd.LIB_PATH:
        raise SystemExit(f"bench.py times only {cask_amd.LIB_PATH}, not {lib_path}")
    with open(lib_path, "rb") as fh:
        lib_sha = hashlib.sha256(fh.read()).hexdigest()

    ctx = ScanContext(dev.index)
    rpf = args.records_per_file
    rl = 18 + CFG2_KSZ + CFG2_VSZ
    files = []
    for i in range(args.files):
        fid = rank * args.files + i + 1  # contiguous file-id range per rank
        seq0 = 1 + (fid - 1) * rpf
        files.append(fixed_file(ctx, fid, rpf, CFG2_KSZ, CFG2_VSZ, seq0, seq0, 0xC0FFEE + fid, device=dev))
    torch.cuda.synchronize(dev)
    views = [(f.file_id, f.data) for f in files]
    bytes_per_step = sum(f.data.numel() for f in files)
    rows = ctx.alloc_rows(args.files * rpf)

    # correctness gate before timing: every record verifies, count exact
    res = ctx.scan_device(views, rows)
    assert res.count == args.files * rpf and res.error is None, (res.count, res.error)
    assert int((rows["status"][:res.count] != 0).sum().item()) == 0

    for _ in range(args.warmup):
        ctx.scan_device(views, rows)

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # the timed loop issues the same C call a compiled caller would (arguments built once); each
    # step's phase times (HIP events inside the library) are copied out of the context after it
    run, timings = ctx.prepare_scan(views, rows)
    tbuf = [(C.c_float * 6)() for _ in range(args.steps)]
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run()
        timings(tbuf[i])
    barrier()
    elapsed = time.perf_counter() - t0
    k1_ms = [float(t[1]) for t in tbuf]  # cask_last_timings: [0] pipeline, [1] chunk scan
    pipe_ms = [float(t[0]) for t in tbuf]
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed * 1e3 / args.steps
    total_bytes = bytes_per_step * world * args.steps
    value = total_bytes / elapsed / 2 ** 30

    k1_avg = sum(k1_ms) / len(k1_ms)
    achieved = bytes_per_step / (k1_avg * 1e-3) / 1e9  # algorithmic GB/s of the dominant kernel
    traffic, traffic_src = load_traffic()

    extra = {"pipeline_breakdown_ms": ctx.last_timings(),
             # SURVEY §8d's definition: device time from the first to the last kernel of a step
             # (HIP events), per GPU; `value` above is the wall clock, host gap included
             "device_gibps_per_gpu": bytes_per_step / (sum(pipe_ms) / len(pipe_ms) * 1e-3) / 2 ** 30}
    counters = ctx.last_counters()
    # segmented output (no dense compaction; every slot row written), same files, same clock
    if not args.no_segmented:
        ctx.scan_device_segmented(views)
        barrier()
        ts = time.perf_counter()
        for _ in range(args.steps):
            ctx.scan_device_segmented(views)
        barrier()
        extra["segmented_gibps"] = bytes_per_step * world * args.steps / (time.perf_counter() - ts) / 2 ** 30
    # keydir block of this rank's files, and the blocks gathered on rank 0 over RCCL,
    # reported separately from the metric; any failure here is reported, not fatal to the line
    if dist is not None and not args.no_gather:
        try:
            from cask_amd.distributed import gather_blocks
            from cask_amd.keydir import shard_keydir
            res = ctx.scan_device(views, rows)
            barrier()
            tb = time.perf_counter()
            blk = shard_keydir(ctx, views, rows, res.count, res.file_row_offset)
            barrier()
            tg = time.perf_counter()
            got = gather_blocks(blk if args.dist_backend == "nccl" else blk.cpu(), dst=0)
            barrier()
            te = time.perf_counter()
            extra["keydir_block_ms"] = (tg - tb) * 1e3
            extra["keydir_gather_ms"] = (te - tg) * 1e3
            extra["keydir_block_bytes_per_rank"] = int(blk.numel())
            if rank == 0:
                extra["keydir_gathered_bytes"] = int(sum(b.numel() for b in got))
                # rank 0's fold of the blocks in rank order (host keydir, exact stats)
                from cask_amd.keydir import KeydirFold
                tf = time.perf_counter()
                fold = KeydirFold()
                for b in got:
                    fold.merge(b.cpu())
                db = fold.finish()
                extra["keydir_fold_ms"] = (time.perf_counter() - tf) * 1e3
                extra["keydir_live_keys"] = len(db)
                db.close()
            del blk, got
        except Exception as e:  # noqa: BLE001 - reported in the line
            extra["keydir_gather_error"] = f"{type(e).__name__}: {e}"[:300]

    # end-to-end: host-resident files -> H2D -> scan -> rows D2H (cask_scan_host)
    if rank == 0 and not args.no_e2e:
        host = [(f.file_id, f.data.cpu().numpy()) for f in files]
        ctx.scan_host(host[:1])
        te = time.perf_counter()
        hr = ctx.scan_host(host)
        e2e = time.perf_counter() - te
        assert hr.count == args.files * rpf
        extra["e2e_host_scan_gibps"] = bytes_per_step / e2e / 2 ** 30
        extra["e2e_note"] = "cask_scan_host: pageable host buffers -> H2D -> scan -> 5 row arrays D2H, 1 GPU"
        del host, hr

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(files, max(1, min(args.cpu_sample_files, len(files))))

    if rank == 0:
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
                "workload": "configs[1]: 8 GiB across 8 data files, fixed 16B keys / 256B values, 1-GPU "
                            "device-resident scan (per GPU; N GPUs scan N x 8 files)",
                "files_per_gpu": args.files,
                "records_per_file": rpf,
                "record_bytes": rl,
                "bytes_per_gpu": bytes_per_step,
                "chunk_bytes": ctx.chunk_bytes(),
                "checksum": "XXH32 seed 0 (the reference's twox-hash, not CRC32: SURVEY.md §0)",
                "parallelism": f"file-sharded x{world}",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_scan_chunks",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel_ms_avg": k1_avg,
                "algorithmic_bytes_per_launch": bytes_per_step,
                "pipeline_ms_avg": sum(pipe_ms) / len(pipe_ms),
            },
            "cpu_baseline": cpu,
            "counters": counters,
            "library": {"path": os.path.relpath(lib_path, ROOT), "sha256": lib_sha},
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

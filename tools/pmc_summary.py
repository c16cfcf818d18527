"""Turn a tools/gpu_profile.sh run (gpurun_out/prof_<tag>/) into the committed evidence under
profiles/: the rocprofv3 kernel stats, a per-kernel HBM-traffic table from the FETCH_SIZE and
WRITE_SIZE passes, and profiles/pmc_traffic.json (read by bench.py for roofline.traffic).

FETCH_SIZE / WRITE_SIZE are in KiB-scaled units of 1024 B per rocprofv3. Per
/opt/skills/guides/MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE reports half of the bytes of a
wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").replace("cask_dev::", "")


def per_kernel(path, counter):
    """Per kernel: the median over its launches (a run that also makes a few small calls — bench.py's
    cold calls over one file — leaves the median on the full-size ones) and the launch count."""
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and "cask_dev::" in r["Kernel_Name"]:
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def median_ns(trace):
    d = defaultdict(list)
    for r in csv.DictReader(open(trace)):
        if "cask_dev::" in r["Kernel_Name"]:
            d[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: sorted(v)[len(v) // 2] for k, v in d.items()}


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    if not os.path.isdir(src):  # tools/gpu_cfg2_pmc.sh's layout
        src = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
    out = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(out, f"{tag}_kernel_stats.csv"))
    fetch, nf = per_kernel(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write, nw = per_kernel(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    med = median_ns(os.path.join(src, "kt", "kt_kernel_trace.csv"))
    # memory-side read requests (tools/gpu_profile.sh's rdreq pass, when present): 128-B requests x
    # 128 + the others x 64. Where present they give the read bytes: FETCH_SIZE x2 under-reports
    # nontemporal whole-line reads.
    rq_path = os.path.join(src, "rdreq", "rdreq_counter_collection.csv")
    rq, rq128 = ({}, {})
    if os.path.exists(rq_path):
        rq, _ = per_kernel(rq_path, "TCC_EA0_RDREQ_sum")
        rq128, _ = per_kernel(rq_path, "TCC_EA0_RDREQ_128B_sum")
    lines = [f"# HBM traffic per launch ({tag}; medians over each kernel's launches, duration from the kernel trace): reads = memory-side read requests (TCC_EA0_RDREQ: 128-B ones x 128, "
             "others x 64) where measured, else FETCH_SIZE x2 (gfx950 correction); + WRITE_SIZE; bytes",
             "kernel,launches,median_ns,fetch_bytes_corrected,rdreq_bytes,write_bytes,hbm_bytes"]
    table = {}
    for k in sorted(set(fetch) | set(write)):
        f2 = 2.0 * fetch.get(k, 0.0)
        w = write.get(k, 0.0)
        avg = float(med[k]) if k in med else float("nan")
        # (per_kernel scales by 1024 for the KiB-unit counters: undone for request counts)
        rb = (rq128[k] / 1024.0 * 128 + (rq[k] - rq128[k]) / 1024.0 * 64) if k in rq and k in rq128 else None
        rd = rb if rb is not None else f2
        table[k] = {"fetch_bytes": rd, "write_bytes": w, "hbm_bytes": rd + w, "avg_ns": avg,
                    "reads_from": "TCC_EA0_RDREQ" if rb is not None else "FETCH_SIZE x2"}
        lines.append(f"{k},{nf.get(k, 0)},{avg:.0f},{f2:.0f},{'' if rb is None else f'{rb:.0f}'},{w:.0f},{rd + w:.0f}")
    with open(os.path.join(out, f"{tag}_pmc_traffic.csv"), "w") as f:
        f.write("\n".join(lines) + "\n")
    # profiles/pmc_traffic.json: per kernel (short name without template arguments), merged into
    # what is there; tools/pmc_summary.py TAG [WORKLOAD] [KERNEL,...]
    workload = sys.argv[2] if len(sys.argv) > 2 else "bench.py"
    want = sys.argv[3].split(",") if len(sys.argv) > 3 else ["k_run_hash", "k_scan_chunks"]
    jp = os.path.join(out, "pmc_traffic.json")
    doc = json.load(open(jp)) if os.path.exists(jp) else {}
    kern = doc.get("kernels", {})
    for k, t in table.items():
        base = k.split("<")[0]
        if base in want:
            kern[base] = {"kernel": k, "hbm_bytes_per_launch": t["hbm_bytes"], "fetch_bytes_per_launch": t["fetch_bytes"],
                          "write_bytes_per_launch": t["write_bytes"], "avg_ns": t["avg_ns"],
                          "source": f"profiles/{tag}_pmc_traffic.csv (rocprofv3 --pmc, reads from {t['reads_from']}, "
                                    f"+ WRITE_SIZE, separate passes, {workload})"}
    with open(jp, "w") as f:
        json.dump({"kernels": kern}, f, indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()

"""Per-kernel averages of every counter collected by tools/gpu_cfg2_pmc.sh (gpurun_out/pmc_<tag>/),
with derived occupancy / stall shares, into profiles/<tag>_cfg2_pmc_stalls.csv.

  python tools/pmc_stall_summary.py r03b
"""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").replace("cask_dev::", "")


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
    vals = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if not k.startswith("k_"):
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    stats = {short(r["Name"]): float(r["AverageNs"])
             for r in csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv")))}
    names = sorted({c for k in vals for c in vals[k]})
    out = os.path.join(ROOT, "profiles", f"{tag}_cfg2_pmc_stalls.csv")
    lines = ["# per-launch averages (rocprofv3 --pmc, one pass per counter group: tools/gpu_cfg2_pmc.sh); "
             "derived: busy = SQ_BUSY_CYCLES/GRBM_GUI_ACTIVE, valu_share = SQ_ACTIVE_INST_VALU/SQ_WAVE_CYCLES, "
             "wait_share = SQ_WAIT_ANY/SQ_WAVE_CYCLES, waves_resident = SQ_WAVE_CYCLES/SQ_BUSY_CYCLES (per SE), "
             "hbm_bytes = FETCH_SIZE*2 + WRITE_SIZE (KiB units x1024)",
             "kernel,avg_ns," + ",".join(names) + ",valu_share,wait_share,inst_wait_share,hbm_bytes"]
    for k in sorted(vals):
        avg = {c: sum(v) / len(v) for c, v in vals[k].items()}
        wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
        row = [k, f"{stats.get(k, float('nan')):.0f}"] + [f"{avg[c]:.4g}" if c in avg else "" for c in names]
        hbm = 2 * avg.get("FETCH_SIZE", 0) * 1024 + avg.get("WRITE_SIZE", 0) * 1024
        row += [f"{avg.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}", f"{avg.get('SQ_WAIT_ANY', 0) / wc:.3f}",
                f"{avg.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}", f"{hbm:.4g}"]
        lines.append(",".join(row))
    open(out, "w").write("\n".join(lines) + "\n")
    for ln in lines[1:]:
        print(ln)


if __name__ == "__main__":
    main()

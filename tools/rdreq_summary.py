"""Summarise tools/gpu_rdreq.sh (gpurun_out/rdreq_<tag>/) into profiles/<tag>_rdreq.csv: per kernel
(name with template arguments) and counter, the mean value per dispatch, plus the bytes those
request counts stand for (RDREQ_32B x 32 + RDREQ_64B x 64 + RDREQ_128B x 128) next to FETCH_SIZE's
own reading of them (RDREQ x 64, MI355X_MICROARCH.md §HBM).

  python tools/rdreq_summary.py r04a            (tools/gpu_rdreq.sh)
  python tools/rdreq_summary.py r04b pmcab      (tools/gpu_pmc_ab.sh: the source column is the build)
"""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    return name.split("(")[0].replace("void ", "").replace("cask_dev::", "").strip()


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04a"
    kind = sys.argv[2] if len(sys.argv) > 2 else "rdreq"
    src = os.path.join(ROOT, "gpurun_out", f"{kind}_{tag}")
    vals = defaultdict(lambda: defaultdict(list))  # (prefix, kernel) -> counter -> per-dispatch values
    for f in glob.glob(os.path.join(src, "*", "*_counter_collection.csv")):
        prefix = os.path.basename(os.path.dirname(f)).rsplit("_", 1)[0]  # u / b, or the build's name
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            k = (prefix, short(r["Kernel_Name"]), r["Dispatch_Id"])
            per[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        for ((p, kn, _), c), v in per.items():
            vals[(p, kn)][c].append(v)
    lines = [f"# {tag}: rocprofv3 --pmc, mean per dispatch; req_bytes = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B",
             "source,kernel,dispatches,counter,mean"]
    for (p, kn), cs in sorted(vals.items()):
        for c, v in sorted(cs.items()):
            lines.append(f"{p},{kn},{len(v)},{c},{sum(v) / len(v):.1f}")
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if all(x in m for x in ("TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")):
            b = 32 * m["TCC_EA0_RDREQ_32B_sum"] + 64 * m["TCC_EA0_RDREQ_64B_sum"] + 128 * m["TCC_EA0_RDREQ_128B_sum"]
            lines.append(f"{p},{kn},,req_bytes,{b:.0f}")
        if "TCC_EA0_RDREQ_sum" in m:
            lines.append(f"{p},{kn},,rdreq_x64_bytes,{64 * m['TCC_EA0_RDREQ_sum']:.0f}")
        if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m and m["TCC_HIT_sum"] + m["TCC_MISS_sum"] > 0:
            lines.append(f"{p},{kn},,l2_hit_rate,{m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.4f}")
    out = os.path.join(ROOT, "profiles", f"{tag}_{kind}.csv")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()

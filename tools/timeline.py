"""Print one step's kernel timeline (start, end, duration in ms, queue) from a rocprofv3
--kernel-trace CSV: the kernels between the last two k_finish launches."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [r for r in rows if "cask_dev" in r["Kernel_Name"] and "encode" not in r["Kernel_Name"]]
fin = [i for i, r in enumerate(ks) if "k_finish" in r["Kernel_Name"]]
seg = ks[(fin[-2] + 1 if len(fin) > 1 else 0): fin[-1] + 1]
t0 = min(int(r["Start_Timestamp"]) for r in seg)
for r in seg:
    n = r["Kernel_Name"].split("(")[0].replace("cask_dev::", "")
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    print(f"{n:18s} q{r['Queue_Id']:>3s} {s:7.3f} {e:7.3f} {e - s:6.3f}")

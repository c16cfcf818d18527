"""Means per build of a tools/ab.py log: GiB/s, ms per step, the hash (or chunk-scan) kernel, and the
search / chase / repair shares of the last step of each run.

  python tools/ab_summary.py gpurun_out/x.log
"""
import collections
import json
import re
import sys

acc = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"round (\d+) (\S+): ([\d.]+) GiB/s\s+([\d.]+) ms/step\s+k_scan ([\d.]+) ms\s+(\{.*\})", line)
    if m:
        d = json.loads(m.group(6))
        acc[m.group(2)].append((float(m.group(3)), float(m.group(4)), float(m.group(5)), d.get("search_ms", 0.0),
                                d.get("chase_ms", 0.0), d.get("repair_ms", 0.0)))
print(f"{'build':10s} {'GiB/s':>9s} {'ms/step':>8s} {'kernel':>7s} {'search':>7s} {'chase':>7s} {'repair':>7s}  runs")
for k, v in acc.items():
    mean = [sum(x[i] for x in v) / len(v) for i in range(6)]
    print(f"{k:10s} {mean[0]:9.1f} {mean[1]:8.4f} {mean[2]:7.4f} {mean[3]:7.4f} {mean[4]:7.4f} {mean[5]:7.4f}  {len(v)}")

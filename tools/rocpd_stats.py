"""Kernel statistics from a rocprofv3 results database (the default rocpd SQLite output of
`rocprofv3 --kernel-trace --stats -d DIR -o NAME`): one CSV row per kernel name with launch count and
mean / median / min / max / total duration in ms, plus the same for launches of at least --min-ms
(the full-size launches of a bench run, apart from its small parity and end-to-end calls).

  python tools/rocpd_stats.py gpurun_out/prof_TAG/run_results.db --min-ms 1.0 > profiles/TAG_kernel_stats.csv
"""
import argparse
import csv
import sqlite3
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--min-ms", type=float, default=0.0)
    ap.add_argument("--top", type=int, default=20)
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    by = {}
    for name, st, en in c.execute("select name, start, end from kernels"):
        by.setdefault(name, []).append((en - st) / 1e6)
    rows = sorted(by.items(), key=lambda kv: -sum(kv[1]))[: args.top]
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "launches", "mean_ms", "median_ms", "min_ms", "max_ms", "total_ms",
                f"launches_ge_{args.min_ms}ms", f"mean_ms_ge_{args.min_ms}ms", f"median_ms_ge_{args.min_ms}ms"])
    for name, d in rows:
        big = [x for x in d if x >= args.min_ms]
        short = name if len(name) < 120 else name[:117] + "..."
        w.writerow([short, len(d), f"{statistics.mean(d):.6f}", f"{statistics.median(d):.6f}", f"{min(d):.6f}",
                    f"{max(d):.6f}", f"{sum(d):.6f}", len(big), f"{statistics.mean(big):.6f}" if big else "",
                    f"{statistics.median(big):.6f}" if big else ""])


if __name__ == "__main__":
    main()

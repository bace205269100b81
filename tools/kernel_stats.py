"""Per-kernel duration summary (calls, total/avg/min/max ns, share) from a rocprofv3 run.

Usage: python tools/kernel_stats.py RESULTS.db|kernel_stats.csv [--out CSV]
Reads the rocpd SQLite database that ``rocprofv3 --kernel-trace --stats`` writes by
default (view ``kernels``), or passes a ``*_kernel_stats.csv`` through unchanged.
"""
import argparse
import csv
import sqlite3
import sys
from collections import defaultdict


def from_db(path):
    c = sqlite3.connect(path)
    d = defaultdict(list)
    for name, start, end in c.execute("select name, start, end from kernels"):
        d[name.split("(")[0].replace("void ", "")].append(end - start)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.src.endswith(".csv"):
        rows = list(csv.reader(open(a.src)))
    else:
        d = from_db(a.src)
        tot = sum(sum(v) for v in d.values())
        rows = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
        for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
            rows.append([k, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])
    w = csv.writer(open(a.out, "w", newline="") if a.out else sys.stdout)
    w.writerows(rows)


if __name__ == "__main__":
    main()

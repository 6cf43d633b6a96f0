"""Summarise a rocprofv3 SQLite output (``*_results.db``) into the kernel_stats.csv layout.

    python tools/rocpd_stats.py gpurun_out/<tag>/prof/run_results.db > profiles/<name>.csv

Columns as rocprofv3 --stats writes them: Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs, StdDev (one row per kernel symbol, sorted by total time).
"""
from __future__ import annotations

import csv
import math
import sqlite3
import sys
from collections import defaultdict


def main(path: str) -> None:
    con = sqlite3.connect(path)
    durs = defaultdict(list)
    for name, start, end in con.execute("select name, start, end from kernels"):
        durs[name].append(end - start)
    total = sum(sum(v) for v in durs.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs",
                "StdDev"])
    for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        n, s = len(v), sum(v)
        mean = s / n
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / n)
        w.writerow([name, n, s, round(mean, 3), round(100.0 * s / total, 2), min(v), max(v),
                    round(sd, 3)])


if __name__ == "__main__":
    main(sys.argv[1])

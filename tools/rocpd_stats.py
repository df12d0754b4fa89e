#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 rocpd database (results.db), written in
the column layout of rocprofv3's `--stats` kernel_stats.csv.

usage: tools/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/rN/kernel_stats_X.csv
"""
import math
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, duration from kernels").fetchall()
    per = {}
    for name, dur in rows:
        per.setdefault(name, []).append(int(dur))
    total = sum(sum(v) for v in per.values()) or 1
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"')
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        n, s = len(v), sum(v)
        avg = s / n
        sd = math.sqrt(sum((x - avg) ** 2 for x in v) / n)
        print(f'"{name}",{n},{s},{avg:.6f},{100.0 * s / total:.4g},{min(v)},{max(v)},{sd:.6f}')


if __name__ == "__main__":
    main(sys.argv[1])

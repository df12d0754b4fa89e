#!/usr/bin/env python3
"""Per-phase kernel durations from a rocprofv3 --kernel-trace CSV of bench.py:
the launches of one kernel name split by the bench phase they belong to
(tools/pmc_traffic.phase_keys: feas / ffd / trunc of the provisioning Solve,
feas_sim / sim / trunc_sim of the consolidation sweep, feas_c5 of the stress
matrix), so each roofline's avg_ms can be checked against the trace.

usage: tools/kernel_phases.py <kt_kernel_trace.csv> > phases.json
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import kernel_key, phase_keys  # noqa: E402


def main(path):
    rows = [r for r in sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
            if kernel_key(r["Kernel_Name"])]
    d = collections.defaultdict(list)
    for r, k in zip(rows, phase_keys([r["Kernel_Name"] for r in rows])):
        d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    out = {k: {"launches": len(v), "avg_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v)}
           for k, v in sorted(d.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])

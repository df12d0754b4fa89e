#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
(tools/profile_round.sh runs one pass per counter per bench leg, bench.py
--only <leg>), corrected as MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE
reports half the bytes of a wide coalesced read on gfx950 (x2); WRITE_SIZE is
read as is; both are in KiB.

usage: tools/pmc_traffic.py <leg> <fetch_counter_collection.csv> <write_counter_collection.csv> [traffic.json]
merges {leg: {kernel: {bytes, fetch_bytes_x2, write_bytes, launches}}} into traffic.json (stdout without it)
"""
import collections
import csv
import json
import os
import sys


def kernel_key(name):
    if name.startswith("void ffdw_kernel"):
        return "ffd"
    if name.startswith("void ffd_kernel"):
        return "sim" if ", true," in name else "ffd"
    if name.startswith("feas_cursor_kernel"):
        return "feas_cursor"
    if name.startswith("feas_kernel") or name.startswith("void feas_kernel"):
        return "feas"
    if name.startswith("trunc_kernel"):
        return "trunc"
    if "claim_filter_kernel" in name:
        return "filter"
    return None


def per_launch(path, counter):
    vals = collections.defaultdict(list)
    with open(path) as f:
        for r in sorted(csv.DictReader(f), key=lambda r: int(r["Dispatch_Id"])):
            k = kernel_key(r["Kernel_Name"])
            if k and r["Counter_Name"] == counter:
                vals[k].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main(leg, fetch_csv, write_csv, out_path=None):
    f = per_launch(fetch_csv, "FETCH_SIZE")
    w = per_launch(write_csv, "WRITE_SIZE")
    out = {}
    for k in sorted(set(f) | set(w)):
        fb = sum(f[k]) / len(f[k]) if f[k] else 0.0
        wb = sum(w[k]) / len(w[k]) if w[k] else 0.0
        out[k] = {"bytes": int(2 * fb + wb), "fetch_bytes_x2": int(2 * fb), "write_bytes": int(wb),
                  "launches": [len(f[k]), len(w[k])]}
    if out_path:
        allv = {}
        if os.path.exists(out_path):
            with open(out_path) as fh:
                allv = json.load(fh)
        allv[leg] = out
        with open(out_path, "w") as fh:
            json.dump(allv, fh, indent=1, sort_keys=True)
    else:
        print(json.dumps({leg: out}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])

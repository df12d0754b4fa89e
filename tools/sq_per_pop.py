"""SQ counters of the wave Solve kernel per pop, from tools/gpu_run.sh sqpmc
output: python tools/sq_per_pop.py <dir> <variant>... > json"""
import csv
import glob
import json
import os
import sys


def counters(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "ffdw_kernel" not in row.get("Kernel_Name", ""):
                continue
            out[row["Counter_Name"]] = out.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return out


def main(root, variants):
    res = {"what": "SQ counters of ffdw_kernel on CM per pop (both waves), rocprofv3 --pmc, two passes per library "
                   "(tools/gpu_run.sh sqpmc)", "per_pop": {}, "ffd_ms_in_the_pmc_run": {}}
    for v in variants:
        c = {}
        pops = None
        for p in ("a", "b"):
            c.update(counters(os.path.join(root, f"sq_{v}_{p}")))
            txt = open(os.path.join(root, f"sq_{v}_{p}.json")).read().strip().split("\n")[-1]
            j = json.loads(txt)
            pops = j["pops"]
            res["ffd_ms_in_the_pmc_run"][f"{v}_{p}"] = j["ffd_ms"]
        res["per_pop"][v] = {k: round(x / pops, 1) for k, x in sorted(c.items())}
        res["pops"] = pops
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])

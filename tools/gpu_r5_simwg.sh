#!/bin/bash
# simulation write traffic vs persistent workgroups per CU (GS_SIM_PER_CU):
# WRITE_SIZE per launch of the simulation kernel and its time
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_simwg
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
for pc in 6 3 1; do
  for leg in c4_e2e c4; do
    GS_SIM_PER_CU=$pc timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_${leg}_$pc -o w -- \
      python3 $R/bench.py --only $leg --steps 2 --warmup 0 --latency-steps 0 --no-cpu-baseline --detail-json $O/d_${leg}_$pc.json > $O/b_${leg}_$pc.out 2> $O/b_${leg}_$pc.err || exit 1
    python3 - <<PY
import csv, json
rows = [r for r in csv.DictReader(open("$O/w_${leg}_$pc/w_counter_collection.csv")) if "ffd_kernel" in r.get("Kernel_Name", "")]
vals = [float(r["Counter_Value"]) for r in rows if r.get("Counter_Name") == "WRITE_SIZE"]
d = json.load(open("$O/d_${leg}_$pc.json"))["consolidation_legs"]["$leg"]
print("$leg per_cu=$pc", "WRITE_SIZE KiB per launch (sum over dims):", [round(v) for v in vals][:6], "sim ms", d["kernel_ms"]["sim"])
PY
  done
done

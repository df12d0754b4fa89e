#!/bin/bash
# round-4: where the simulation kernel's writes come from (c4_mixed): vector
# memory / flat / scratch store instructions and the L2's write requests
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4p
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAVES SQ_INSTS_VMEM_RD TA_FLAT_WRITE_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $O/p1 -o p1 -- python3 bench.py --only c4_mixed --no-cpu-baseline --steps 2 --warmup 1 --detail-json $O/d1.json > $O/p1.log 2>&1 || exit 1
grep -h "ffd_kernel" $O/p1/p1_counter_collection.csv | awk -F, '{print $0}' | head -3 > /dev/null
python3 - $O/p1/p1_counter_collection.csv <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    if "ffd_kernel" not in r["Kernel_Name"]: continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(agg): print(k, agg[k] / max(1, n[k]), "per dispatch-row", n[k])
PY

#!/bin/bash
# Same-session A/B of gs_rank_instance_types (bench.py --only ranking):
# LIBS="libgpusched.so libgpusched_x.so"
set -euo pipefail
for k in 1 2 3; do
  for lib in ${LIBS:-libgpusched.so}; do
    r=$(GPUSCHED_LIB=$lib timeout -k 10 120 python3 bench.py --only ranking --no-cpu-baseline |
      python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ranking"]["ms_per_call_pcie_inclusive"])')
    echo "$lib $r"
  done
done

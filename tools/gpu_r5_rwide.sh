#!/bin/bash
# round 5: run mode in the wide-row instantiation (GS_RUN_WIDE, fast accepts
# only) -- C5 Solve parity at 50k against the oracle, then a same-session A/B
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_rwide
mkdir -p $O
cd $R
for rep in 1 2; do
  for lib in libgpusched.so libgpusched_rwide.so; do
    GPUSCHED_LIB=$lib timeout -k 10 200 python3 tools/ffd_diag.py --c5 > $O/c5_${lib}_$rep.json 2>&1 || exit 1
    echo "$rep $lib: $(head -c 330 $O/c5_${lib}_$rep.json)"
  done
done

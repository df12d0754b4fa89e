#!/bin/bash
# round 5: run mode in the wide-row instantiation with its exact checks
# (GS_RUN_WIDE=1, libgpusched_rwx.so) -- C5 parity (50k live oracle, 200k
# digest) with that library, then a same-session A/B of the C5 Solve
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_rwx
mkdir -p $O
cd $R
GPUSCHED_LIB=libgpusched_rwx.so timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 600 --timeout-method thread -k "c5" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in libgpusched.so libgpusched_rwx.so; do
    GPUSCHED_LIB=$lib timeout -k 10 200 python3 tools/ffd_diag.py --c5 > $O/c5_${lib}_$rep.json 2>&1 || exit 1
    echo "$rep $lib: $(head -c 400 $O/c5_${lib}_$rep.json)"
  done
done

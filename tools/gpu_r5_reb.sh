#!/bin/bash
# round 5: window rebase inside run mode (GS_RUN_REBASE) -- parity on the full-size
# Solves and the random suites, then a same-session A/B of the FFD device time
# against the same library built with GS_RUN_REBASE=0
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_reb
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_wave_sort.py tests/test_e2e_scenarios.py tests/test_node_labels.py tests/test_startup_taints.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for w in "" --c2 --c3 --e2e --c5; do
  for lib in libgpusched.so libgpusched_noreb.so; do
    GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w > $O/diag${w}_${lib}_$rep.json 2>&1 || exit 1
    echo "$rep $w $lib: $(head -c 200 $O/diag${w}_${lib}_$rep.json)"
  done
done
done
# shader cycles per pod category on CM (GS_CAT_TL build)
GPUSCHED_LIB=libgpusched_cat.so timeout -k 10 150 python3 tools/ffd_diag.py --cat > $O/diag_cat.json 2>&1 || exit 1
head -c 1500 $O/diag_cat.json

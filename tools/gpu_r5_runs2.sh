#!/bin/bash
# round 5: run mode restricted to the narrow non-topology instantiation;
# parity (full-size and random suites) and FFD device ms against GS_RUNS=0
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_runs2
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_wave_sort.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for w in "" --c2 --c3 --e2e --c5; do
  for lib in libgpusched.so libgpusched_noruns.so; do
    GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w > $O/diag${w}_${lib}.json 2>&1 || exit 1
    echo "$w $lib: $(head -c 60 $O/diag${w}_${lib}.json)"
  done
done

#!/bin/bash
# register-mode wave kernel: timing on CM / C3 / e2e, then the Solve parity suites
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for w in "" --c3 --e2e; do
  timeout -k 10 150 python3 tools/ffd_diag.py $w >> $O/rg_diag.txt 2>&1
done
cat $O/rg_diag.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_e2e_scenarios.py tests/test_topology.py tests/test_affinity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/rg_parity.log 2>&1
tail -3 $O/rg_parity.log

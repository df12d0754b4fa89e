#!/bin/bash
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 560 python -u -m pytest tests/test_gpu_parity.py tests/test_affinity.py tests/test_topology.py \
  tests/test_min_values.py tests/test_volumes.py tests/test_zone_anti_affinity.py -m gpu -x -q --timeout 240 \
  --timeout-method thread > $O/r3_hbm.log 2>&1
tail -3 $O/r3_hbm.log
timeout -k 10 300 python -u tools/cmc4_probe.py 5000 20000 > $O/r3_cmc4_probe.log 2>&1
cat $O/r3_cmc4_probe.log

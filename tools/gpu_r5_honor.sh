#!/bin/bash
# round 5: nodeAffinityPolicy Honor past the zone key (wave / block / hbm Solve, consolidation)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_honor
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_topology.py tests/test_consolidation_general.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > $O/pytest_gpu_honor.log 2>&1
tail -3 $O/pytest_gpu_honor.log

#!/bin/bash
# GPU parity of consolidation (plain and general simulation variants) and the
# topology-bearing Solve suites
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 560 python -u -m pytest tests/test_consolidation_general.py tests/test_consolidation.py tests/test_volumes.py \
  tests/test_multi_shard.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r3_cons.log 2>&1
tail -3 $O/r3_cons.log

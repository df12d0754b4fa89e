#!/bin/bash
# GPU parity of the topology refactor: topology, affinity, zone anti-affinity,
# minValues, volumes and the base parity suite (both Solve kernels)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_zone_anti_affinity.py tests/test_affinity.py tests/test_topology.py \
  tests/test_min_values.py tests/test_volumes.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > $O/r3_topo.log 2>&1
tail -3 $O/r3_topo.log

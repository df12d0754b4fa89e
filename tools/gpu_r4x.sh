#!/bin/bash
# round-4: nodeAffinityPolicy Honor with zone-only node affinity (topology
# parity), wide exact checks at 2 chunks per round trip (full-size digests)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4x
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_topology.py tests/test_gpu_fullsize.py tests/test_e2e_scenarios.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; exit $rc

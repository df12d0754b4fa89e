#!/bin/bash
# round-4: stamped simulation overlays: consolidation / topology parity, then PMC traffic of the consolidation legs
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4f
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_consolidation.py tests/test_consolidation_general.py tests/test_e2e_scenarios.py tests/test_zone_anti_affinity.py tests/test_affinity.py tests/test_volumes.py tests/test_multi_shard.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SKIP_KT=1 LEGS="c4_e2e c4_mixed c4 c4_e2e_multi c4_multi" TRAFFIC=traffic_r4f.json bash tools/profile_round.sh > $O/prof.log 2>&1
rc=$?; tail -c 300 $O/prof.log; exit $rc

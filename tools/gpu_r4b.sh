#!/bin/bash
# round-4: consolidation parity after the sparse candidate exclusion, then PMC traffic of the consolidation legs
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_consolidation.py tests/test_consolidation_general.py tests/test_e2e_scenarios.py tests/test_zone_anti_affinity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/r4b_tests.log 2>&1
tail -3 $O/r4b_tests.log
SKIP_KT=1 LEGS="${LEGS:-c4_e2e c4_mixed c4 c4_e2e_multi}" TRAFFIC=traffic_r4b.json bash tools/profile_round.sh > $O/r4b_prof.log 2>&1
tail -c 200 $O/r4b_prof.log

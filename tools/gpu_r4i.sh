#!/bin/bash
# round-4: simulation overlay changes (free-key copy on write, LDS node->entry hash) under the
# consolidation parity tests, PMC traffic of the consolidation legs, then the same-session FFD A/B
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4i
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_consolidation.py tests/test_consolidation_general.py tests/test_e2e_scenarios.py tests/test_zone_anti_affinity.py tests/test_volumes.py tests/test_affinity.py tests/test_min_values.py tests/test_multi_shard.py tests/test_free_keys_wide.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
SKIP_KT=1 LEGS="c4_e2e c4_mixed c4 c4_e2e_multi c4_multi" TRAFFIC=traffic_r4i.json bash tools/profile_round.sh > $O/prof.log 2>&1 || exit 1
cp $R/gpurun_out/prof/traffic_r4i.json $O/
timeout -k 10 300 python bench.py --only c4_e2e --no-cpu-baseline --detail-json $O/c4e2e.json > $O/c4e2e.out 2>&1 || exit 1
bash tools/gpu_r4h.sh

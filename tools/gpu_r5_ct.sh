#!/bin/bash
# round 5: topology spread on the capacity-type key (the zone-count machinery
# on that key): topology / consolidation / Solve parity, then C3 / e2e / CM
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_ct
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_topology.py tests/test_consolidation_general.py tests/test_consolidation.py tests/test_affinity.py tests/test_zone_anti_affinity.py tests/test_e2e_scenarios.py tests/test_gpu_parity.py tests/test_node_labels.py tests/test_startup_taints.py tests/test_run_mode.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k "c3 or cm" --timeout 300 --timeout-method thread > $O/tests_full.log 2>&1
rc=$?; tail -2 $O/tests_full.log; [ $rc -eq 0 ] || exit $rc
for leg in c3 e2e; do
  timeout -k 10 400 python3 bench.py --only $leg --steps 3 --warmup 1 --latency-steps 0 --no-cpu-baseline --detail-json $O/d_${leg}.json > /dev/null 2> $O/e_${leg}.err || exit 1
  python3 -c "import json;d=json.load(open('$O/d_${leg}.json'))['configs'];k=list(d)[0];print(k, d[k]['ms_per_step'])"
done

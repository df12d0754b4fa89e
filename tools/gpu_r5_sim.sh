#!/bin/bash
# round 5: simulation queue arrays + add log in LDS -- consolidation parity,
# the C4 legs, then FETCH / WRITE PMC passes of the simulation legs
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_sim
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_consolidation.py tests/test_consolidation_general.py tests/test_e2e_scenarios.py tests/test_startup_taints.py tests/test_node_labels.py tests/test_multi_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for leg in c4 c4_mixed c4_multi c4_e2e c4_e2e_multi; do
  timeout -k 10 300 python3 bench.py --only $leg --steps 10 --warmup 2 --latency-steps 0 --no-cpu-baseline --detail-json $O/detail_$leg.json > $O/bench_$leg.out 2> $O/bench_$leg.err || exit 1
  python3 -c "import json;d=json.load(open('$O/detail_$leg.json'))['consolidation_legs']['$leg'];print('$leg', d['ms_per_sweep'], d['kernel_ms'])"
done
SKIP_KT=1 LEGS="c4 c4_mixed c4_e2e" TRAFFIC=traffic_r5_sim.json bash tools/profile_round.sh > $O/prof.log 2>&1
rc=$?; tail -3 $O/prof.log; exit $rc

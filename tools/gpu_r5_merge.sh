#!/bin/bash
# round 5: spread groups whose node filter cannot matter shared across
# filters (GS_GROUP_MERGE=1, default) vs one group per upstream group (0):
# topology / consolidation parity, then C3 and e2e A/B in one session
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_merge
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_topology.py tests/test_affinity.py tests/test_consolidation_general.py tests/test_e2e_scenarios.py tests/test_zone_anti_affinity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k c3 --timeout 300 --timeout-method thread > $O/tests_full.log 2>&1
rc=$?; tail -2 $O/tests_full.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in 1 0; do
    for leg in c3 e2e; do
      GS_GROUP_MERGE=$m timeout -k 10 400 python3 bench.py --only $leg --steps 3 --warmup 1 --latency-steps 0 --no-cpu-baseline --detail-json $O/d_${leg}_${m}_$rep.json > /dev/null 2> $O/e_${leg}_${m}_$rep.err || exit 1
      python3 -c "import json;d=json.load(open('$O/d_${leg}_${m}_$rep.json'))['configs'];k=list(d)[0];print('$rep merge=$m', k, d[k]['ms_per_step'], d[k].get('device_kernel_ms'))"
    done
  done
done

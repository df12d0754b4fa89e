#!/bin/bash
# round 5: per-NodeClaim instance-type summary in LDS as the scan's necessary
# test for pods with requirements (GS_OSUM=1, default) vs without (0):
# Solve parity, then CM / C3 / C2 / e2e / CM_C4 A/B in one session
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_osum
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_run_mode.py tests/test_topology.py tests/test_affinity.py tests/test_min_values.py tests/test_free_keys_wide.py tests/test_node_labels.py tests/test_startup_taints.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in 1 0; do
    for leg in cm c3 c2 e2e cm_c4; do
      GS_OSUM=$m timeout -k 10 400 python3 bench.py --only $leg --steps 3 --warmup 1 --latency-steps 0 --no-cpu-baseline --detail-json $O/d_${leg}_${m}_$rep.json > /dev/null 2> $O/e_${leg}_${m}_$rep.err || exit 1
      python3 -c "import json;d=json.load(open('$O/d_${leg}_${m}_$rep.json'))['configs'];k=list(d)[0];print('$rep osum=$m', k, d[k]['ms_per_step'], d[k].get('device_kernel_ms'))"
    done
  done
done

#!/bin/bash
# round-4: the wave scan's fast accept for hostname-only topology pods
# (VF_HOSTFA; nohf = without): topology / affinity / e2e parity, then e2e /
# e2e200 shapes (diag), C3, CM
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4ah
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_topology.py tests/test_affinity.py tests/test_zone_anti_affinity.py tests/test_e2e_scenarios.py tests/test_volumes.py tests/test_min_values.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in nohf base; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in --e2e --c3 ""; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"], d["cand_full"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done

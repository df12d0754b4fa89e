#!/bin/bash
# round-4: exact-check lanes also load the topology claim fields (zone
# requirement, first hostname count) with the header (this tree) vs not (notp)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4af
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_topology.py tests/test_affinity.py tests/test_zone_anti_affinity.py tests/test_e2e_scenarios.py tests/test_volumes.py tests/test_min_values.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in notp base; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in --e2e --c3; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done

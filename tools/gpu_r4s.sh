#!/bin/bash
# round-4: selection lists staged in lanes, hostname counts read past the L1
# and bumped by no-return atomics; block kernel: owned groups in LDS; plus the
# round-4 owned topology groups staged in lanes at the pop, per-pod zone
# minimum only for zone-spread owners: topology parity, then e2e / C3 / CM / C5
# against the previous commit's library
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4s
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_topology.py tests/test_affinity.py tests/test_zone_anti_affinity.py tests/test_e2e_scenarios.py tests/test_volumes.py tests/test_min_values.py tests/test_gpu_fullsize.py tests/test_consolidation_general.py tests/test_consolidation.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in prev base; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in --e2e --c3 "" --c5; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done

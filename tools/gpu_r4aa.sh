#!/bin/bash
# round-4: wide-row scans read the next chunk's order words with this chunk's
# codes, for TOPO too (pft) or every instantiation (pfa): e2e / C3 / CM
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4aa
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_topology.py tests/test_e2e_scenarios.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base pft pfa; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in --e2e --c3 ""; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done

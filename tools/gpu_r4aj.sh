#!/bin/bash
# round-4: the wave scan's fast accept for hostname-only topology pods
# (VF_HOSTFA; nohf = without; hf1 = one walk; this tree: the walk split): e2e /
# C3 / CM
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python -u -m pytest tests/test_topology.py tests/test_affinity.py tests/test_e2e_scenarios.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > /tmp/r4aj_tests.log 2>&1 || { tail -5 /tmp/r4aj_tests.log; exit 1; }
tail -1 /tmp/r4aj_tests.log
O=$R/gpurun_out/r4aj
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in nohf hf1 base; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in --e2e --c3 ""; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"], d["cand_full"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done

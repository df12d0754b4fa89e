#!/bin/bash
# round-4: per-simulation outcome records (SimCtrl) under the consolidation tests and PMC, then the
# CM bisection: round-3 library, this tree, va (free-key words 1), vb (round-4 wave-kernel changes
# compiled out), vc (both)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4k
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_consolidation.py tests/test_consolidation_general.py tests/test_e2e_scenarios.py tests/test_volumes.py tests/test_min_values.py tests/test_multi_shard.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in r3 base va vb vc; do
    lib=libgpusched_$v.so
    [ "$v" = base ] && lib=libgpusched.so
    for w in "" --c5; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"], d["sorts_generic"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done
SKIP_KT=1 LEGS="c4_e2e c4_mixed c4" TRAFFIC=traffic_r4k.json bash tools/profile_round.sh > $O/prof.log 2>&1 || exit 1
cp $R/gpurun_out/prof/traffic_r4k.json $O/

#!/bin/bash
# round-4: wave kernel split into narrow / wide option-row instantiations:
# the whole GPU suite, the CM / e2e / C5 timings against round 3, then the
# consolidation traffic with NodeClaim hostname rows zero at rest
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4o
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in r3 base; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in "" --e2e --c5 --c3; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done
SKIP_KT=1 LEGS="c4_e2e c4_mixed" TRAFFIC=traffic_r4o.json bash tools/profile_round.sh > $O/prof.log 2>&1 || exit 1
cp $R/gpurun_out/prof/traffic_r4o.json $O/

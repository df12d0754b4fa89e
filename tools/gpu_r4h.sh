#!/bin/bash
# round-4 same-session A/B of FFD builds: the round-3 library (r3), this tree (base), the counter
# experiments (noctr: no instrumentation counters, ctrlds: counters as LDS atomics), then the
# generic sort's parts (sorttl timeline build) on e2e and CM
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4h
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in r3 base noctr ctrlds; do
    lib=libgpusched_$v.so
    [ "$v" = base ] && lib=libgpusched.so
    for w in "" --c3 --e2e --c5; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"], d["sorts_generic"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done
for w in --e2e ""; do
  GPUSCHED_LIB=libgpusched_sorttl.so timeout -k 10 150 python3 tools/ffd_diag.py $w --tl --sorttl > $O/sorttl$w.json 2>&1 || exit 1
  head -c 600 $O/sorttl$w.json; echo
done

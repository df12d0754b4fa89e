#!/bin/bash
# round-4 bisection of the CM FFD time: same-session A/B of the round-3 library, this tree, and
# this tree with one round-4 change compiled out each (noaddl, noxl, nomask, nouni)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4j
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for v in r3 base noaddl noxl nomask nouni; do
    lib=libgpusched_$v.so
    [ "$v" = base ] && lib=libgpusched.so
    for w in "" --e2e; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"], d["sorts_generic"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done

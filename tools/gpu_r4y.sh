#!/bin/bash
# round-4: the wave kernel compiled with other machine-scheduler strategies
# (s1 max-ilp, s2 max-memory-clause) and at -O2 (s3): CM / e2e / C3 / C5
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4y
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in base s1 s2 s3; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in "" --e2e --c3 --c5; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done

#!/bin/bash
# round-4: CM with the wave kernel compiled for narrow option rows (W <= 4) and
# free-key words 1 / sort toggles off, against round 3 and this tree
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4n
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for v in r3 base vc n1 n2 n3; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])') || exit 1
    echo "$rep $v $ms" | tee -a $O/ab.txt
  done
done

#!/bin/bash
# round-4: the wave scan's fast accept for hostname-only topology pods
# (VF_HOSTFA; nohf = without; hfu = its check unrolled): e2e /
# C3 / CM
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4ai
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in nohf base hfu; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in --e2e --c3 ""; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"], d["cand_full"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done

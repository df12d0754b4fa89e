#!/bin/bash
# A/B of wave-kernel builds on C1 / C2 / e2e / CM (FFD device ms), same session:
# VARIANTS = libgpusched_<v>.so names (base = libgpusched.so)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for w in --c1 --c2 --e2e ""; do
  for v in ${VARIANTS:-} base; do
    lib=libgpusched_$v.so
    [ "$v" = base ] && lib=libgpusched.so
    ms=$(GPUSCHED_LIB=$lib timeout -k 10 120 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().split("\n")[-1]); print(round(d["ffd_ms"],2), d["claims"], d["sorts_generic"])')
    echo "${w:---cm} $v $ms"
  done
done

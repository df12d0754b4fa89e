#!/bin/bash
# FFD wave-kernel variants, same session: device ms on CM / C3 / e2e per
# library (VARIANTS = libgpusched_<v>.so names; base = libgpusched.so), then
# the timeline build's cycles per pod-loop segment (TL=1)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
for v in ${VARIANTS:-base}; do
  lib=libgpusched_$v.so
  [ "$v" = base ] && lib=libgpusched.so
  for w in "" --c3 --e2e; do
    ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"], d["cand_evals"])')
    echo "$v ${w:-cm} $ms" | tee -a $O/variants.txt
  done
done
if [ -n "${TL:-}" ]; then
  for w in "" --c3 --e2e; do
    GPUSCHED_LIB=libgpusched_tl.so timeout -k 10 150 python3 tools/ffd_diag.py $w --tl | tee -a $O/variants_tl.txt
  done
fi

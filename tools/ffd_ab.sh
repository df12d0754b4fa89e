#!/bin/bash
# A/B of wave-kernel experiment builds (csrc: make wavex V=<name> X=...):
# CM Solve device ms per build, 3 runs each, same session
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in ${VARIANTS:-} base; do
  lib=libgpusched_$v.so
  [ "$v" = base ] && lib=libgpusched.so
  for k in 1 2 3; do
    ms=$(GPUSCHED_LIB=$lib timeout -k 10 120 python3 $R/tools/ffd_diag.py | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])')
    echo "$v $ms"
  done
done

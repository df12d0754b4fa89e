#!/bin/bash
# Same-session A/B of FFD device ms per workload for diagnostic builds:
# LIBS="libgpusched.so libgpusched_x.so" CONFIGS="--c1 --c2 --c3 --e2e cm"
set -euo pipefail
for k in 1 2; do
  for lib in ${LIBS:-libgpusched.so}; do
    for c in ${CONFIGS:---c1 --c2 cm}; do
      [ "$c" = cm ] && c=""
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 120 python3 tools/ffd_diag.py $c | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],2), d["claims"], d["sorts_generic"])')
      echo "$lib ${c:-cm} $ms"
    done
  done
done

#!/bin/bash
# A/B of feasibility-kernel experiment builds (csrc: make kx V=<name> X=...)
# on the C5 static matrix: kernel ms per build, same session.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
for v in ${VARIANTS:-} base; do
  lib=libgpusched_$v.so
  [ "$v" = base ] && lib=libgpusched.so
  ms=$(GPUSCHED_LIB=$lib timeout -k 10 120 python3 $R/bench.py --only c5 --steps 10 --warmup 2 --no-cpu-baseline \
       | python3 -c 'import json,sys; d=json.load(sys.stdin)["stress"]; print(d["kernel_ms"], d["ms_per_step"])')
  echo "$v $ms"
done

#!/bin/bash
# Same-session A/B of the consolidation simulation kernel per leg:
# LIBS="libgpusched.so libgpusched_x.so" LEGS="c4 c4_mixed c4_multi"
set -euo pipefail
for k in 1 2; do
  for lib in ${LIBS:-libgpusched.so}; do
    for leg in ${LEGS:-c4 c4_mixed c4_multi}; do
      r=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 bench.py --only $leg --steps 10 --warmup 2 --latency-steps 0 --no-cpu-baseline |
        python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); c=d.get("consolidation_legs",{}); c=next(iter(c.values())) if c else d.get("consolidation",{}); print(c["kernel_ms"]["sim"], c["ms_per_sweep"], c.get("decisions"))')
      echo "$lib $leg $r"
    done
  done
done

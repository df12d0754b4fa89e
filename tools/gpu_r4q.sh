#!/bin/bash
# round-4: the narrow simulation shape at 2 waves per SIMD (no VGPR spills,
# 4 workgroups per CU) against 3 (spills, 6 per CU): consolidation timings and
# write traffic (after the taint-class parity tests)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4q
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_taint_classes.py tests/test_topology.py tests/test_gpu_parity.py tests/test_consolidation.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in base w2; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for leg in c4 c4_mixed c4_e2e; do
      GPUSCHED_LIB=$lib timeout -k 10 200 python3 bench.py --only $leg --no-cpu-baseline --steps 10 --warmup 2 --detail-json $O/${v}_${leg}_$rep.json > $O/${v}_${leg}_$rep.out 2>&1 || exit 1
      python3 -c "
import json,sys; d=json.load(open('$O/${v}_${leg}_$rep.json')); l=d['consolidation_legs']['$leg']
print('$rep $v $leg', l['kernel_ms'], l['ms_per_sweep'])" | tee -a $O/ab.txt
    done
  done
done
export GPUSCHED_LIB=libgpusched_w2.so
SKIP_KT=1 LEGS="c4 c4_mixed c4_e2e" TRAFFIC=traffic_w2.json bash tools/profile_round.sh > $O/prof.log 2>&1 || exit 1
cp $R/gpurun_out/prof/traffic_w2.json $O/

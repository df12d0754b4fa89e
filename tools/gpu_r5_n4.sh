#!/bin/bash
# round 5: the narrow simulation shape at 4 waves per SIMD (128 registers, spills,
# 8 workgroups per CU) against 3 (168 registers, 6 per CU), same session
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_n4
mkdir -p $O
cd $R
for rep in 1 2; do
for lib in libgpusched.so libgpusched_n4.so; do
for leg in c4 c4_mixed c4_multi c4_e2e; do
  GPUSCHED_LIB=$lib timeout -k 10 300 python3 bench.py --only $leg --steps 10 --warmup 2 --latency-steps 0 --no-cpu-baseline --detail-json $O/d_${leg}_${lib}.json > /dev/null 2> $O/e_${leg}_${lib}.err || exit 1
  python3 -c "import json;d=json.load(open('$O/d_${leg}_${lib}.json'))['consolidation_legs']['$leg'];print('$rep $lib $leg', d['ms_per_sweep'], d['kernel_ms'])"
done
done
done
GPUSCHED_LIB=libgpusched_n4.so timeout -k 10 600 python -u -m pytest tests/test_consolidation.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -2 $O/tests.log

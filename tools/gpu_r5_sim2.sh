#!/bin/bash
# simulation queue arrays in LDS: A/B (GS_SIM_LDS=0/1) of the C4 legs
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_sim2
mkdir -p $O
cd $R
for ab in 0 1 0 1; do
for leg in c4 c4_mixed c4_multi c4_e2e c4_e2e_multi; do
  GS_SIM_DEBUG=1 GS_SIM_LDS=$ab timeout -k 10 300 python3 bench.py --only $leg --steps 10 --warmup 2 --latency-steps 0 --no-cpu-baseline --detail-json $O/detail_$leg.json > $O/bench_$leg.out 2> $O/bench_${leg}_$ab.err || exit 1
  python3 -c "import json;d=json.load(open('$O/detail_$leg.json'))['consolidation_legs']['$leg'];print('$ab $leg', d['ms_per_sweep'], d['kernel_ms'])"
done
done
grep -h "sim plan" $O/*.err | sort | uniq | head

#!/bin/bash
# round 5: simulation sweep time against the persistent grid's workgroups per
# CU (GS_SIM_PER_CU caps them; unset = the occupancy limit), same session
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_percu
mkdir -p $O
cd $R
for rep in 1 2; do
for pc in 0 4 3 2; do
for leg in c4 c4_mixed c4_e2e; do
  if [ $pc = 0 ]; then unset GS_SIM_PER_CU; else export GS_SIM_PER_CU=$pc; fi
  timeout -k 10 300 python3 bench.py --only $leg --steps 10 --warmup 2 --latency-steps 0 --no-cpu-baseline --detail-json $O/d_${leg}_$pc.json > /dev/null 2> $O/e_${leg}_$pc.err || exit 1
  python3 -c "import json;d=json.load(open('$O/d_${leg}_$pc.json'))['consolidation_legs']['$leg'];print('$rep per_cu=$pc $leg', d['ms_per_sweep'], d['kernel_ms']['sim'])"
done
done
done

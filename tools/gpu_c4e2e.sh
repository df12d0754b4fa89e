#!/bin/bash
# c4_e2e consolidation legs: timing, FETCH / WRITE passes, then the
# consolidation parity suites
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --only c4_e2e --steps 3 --warmup 1 --no-cpu-baseline > $O/c4e2e.json 2> $O/c4e2e.err
cd /tmp
export TMPDIR=/tmp
for leg in c4_e2e c4_e2e_multi; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf_$leg -o fetch -- python3 $R/bench.py --only $leg --steps 1 --warmup 0 --latency-steps 0 --no-cpu-baseline > /dev/null 2> $O/pf_$leg.err
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw_$leg -o write -- python3 $R/bench.py --only $leg --steps 1 --warmup 0 --latency-steps 0 --no-cpu-baseline > /dev/null 2> $O/pw_$leg.err
  python3 $R/tools/pmc_traffic.py $leg $O/pf_$leg/fetch_counter_collection.csv $O/pw_$leg/write_counter_collection.csv $O/traffic_c.json
done
cd $R
timeout -k 10 600 python -u -m pytest tests/test_consolidation.py tests/test_consolidation_general.py tests/test_e2e_scenarios.py tests/test_multi_shard.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/par.log 2>&1
tail -2 $O/par.log

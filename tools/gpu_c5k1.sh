#!/bin/bash
# K1 at C5: stress-leg timing, a FETCH_SIZE pass, then the parity suites the
# static matrix and the Solve share
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --only c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/c5.json 2> $O/c5.err
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c5f -o fetch -- python3 $R/bench.py --only c5 --steps 1 --warmup 0 --latency-steps 0 --no-cpu-baseline > /dev/null 2> $O/c5f.err
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_multi_shard.py tests/test_min_values.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/par.log 2>&1
tail -2 $O/par.log

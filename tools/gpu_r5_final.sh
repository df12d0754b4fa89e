#!/bin/bash
# round 5 end: the whole GPU suite and smoke, then the default bench, each
# under its own time limit
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_final
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu_all.log 2>&1
tail -3 $O/pytest_gpu_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -3 $O/smoke.log
timeout -k 10 600 python -u bench.py --detail-json $O/bench_detail.json > $O/bench.out 2> $O/bench.err
tail -c 700 $O/bench.out

#!/bin/bash
# round-4 first pass: the new e2e scenarios + multi-shard tests, then the default bench (compact headline)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_e2e_scenarios.py tests/test_multi_shard.py -m gpu -v --timeout 120 --timeout-method thread > $O/r4a_tests.log 2>&1
tail -5 $O/r4a_tests.log
timeout -k 10 480 python bench.py --detail-json $O/r4a_bench_detail.json > $O/r4a_bench.out 2> $O/r4a_bench.err
tail -c 300 $O/r4a_bench.out; echo
tail -1 $O/r4a_bench.out | wc -c

#!/bin/bash
# round-3 GPU pass: the whole GPU suite, smoke, then the default bench line
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/r3_all.log 2>&1
tail -3 $O/r3_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r3_smoke.log 2>&1
cat $O/r3_smoke.log
timeout -k 10 420 python bench.py > $O/r3_bench.json 2> $O/r3_bench.err
head -c 400 $O/r3_bench.json; echo

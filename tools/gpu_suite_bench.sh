#!/bin/bash
# whole GPU suite, smoke, then the default bench line (each step time-limited;
# the chain stops at the first failure)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-r3}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/${TAG}_all.log 2>&1
tail -3 $O/${TAG}_all.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
cat $O/${TAG}_smoke.log
timeout -k 10 700 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err
head -c 300 $O/${TAG}_bench.json; echo

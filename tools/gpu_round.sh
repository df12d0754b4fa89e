#!/bin/bash
# One GPU-box pass: parity tests, smoke, the default bench line, then the
# rocprofv3 evidence (tools/profile_round.sh).  Every GPU step has its own
# time limit and the chain stops at the first failure.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err
head -c 600 $O/bench.json; echo
if [ "${1:-}" = "prof" ]; then
  bash $R/tools/profile_round.sh
fi

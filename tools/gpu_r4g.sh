#!/bin/bash
# round-4: whole GPU suite on the new tree, FFD timings, consolidation PMC traffic, then the default bench
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4g
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for w in --e2e "" --c3 --c5; do
  timeout -k 10 150 python3 tools/ffd_diag.py $w > $O/diag$w.json 2>&1 || exit 1
  GPUSCHED_LIB=libgpusched_tl.so timeout -k 10 150 python3 tools/ffd_diag.py $w --tl > $O/tl$w.json 2>&1 || exit 1
  echo "diag $w: $(head -c 100 $O/diag$w.json)"
done
SKIP_KT=1 LEGS="c4_e2e c4_mixed c4 c4_e2e_multi c4_multi c5" TRAFFIC=traffic_r4g.json bash tools/profile_round.sh > $O/prof.log 2>&1 || exit 1
cp $R/gpurun_out/prof/traffic_r4g.json $O/
timeout -k 10 600 python bench.py --detail-json $O/bench_detail.json > $O/bench.out 2> $O/bench.err
rc=$?; tail -c 300 $O/bench.out; exit $rc

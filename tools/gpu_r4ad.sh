#!/bin/bash
# round-4: wide-row scans also gather the next chunk's codes (pf2) vs order
# words only (this tree): C5 digest + parity, C5 timings; PMC traffic of the
# e2e and c4_e2e_multi legs
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4ad
mkdir -p $O
cd $R
GPUSCHED_LIB=libgpusched_pf2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_free_keys_wide.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base pf2; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py --c5 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])') || exit 1
    echo "$rep $v c5 $ms" | tee -a $O/ab.txt
  done
done
SKIP_KT=1 LEGS="e2e c4_e2e_multi" TRAFFIC=traffic_extra.json timeout -k 10 600 bash tools/profile_round.sh > $O/prof.log 2>&1 || exit 1
cp $R/gpurun_out/prof/traffic_extra.json $O/

#!/bin/bash
# round-4: wide exact checks with 1 / 2 / 4 chunks of 4 words per round trip
# (C5 Solve), digest parity at full size for the default (2)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4w
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_free_keys_wide.py tests/test_min_values.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in xc1 base xc4; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py --c5 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"])') || exit 1
    echo "$rep $v c5 $ms" | tee -a $O/ab.txt
  done
done

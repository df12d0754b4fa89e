#!/bin/bash
# round-4: which writes the simulation kernel issues (request counts and store instructions per launch)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4c
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -oE "(TCC|SQ|TCP|TA|TD)_[A-Z0-9_]+" $O/avail.txt | sort -u > $O/names.txt || true
for leg in c4_e2e c4; do
  for set in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES" "TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    tag=$(echo $set | tr ' ' '_' | cut -c1-40)
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/${leg}_$tag -o p -- \
      python3 $R/bench.py --only $leg --steps 1 --warmup 0 --latency-steps 0 --no-cpu-baseline --detail-json $O/d.json > /dev/null 2> $O/${leg}_$tag.err
    echo "$leg $set rc=$?"
  done
done
python3 - <<'PY'
import csv, glob, os, collections
O=os.environ.get("O") or "."
PY

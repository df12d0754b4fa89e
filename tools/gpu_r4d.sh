#!/bin/bash
# round-4: wave-sort parity (uniform-frame shortcut), e2e/C5 timelines, simulation write counters
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4d
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_wave_sort.py tests/test_rank.py tests/test_e2e_scenarios.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for w in --e2e "" --c3 --c2 --c5; do
  timeout -k 10 150 python3 tools/ffd_diag.py $w > $O/diag$w.json 2>&1 || exit 1
  GPUSCHED_LIB=libgpusched_tl.so timeout -k 10 150 python3 tools/ffd_diag.py $w --tl > $O/tl$w.json 2>&1 || exit 1
  echo "diag $w: $(head -c 300 $O/diag$w.json)"
done
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
for leg in c4_e2e c4; do
  for set in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/${leg}_$tag -o p -- \
      python3 $R/bench.py --only $leg --steps 1 --warmup 0 --latency-steps 0 --no-cpu-baseline --detail-json $O/d.json > /dev/null 2> $O/${leg}_$tag.err
    echo "$leg $set rc=$?"
  done
done

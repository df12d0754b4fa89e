#!/bin/bash
# round-4 end: whole GPU suite on this tree (scan walk split by the hostname
# fast accept), the A/B against the single walk (hf1) and without it (nohf),
# per-pop timelines, the default bench, then the CM kernel trace + stats
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4ak
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in nohf hf1 base; do
    lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
    for w in --e2e --c3 ""; do
      ms=$(GPUSCHED_LIB=$lib timeout -k 10 150 python3 tools/ffd_diag.py $w | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["ffd_ms"],1), d["claims"], d["cand_full"])') || exit 1
      echo "$rep $v ${w:-cm} $ms" | tee -a $O/ab.txt
    done
  done
done
for w in --e2e "" --c3 --c5; do
  GPUSCHED_LIB=libgpusched_tl.so timeout -k 10 150 python3 tools/ffd_diag.py $w --tl > $O/tl$w.json 2>&1 || exit 1
done
timeout -k 10 600 python bench.py --detail-json $O/bench_detail.json > $O/bench.out 2> $O/bench.err
rc=$?; tail -c 300 $O/bench.out; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cm -o kt -- python3 $R/bench.py --only cm --steps 5 --warmup 1 --latency-steps 0 --no-cpu-baseline > $O/bench_kt_cm.json 2> $O/kt_cm.err

#!/bin/bash
# round-4: topology parity (nodeTaintsPolicy Honor), then the CM regression by
# segment: timeline builds of this tree and of round 3, and SQ instruction
# counters of the two product libraries
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4l
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_topology.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in tl tlr3; do
    GPUSCHED_LIB=libgpusched_$v.so timeout -k 10 150 python3 tools/ffd_diag.py --tl > $O/tl_${v}_$rep.json || exit 1
    echo "$v $rep $(cat $O/tl_${v}_$rep.json)"
  done
done
for v in r3 base; do
  lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
  GPUSCHED_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d $O/pmc_$v -o pmc -- python3 tools/ffd_diag.py > $O/pmc_$v.log 2>&1 || exit 1
done
find $O -name "*counter_collection.csv" | head

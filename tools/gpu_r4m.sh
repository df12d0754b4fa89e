#!/bin/bash
# round-4: I-cache and issue counters of the CM wave kernel, round 3 vs this tree vs vc
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r4m
mkdir -p $O
cd $R
export TMPDIR=/tmp
for v in r3 base vc; do
  lib=libgpusched_$v.so; [ "$v" = base ] && lib=libgpusched.so
  GPUSCHED_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_IFETCH -d $O/pmc_$v -o pmc -- python3 tools/ffd_diag.py > $O/pmc_$v.log 2>&1 || exit 1
  tail -1 $O/pmc_$v.log
done

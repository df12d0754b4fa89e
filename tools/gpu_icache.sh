#!/bin/bash
# instruction-cache evidence for the wave kernel: available counters, then
# SQC instruction-cache hits / misses per library on the CM Solve
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/icache
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
for v in ${VARIANTS:-base}; do
  lib=libgpusched_$v.so
  [ "$v" = base ] && lib=libgpusched.so
  GPUSCHED_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM --output-format csv -d $O/$v -o pmc -- python3 $R/tools/ffd_diag.py > $O/$v.json 2> $O/$v.err
  echo "$v done"
done

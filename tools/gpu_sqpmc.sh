#!/bin/bash
# SQ instruction / stall counters of the wave Solve kernel on CM, two passes
# per library (VARIANTS: libgpusched_<v>.so, base = libgpusched.so)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sqpmc
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  lib=libgpusched_$v.so
  [ "$v" = base ] && lib=libgpusched.so
  GPUSCHED_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $O/${v}_a -o pmc -- python3 $R/tools/ffd_diag.py > $O/${v}_a.json 2> $O/${v}_a.err
  GPUSCHED_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/${v}_b -o pmc -- python3 $R/tools/ffd_diag.py > $O/${v}_b.json 2> $O/${v}_b.err
  echo "$v done"
done

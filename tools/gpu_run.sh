#!/bin/bash
# One parametrised GPU-box pass (replaces the per-experiment gpu_r4* / gpu_r5*
# scripts).  Every GPU step runs under its own time limit and the chain stops
# at the first failure (set -e).  Run from the repo root through gpurun:
#   gpurun -- bash tools/gpu_run.sh <tag> <step>...
# steps:
#   suite          whole -m gpu suite + smoke
#   tests:<expr>   pytest -m gpu -k <expr>
#   file:<path>    pytest -m gpu on one test file
#   bench          the default bench line (+ per-leg detail json)
#   only:<leg>     bench.py --only <leg> (5 steps)
#   ffd            tools/ffd_diag.py FFD device ms on cm / c3 / e2e / c2
#   prof           tools/profile_round.sh (kernel stats + PMC traffic)
#   sqpmc          SQ instruction / stall counters of the wave Solve on CM, two
#                  rocprofv3 passes per library (VARIANTS; base = libgpusched.so)
#   lib:<name>     use gpusched/libgpusched_<name>.so for the steps after it
#                  (lib:base: the default library again); their outputs carry _<name>
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?tag}
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
LS=
PYT="python -u -m pytest -m gpu -x -q --timeout 240 --timeout-method thread"
for step in "$@"; do
  case $step in
    suite)
      timeout -k 10 900 $PYT tests > $O/pytest_gpu_all.log 2>&1
      tail -3 $O/pytest_gpu_all.log
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      tail -3 $O/smoke.log ;;
    tests:*)
      k=${step#tests:}
      timeout -k 10 600 $PYT tests -k "$k" > $O/pytest_${k//[^a-zA-Z0-9_]/_}.log 2>&1
      tail -3 $O/pytest_${k//[^a-zA-Z0-9_]/_}.log ;;
    file:*)
      f=${step#file:}
      b=$(basename $f .py)
      timeout -k 10 600 $PYT $f > $O/pytest_$b.log 2>&1
      tail -3 $O/pytest_$b.log ;;
    bench)
      timeout -k 10 600 python -u bench.py --detail-json $O/bench_detail.json > $O/bench.out 2> $O/bench.err
      tail -c 700 $O/bench.out ;;
    only:*)
      leg=${step#only:}
      timeout -k 10 300 python -u bench.py --only $leg --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_$leg$LS.out 2> $O/bench_$leg$LS.err
      tail -c 400 $O/bench_$leg$LS.out ;;
    ffd)
      timeout -k 10 400 python -u tools/ffd_diag.py > $O/ffd_diag.txt 2>&1
      tail -20 $O/ffd_diag.txt ;;
    prof)
      bash tools/profile_round.sh ;;
    sqpmc)
      for v in ${VARIANTS:-} base; do
        lib=libgpusched_$v.so
        [ "$v" = base ] && lib=libgpusched.so
        (cd /tmp && TMPDIR=/tmp GPUSCHED_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $O/sq_${v}_a -o pmc -- python3 $R/tools/ffd_diag.py > $O/sq_${v}_a.json 2> $O/sq_${v}_a.err)
        (cd /tmp && TMPDIR=/tmp GPUSCHED_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/sq_${v}_b -o pmc -- python3 $R/tools/ffd_diag.py > $O/sq_${v}_b.json 2> $O/sq_${v}_b.err)
        echo "sqpmc $v done"
      done ;;
    lib:base)
      LS=_base
      unset GPUSCHED_LIB ;;
    lib:*)
      LS=_${step#lib:}  # output files of the steps after it carry the library's name
      export GPUSCHED_LIB=$R/karpenter-provider-ibm-cloud_amd/gpusched/libgpusched_${step#lib:}.so ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done

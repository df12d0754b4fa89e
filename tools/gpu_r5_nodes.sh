#!/bin/bash
# round 5: run mode with existing nodes once the node hint covers every node
# (GS_RUN_NODES) -- run-mode parity (CanAdd counters included), then the
# CM-onto-C4-nodes leg against the same library built without it
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_nodes
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_run_mode.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in libgpusched.so libgpusched_nonodes.so; do
    GPUSCHED_LIB=$lib timeout -k 10 400 python3 bench.py --only cm_c4 --steps 3 --warmup 1 --latency-steps 0 --no-cpu-baseline --detail-json $O/d_${lib}_$rep.json > /dev/null 2> $O/e_${lib}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$O/d_${lib}_$rep.json'))['configs']['CM_C4'];print('$rep $lib', d['ms_per_step'], d['device_kernel_ms'])"
  done
done
GPUSCHED_LIB=libgpusched.so timeout -k 10 400 python3 bench.py --only cm_c4 --steps 2 --warmup 1 --latency-steps 0 --detail-json $O/x.json > /dev/null 2> $O/x.err || exit 1
python3 -c "import json;d=json.load(open('$O/x.json'))['configs']['CM_C4'];print('cpu', d['cpu_baseline'])"

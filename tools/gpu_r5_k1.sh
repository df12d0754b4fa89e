#!/bin/bash
# round 5, K1 at C5: the cheapest-offering search over rank blocks (GS_K1_BLOCKS) against the list walk
# lanes per (variant, template) pair capped below the row width (GS_K1_LPMAX) --
# parity of the static matrix, then a same-session A/B of the stress leg
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r5_k1
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_shard.py tests/test_min_values.py tests/test_catalog_ingest.py tests/test_create_filter.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in libgpusched.so libgpusched_scan.so; do
    GPUSCHED_LIB=$lib timeout -k 10 200 python3 bench.py --only c5 --steps 10 --warmup 2 --latency-steps 0 --no-cpu-baseline --detail-json $O/d_${lib}_$rep.json > /dev/null 2> $O/e_${lib}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('$O/d_${lib}_$rep.json'))['stress'];print('$rep $lib', d['kernel_ms'], d.get('ms_per_step'), d.get('cpu_baseline',{}) and '', d['roofline']['frac'])"
  done
done
# the capped variants' static matrix against the oracle on a C5 sample (bench cpu_baseline)
for lib in libgpusched.so; do
  GPUSCHED_LIB=$lib timeout -k 10 300 python3 bench.py --only c5 --steps 3 --warmup 1 --latency-steps 0 --detail-json $O/x_${lib}.json > /dev/null 2> $O/x_${lib}.err || exit 1
  python3 -c "import json;d=json.load(open('$O/x_${lib}.json'))['stress'];print('$lib', d['kernel_ms'], d['cpu_baseline'])"
done

#!/bin/bash
# library multi-GPU: sharded-context tests and the C5 stress leg (library_shards)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_multi_shard.py tests/test_gpu_parity.py -k "shard" -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/r3_multi.log 2>&1
tail -3 $O/r3_multi.log
timeout -k 10 300 python -u bench.py --only c5 --no-cpu-baseline --steps 5 --warmup 2 > $O/r3_c5.json 2> $O/r3_c5.err
python -c "import json;d=json.load(open('$O/r3_c5.json'))['stress'];print({k:d[k] for k in ('kernel_ms','ms_per_step','library_shards','shards_equal_whole')})"

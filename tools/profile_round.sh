#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats of the bench, then
# FETCH_SIZE and WRITE_SIZE in passes of their own (MI355X_MICROARCH.md
# "HBM" / "rocprofv3 PMC slots").  Run on the GPU box from the repo root.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_kt.json 2> $O/kt.err
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_fetch.json 2> $O/fetch.err
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/bench_write.json 2> $O/write.err
python3 $R/tools/kernel_phases.py $O/kt/kt_kernel_trace.csv > $O/phases.json
python3 $R/tools/pmc_traffic.py $O/fetch/fetch_counter_collection.csv $O/write/write_counter_collection.csv > $O/traffic.json
find $O -name "*.csv" | head -50

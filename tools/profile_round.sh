#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats of the whole bench,
# then FETCH_SIZE and WRITE_SIZE in passes of their own per bench leg
# (MI355X_MICROARCH.md "HBM" / "rocprofv3 PMC slots").  Run on the GPU box
# from the repo root; LEGS overrides the leg list.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
LEGS=${LEGS:-"cm c3 c4 c4_mixed c4_e2e c4_multi c5"}
if [ -z "${SKIP_KT:-}" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- \
    python3 $R/bench.py --steps 3 --warmup 1 --latency-steps 1 --no-cpu-baseline > $O/bench_kt.json 2> $O/kt.err
  echo "kernel trace done"
  # CM alone: the ffdw average in its stats is the headline leg's kernel only
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cm -o kt -- \
    python3 $R/bench.py --only cm --steps 5 --warmup 1 --latency-steps 0 --no-cpu-baseline > $O/bench_kt_cm.json 2> $O/kt_cm.err
  echo "cm kernel trace done"
fi
TJ=$O/${TRAFFIC:-traffic.json}
rm -f $TJ
for leg in $LEGS; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$leg -o fetch -- \
    python3 $R/bench.py --only $leg --steps 1 --warmup 0 --latency-steps 0 --no-cpu-baseline > $O/bench_fetch_$leg.json 2> $O/fetch_$leg.err
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$leg -o write -- \
    python3 $R/bench.py --only $leg --steps 1 --warmup 0 --latency-steps 0 --no-cpu-baseline > $O/bench_write_$leg.json 2> $O/write_$leg.err
  python3 $R/tools/pmc_traffic.py $leg $O/fetch_$leg/fetch_counter_collection.csv $O/write_$leg/write_counter_collection.csv $TJ
  echo "pmc $leg done"
done
cat $TJ

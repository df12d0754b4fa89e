#!/bin/bash
# round-4 record: rocprofv3 kernel trace + stats of the bench and of CM alone,
# FETCH_SIZE / WRITE_SIZE passes per leg
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LEGS="cm c3 c5 c4 c4_mixed c4_e2e c4_multi" TRAFFIC=traffic.json timeout -k 10 1100 bash tools/profile_round.sh > gpurun_out/prof_r4ac.log 2>&1
rc=$?; tail -3 gpurun_out/prof_r4ac.log; exit $rc

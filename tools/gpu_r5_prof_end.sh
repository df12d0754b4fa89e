#!/bin/bash
# round 5 end: rocprofv3 kernel trace of the bench and of CM alone, and
# FETCH_SIZE / WRITE_SIZE passes for CM and C3 into traffic_end.json
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
LEGS="cm c3" TRAFFIC=traffic_end.json bash tools/profile_round.sh

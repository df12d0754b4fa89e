#!/bin/bash
# round-end pass: the round-3 suite / smoke / bench, then a same-session A/B
# of an experiment build against the shipped library
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_round3.sh
VARIANTS="${AB:-base}" bash tools/gpu_variants.sh

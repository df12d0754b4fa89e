#!/bin/bash
# FFD build variants on the GPU box (diagnostic): rebuild ffd.o with a macro
# set, relink, time the CM Solve
set -e
cd $GRAFT_REPO_ROOT/karpenter-provider-ibm-cloud_amd/csrc
for F in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $F -c -o ffd.o ffd.hip 2>/dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../gpusched/libgpusched.so kernels.o ffd.o encode.o capi.o consolidate.o rank.o
  echo "== $F"
  timeout -k 10 120 python -u $GRAFT_REPO_ROOT/tools/ffd_diag.py | cut -c1-200
done
rm -f ffd.o

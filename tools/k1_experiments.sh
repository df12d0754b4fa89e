#!/bin/bash
# K1 ablations on the GPU box (diagnostic only): rebuild kernels.o with a
# macro set, relink, time the C5 feasibility kernel
set -e
cd $GRAFT_REPO_ROOT/karpenter-provider-ibm-cloud_amd/csrc
for F in "" "-DK1_NO_SCAN" "-DK1_NO_NFO" "-DK1_NO_SCAN -DK1_NO_NFO"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $F -c -o kernels.o kernels.hip
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../gpusched/libgpusched.so kernels.o ffd.o encode.o capi.o consolidate.o
  echo "== $F"
  timeout -k 10 120 python -u $GRAFT_REPO_ROOT/tools/c5_diag.py 200000 | grep feas_kernel
done

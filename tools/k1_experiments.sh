#!/bin/bash
# K1 ablations on the GPU box (diagnostic only): rebuild kernels.o with a
# macro set, relink, time the C5 feasibility kernel; then one SQ counter pass
# of the default build
set -e
cd $GRAFT_REPO_ROOT/karpenter-provider-ibm-cloud_amd/csrc
build() {
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $1 -c -o kernels.o kernels.hip 2>/dev/null
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../gpusched/libgpusched.so kernels.o ffd.o encode.o capi.o consolidate.o
}
for F in ${K1_VARIANTS:-"-DK1_NOP"}; do
  build "$F"
  echo "== $F"
  timeout -k 10 120 python -u $GRAFT_REPO_ROOT/tools/c5_diag.py 200000 | grep feas_kernel
done
build ""
if [ -n "$K1_PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 90 rocprofv3 --pmc $K1_PMC --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/k1pmc -o k1 -- \
    python3 $GRAFT_REPO_ROOT/tools/c5_diag.py 200000
fi

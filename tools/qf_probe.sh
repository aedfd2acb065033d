#!/bin/bash
# Timing probes of qf_rev_kernel (qf_kernel.hpp QF_PROBE / QF_PREFETCH_N): tu_hess.hip rebuilt with the given defines
# and linked with the cached objects of the product build (build/obj) into tools/probe/lib_<tag>.so. Numerically
# meaningless for QF_PROBE > 0; use with SIREN_AMD_LIB. usage: bash tools/qf_probe.sh <tag> "<-D flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1
mkdir -p $R/tools/probe $R/build/probe_$TAG
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -pragma-unroll-threshold=1000000 $2 -c \
  -I $R/include -o $R/build/probe_$TAG/tu_hess.o $R/siren_amd/csrc/tu_hess.hip
objs=$(ls $R/build/obj/*.o | grep -v '/tu_hess\.')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/probe/lib_$TAG.so $objs $R/build/probe_$TAG/tu_hess.o \
  -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
echo built tools/probe/lib_$TAG.so

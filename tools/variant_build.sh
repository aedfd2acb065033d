#!/bin/bash
# A/B library variants (not product builds): rebuild the given translation units with extra flags, link them with the
# cached objects of every other TU (build/obj, from the last build()) into tools/probe/lib_<tag>.so. Use on the GPU box
# with SIREN_AMD_LIB=tools/probe/lib_<tag>.so.   usage: tools/variant_build.sh <tag> "<flags>" tu_a tu_b ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=$1; FLAGS=$2; shift 2
O=$R/build/var_$TAG
mkdir -p $O $R/tools/probe
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -pragma-unroll-threshold=1000000 $FLAGS"
objs=""
skip=""
for tu in "$@"; do
  while [ $(jobs -r | wc -l) -ge ${VB_JOBS:-6} ]; do wait -n; done
  /opt/rocm/bin/hipcc $FL -c -I $R/include -o $O/$tu.o $R/siren_amd/csrc/$tu.hip &
  objs="$objs $O/$tu.o"; skip="$skip $tu"
done
wait
for o in $R/build/obj/*.o; do
  b=$(basename $o); b=${b%%.*}
  case " $skip " in *" $b "*) ;; *) objs="$objs $o";; esac
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/probe/lib_$TAG.so $objs -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
echo built $R/tools/probe/lib_$TAG.so

#!/bin/bash
# Timing probes (not a product build): libsiren_amd.so with -DSIREN_PROBE=<level> (jet_kernel.hpp: 1 = no epilogue
# arithmetic, 2 = also no tile stores) into tools/probe/libsiren_probe<level>.so; results are numerically meaningless,
# the kernel times tell where the time goes. Use with SIREN_AMD_LIB=tools/probe/libsiren_probe<level>.so.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
LVL=${1:-1}
O=$R/build/probe$LVL
mkdir -p $O $R/tools/probe
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mllvm -pragma-unroll-threshold=1000000 -DSIREN_PROBE=$LVL $EXTRA"
objs=""
TUS=$(cd $R && python -c "import __graft_entry__ as g; print(' '.join(t[:-4] for t in g.TUS))")
for tu in $TUS; do
  /opt/rocm/bin/hipcc $FL -c -I $R/include -o $O/$tu.o $R/siren_amd/csrc/$tu.hip &
  objs="$objs $O/$tu.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/probe/libsiren_probe$LVL.so $objs -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
echo built $R/tools/probe/libsiren_probe$LVL.so

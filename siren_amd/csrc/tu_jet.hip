// tu_jet.hip — W4s: backward of the fused Laplacian (jet_kernel.hpp).
#include "jet_kernel.hpp"
#include "launch.h"

namespace siren {

void launch_jet_store(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* glap,
                      float* gx, int d, int o, int lh, float w0, float w, float* spill, float* abuf, float* dbuf,
                      int64_t n_pad) {
    hipLaunchKernelGGL(jet_store_kernel, grid, dim3(THREADS), 0, st, ws, x, n, glap, gx, d, o, lh, w0, w, spill, abuf,
                       dbuf, n_pad);
}

void launch_small_jet(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x,
                      const float* glap, int64_t n, int64_t n_pad, int64_t tps, float* partial, int64_t P, int d,
                      int o, int lh) {
    hipLaunchKernelGGL(small_jet_kernel, grid, dim3(THREADS), 0, st, abuf, dbuf, x, glap, n, n_pad, tps, partial, P,
                       d, o, lh);
}

}  // namespace siren

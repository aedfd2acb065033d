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


}  // namespace siren

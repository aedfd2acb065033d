// tu_wide_jet.hip — second order at hidden width 512 (wide_jet_kernel.hpp: two-stream jet).
#include "launch.h"
#include "wide_jet_kernel.hpp"

namespace siren {

void launch_wide_jet2(dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* gy,
                      const float* u, int64_t n, int d, int o, int lh, float w0, float w, float* gx, float* ydot,
                      float* spill, float* abuf, float* dbuf, int64_t n_pad) {
    hipLaunchKernelGGL(wide_jet2_kernel, grid, dim3(THREADS), 0, st, ws, x, v, gy, u, n, d, o, lh, w0, w, gx, ydot,
                       spill, abuf, dbuf, n_pad);
}

}  // namespace siren

// tu_wide_jet.hip — second order at hidden width 512 (wide_jet_kernel.hpp: two-stream jet).
#include "launch.h"
#include "wide_jet_kernel.hpp"

namespace siren {

void launch_wide_jet2(dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* gy,
                      const float* u, int64_t n, int d, int o, int lh, float w0, float w, float* gx, float* ydot,
                      float* spill, float* abuf, float* dbuf, int64_t n_pad) {
    hipLaunchKernelGGL(wide_jet_kernel<2>, grid, dim3(THREADS), 0, st, ws, x, v, (const float*)nullptr, gy, u, n, d,
                       o, lh, w0, w, gx, ydot, (float*)nullptr, spill, abuf, dbuf, n_pad);
}

void launch_wide_mix(dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* g,
                     const float* u, int64_t n, int d, int o, int lh, float w0, float w, float* gx, float* gv,
                     float* gu, float* spill, float* abuf, float* dbuf, int64_t n_pad) {
    hipLaunchKernelGGL(wide_jet_kernel<4>, grid, dim3(THREADS), 0, st, ws, x, v, g, (const float*)nullptr, u, n, d, o,
                       lh, w0, w, gx, gv, gu, spill, abuf, dbuf, n_pad);
}

}  // namespace siren

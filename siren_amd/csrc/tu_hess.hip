// tu_hess.hip — the Hessian node's forward (hess_kernel.hpp).
#include "hess_kernel.hpp"
#include "qf_kernel.hpp"
#include "launch.h"

namespace siren {

void launch_hess(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* u, int d, int o,
                 int lh, float w0, float w, float* hm, float* kept, float* y, float* gx) {
    if (kept != nullptr)
        hipLaunchKernelGGL(hess_kernel<true>, grid, dim3(THREADS), 0, st, ws, x, n, u, d, o, lh, w0, w, hm, kept, y,
                           gx);
    else
        hipLaunchKernelGGL(hess_kernel<false>, grid, dim3(THREADS), 0, st, ws, x, n, u, d, o, lh, w0, w, hm, kept, y,
                           gx);
}

void launch_qf_rev(int64_t ngroups, hipStream_t st, const float* ws, const float* x, int64_t n, const float* G,
                   const float* u, const float* kept, float* gx, float* gu, int d, int o, int lh, float w0, float w,
                   float* abuf, float* dbuf, int64_t n_pad) {
    hipLaunchKernelGGL(qf_rev_kernel, dim3((unsigned)(ngroups / WAVES)), dim3(THREADS), 0, st, ws, x, n, G, u, kept,
                       gx, gu, d, o, lh, w0, w, abuf, dbuf, n_pad);
}

}  // namespace siren

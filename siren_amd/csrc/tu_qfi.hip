// tu_qfi.hip — the kept Hessian-node backward with interleaved epilogues (qfi_kernel.hpp), 1..5 hidden layers.
#include "qfi_kernel.hpp"
#include "launch.h"

namespace siren {

void launch_qfi_rev(int64_t ngroups, hipStream_t st, const float* ws, const float* x, int64_t n, const float* G,
                    const float* u, const float* kept, float* gx, float* gu, int d, int o, int lh, float w0, float w,
                    float* abuf, float* dbuf, int64_t n_pad) {
    const dim3 grid((unsigned)(ngroups / WAVES)), block(THREADS);
    switch (lh) {
        case 1: hipLaunchKernelGGL(qfi_rev_kernel<1>, grid, block, 0, st, ws, x, n, G, u, kept, gx, gu, d, o, w0, w, abuf, dbuf, n_pad); break;
        case 2: hipLaunchKernelGGL(qfi_rev_kernel<2>, grid, block, 0, st, ws, x, n, G, u, kept, gx, gu, d, o, w0, w, abuf, dbuf, n_pad); break;
        case 3: hipLaunchKernelGGL(qfi_rev_kernel<3>, grid, block, 0, st, ws, x, n, G, u, kept, gx, gu, d, o, w0, w, abuf, dbuf, n_pad); break;
        case 4: hipLaunchKernelGGL(qfi_rev_kernel<4>, grid, block, 0, st, ws, x, n, G, u, kept, gx, gu, d, o, w0, w, abuf, dbuf, n_pad); break;
        default: hipLaunchKernelGGL(qfi_rev_kernel<5>, grid, block, 0, st, ws, x, n, G, u, kept, gx, gu, d, o, w0, w, abuf, dbuf, n_pad); break;
    }
}

}  // namespace siren

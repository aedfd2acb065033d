// tu_w3i_tt.hip — the interleaved second-order adjoint (w3i_kernel.hpp), THETA = true, KEPT = true (one translation unit
// per variant: each holds three fully unrolled kernels of ~190 KiB, compiled in parallel).
#include "launch.h"
#include "w3i_kernel.hpp"

namespace siren {

void launch_w3i_tt(dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* gy,
                   const float* u, float* ydot, int o, int64_t n, float* gx, float* spill, float* A, float* At, float* D,
                   float* Dt, int64_t n_pad, int d, int lh, float w0, float w, const float* kA, const float* kC,
                   int64_t ws_bs, int64_t spill_bs, int64_t buf_bs) {
#define SIREN_L(LHV)                                                                                                   \
    hipLaunchKernelGGL((w3i_kernel<LHV, true, true>), grid, dim3(THREADS), 0, st, ws, x, v, gy, u, ydot, o, n, gx, spill, \
                       A, At, D, Dt, n_pad, d, w0, w, kA, kC, ws_bs, spill_bs, buf_bs)
    switch (lh) {
        case 1: SIREN_L(1); break;
        case 2: SIREN_L(2); break;
        default: SIREN_L(3); break;
    }
#undef SIREN_L
}

}  // namespace siren

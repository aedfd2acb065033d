// tu_w3.hip — second-order adjoint kernels (W3).
#include "launch.h"
#include "siren_params.h"
#include "w3_kernel.hpp"

namespace siren {

void launch_w3(bool theta, dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* gy,
               const float* u, float* ydot, int o, int64_t n, float* gx, float* spill, float* A, float* At, float* D, float* Dt, int64_t n_pad, int d, int lh,
               float w0, float w) {
#define SIREN_L(LHV, TH)                                                                                      \
    hipLaunchKernelGGL((w3_kernel<LHV, TH>), grid, dim3(THREADS), 0, st, ws, x, v, gy, u, ydot, o, n, gx, spill, A, At, D, Dt, n_pad, \
                       d, w0, w)
    if (theta) {
        switch (lh) {
            case 1: SIREN_L(1, true); break;
            case 2: SIREN_L(2, true); break;
            default: SIREN_L(3, true); break;
        }
    } else {
        switch (lh) {
            case 1: SIREN_L(1, false); break;
            case 2: SIREN_L(2, false); break;
            default: SIREN_L(3, false); break;
        }
    }
#undef SIREN_L
}


}  // namespace siren

// tu_w3.hip — second-order adjoint kernels (W3).
#include "launch.h"
#include "siren_params.h"
#include "w3_kernel.hpp"

namespace siren {

// kA / kC non-null: the KEPT variant (primal a_l / cos from a stored forward; theta path uses kA as A)
void launch_w3(bool theta, dim3 grid, hipStream_t st, const float* ws, const float* x, const float* v, const float* gy,
               const float* u, float* ydot, int o, int64_t n, float* gx, float* spill, float* A, float* At, float* D,
               float* Dt, int64_t n_pad, int d, int lh, float w0, float w, const float* kA, const float* kC,
               unsigned long long* prof, int64_t ws_bs, int64_t spill_bs, int64_t buf_bs, bool serial) {
    const bool kept = kA != nullptr && kC != nullptr;
    if (!serial && prof == nullptr && lh <= MAX_LH_GRAD) {  // 4..5 hidden layers: the serial kernel's layer loops
#define SIREN_I(TK)                                                                                                 \
    launch_w3i_##TK(grid, st, ws, x, v, gy, u, ydot, o, n, gx, spill, A, At, D, Dt, n_pad, d, lh, w0, w, kA, kC, ws_bs, \
                    spill_bs, buf_bs)
        if (theta && kept)
            SIREN_I(tt);
        else if (theta)
            SIREN_I(tf);
        else if (kept)
            SIREN_I(ft);
        else
            SIREN_I(ff);
#undef SIREN_I
        return;
    }
#define SIREN_L(LHV, TH, KP)                                                                                    \
    hipLaunchKernelGGL((w3_kernel<LHV, TH, KP>), grid, dim3(THREADS), 0, st, ws, x, v, gy, u, ydot, o, n, gx, spill, A, \
                       At, D, Dt, n_pad, d, w0, w, kA, kC, prof, ws_bs, spill_bs, buf_bs)
#define SIREN_LH(TH, KP)                   \
    switch (lh) {                          \
        case 1: SIREN_L(1, TH, KP); break; \
        case 2: SIREN_L(2, TH, KP); break; \
        case 3: SIREN_L(3, TH, KP); break; \
        case 4: SIREN_L(4, TH, KP); break; \
        default: SIREN_L(5, TH, KP); break; \
    }
    if (theta && kept) {
        SIREN_LH(true, true);
    } else if (theta) {
        SIREN_LH(true, false);
    } else if (kept) {
        SIREN_LH(false, true);
    } else {
        SIREN_LH(false, false);
    }
#undef SIREN_LH
#undef SIREN_L
}

}  // namespace siren

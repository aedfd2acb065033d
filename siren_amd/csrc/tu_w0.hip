// tu_w0.hip — forward-only (W0) mode of the W1 kernel, 1..5 hidden layers.
#include "launch.h"
#include "w1_kernel.hpp"

namespace siren {

void launch_w0(dim3 grid, hipStream_t st, const FusedArgs& a) {
#define SIREN_L(LHV)                                                                                            \
    hipLaunchKernelGGL((w1_kernel<LHV, MODE_FWD>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, (const float*)nullptr, \
                       a.y, (float*)nullptr, a.d, a.o, a.w0, a.w, (float*)nullptr, (float*)nullptr, (int64_t)0,     \
                       a.ws_bstride)
    switch (a.lh) {
        case 1: SIREN_L(1); break;
        case 2: SIREN_L(2); break;
        case 3: SIREN_L(3); break;
        case 4: SIREN_L(4); break;
        default: SIREN_L(5); break;
    }
#undef SIREN_L
}

// MODE_FWDS: W0 + a_l tiles (a.abuf) and lane-major cos (a.dbuf) for the stored-forward W2 split
void launch_w0s(dim3 grid, hipStream_t st, const FusedArgs& a) {
    if (a.abuf == nullptr) {  // lane-major cos only
        launch_w1_notile(MODE_FWDS, grid, st, a);
        return;
    }
#define SIREN_L(LHV)                                                                                             \
    hipLaunchKernelGGL((w1_kernel<LHV, MODE_FWDS>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, (const float*)nullptr, \
                       a.y, (float*)nullptr, a.d, a.o, a.w0, a.w, a.abuf, a.dbuf, a.n_pad, a.ws_bstride)
    switch (a.lh) {
        case 1: SIREN_L(1); break;
        case 2: SIREN_L(2); break;
        case 3: SIREN_L(3); break;
        default: launch_w1_deep(MODE_FWDS, grid, st, a); break;
    }
#undef SIREN_L
}

}  // namespace siren

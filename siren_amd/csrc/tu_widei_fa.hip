// tu_widei_fa.hip — the hidden-512 stored-forward split with interleaved epilogues (widei_kernel.hpp): the forward half, 1..3 hidden layers.
#include "widei_kernel.hpp"
#include "launch.h"

namespace siren {

void launch_widei_fa(int lh, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill) {
#define SIREN_WI(LH)                                                                                                 \
    hipLaunchKernelGGL((widei_kernel<LH, MODE_FWDS>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, a.gy, a.y, a.gx,   \
                       a.d, a.o, a.w0, a.w, spill, a.abuf, a.dbuf, a.n_pad)
    switch (lh) {
        case 1: SIREN_WI(1); break;
        case 2: SIREN_WI(2); break;
        case 3: SIREN_WI(3); break;
        default: break;
    }
#undef SIREN_WI
}

}  // namespace siren

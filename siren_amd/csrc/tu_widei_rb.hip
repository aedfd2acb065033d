// tu_widei_rb.hip — the hidden-512 stored-forward split with interleaved epilogues (widei_kernel.hpp): the reverse half, 4..5 hidden layers.
#include "widei_kernel.hpp"
#include "launch.h"

namespace siren {

void launch_widei_rb(int lh, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill) {
#define SIREN_WI(LH)                                                                                                 \
    hipLaunchKernelGGL((widei_kernel<LH, MODE_REV>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, a.gy, a.y, a.gx,   \
                       a.d, a.o, a.w0, a.w, spill, a.abuf, a.dbuf, a.n_pad)
    switch (lh) {
        case 4: SIREN_WI(4); break;
        case 5: SIREN_WI(5); break;
        default: break;
    }
#undef SIREN_WI
}

}  // namespace siren

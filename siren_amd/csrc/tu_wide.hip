// tu_wide.hip — hidden width 512 kernels (wide_kernel.hpp).
#include "launch.h"
#include "wide_kernel.hpp"

namespace siren {

void launch_wide(int mode, dim3 grid, hipStream_t st, const FusedArgs& a, float* spill) {
#define SIREN_L(M)                                                                                              \
    hipLaunchKernelGGL((wide_kernel<M>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, a.gy, a.y, a.gx, a.d, a.o, \
                       a.lh, a.w0, a.w, a.final_sine, spill, a.abuf, a.dbuf, a.n_pad)
    if (mode == MODE_FWD)
        SIREN_L(MODE_FWD);
    else if (mode == MODE_STORE)
        SIREN_L(MODE_STORE);
    else if (mode == MODE_FWDS)
        SIREN_L(MODE_FWDS);
    else if (mode == MODE_REV)
        SIREN_L(MODE_REV);
    else
        SIREN_L(MODE_W1);
#undef SIREN_L
}

}  // namespace siren

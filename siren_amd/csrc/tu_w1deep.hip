// tu_w1deep.hip — the stored-split halves of the W1 kernel at 4..5 hidden layers (hidden 256): MODE_FWDS (forward +
// lane-major cos and a_l tiles) and MODE_REV (reverse GEMMs from the stored cos, delta tiles; tu_w1nt.hip without tiles). At these depths cos(w z_l) of
// every layer no longer fits the register file beside the accumulators, so W1 / W2 / the kept W3 run through HBM
// (siren_capi.hip deep()); one translation unit of its own so the fully unrolled bodies compile in parallel.
#include "launch.h"
#include "w1_kernel.hpp"

namespace siren {

void launch_w1_deep(int mode, dim3 grid, hipStream_t st, const FusedArgs& a) {
#define SIREN_L(LHV, M)                                                                                       \
    hipLaunchKernelGGL((w1_kernel<LHV, M>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, a.gy, a.y, a.gx, a.d, a.o, \
                       a.w0, a.w, a.abuf, a.dbuf, a.n_pad, a.ws_bstride)
    if (mode == MODE_FWDS) {
        if (a.lh == 4)
            SIREN_L(4, MODE_FWDS);
        else
            SIREN_L(5, MODE_FWDS);
    } else {
        if (a.lh == 4)
            SIREN_L(4, MODE_REV);
        else
            SIREN_L(5, MODE_REV);
    }
#undef SIREN_L
}

}  // namespace siren

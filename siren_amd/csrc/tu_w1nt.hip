// tu_w1nt.hip — the stored-split halves of the W1 kernel without tile stores (MODE_NOTILE): MODE_FWDS keeping only the
// lane-major cos (the 4..5-layer siren_forward_grad's forward half) and MODE_REV with gx only (siren_forward_grad /
// siren_forward_grad_store). Compile-time, so the slice loops count every epilogue store exactly (w1_kernel.hpp
// w1_allow); one translation unit of its own so the unrolled bodies compile in parallel with tu_w1 / tu_w1deep.
#include "launch.h"
#include "w1_kernel.hpp"

namespace siren {

void launch_w1_notile(int mode, dim3 grid, hipStream_t st, const FusedArgs& a) {
#define SIREN_L(LHV, M)                                                                                       \
    hipLaunchKernelGGL((w1_kernel<LHV, M | MODE_NOTILE>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, a.gy, a.y, \
                       a.gx, a.d, a.o, a.w0, a.w, a.abuf, a.dbuf, a.n_pad, a.ws_bstride)
#define SIREN_SW(M)                        \
    switch (a.lh) {                        \
        case 1: SIREN_L(1, M); break;      \
        case 2: SIREN_L(2, M); break;      \
        case 3: SIREN_L(3, M); break;      \
        case 4: SIREN_L(4, M); break;      \
        default: SIREN_L(5, M); break;     \
    }
    if (mode == MODE_FWDS) {
        SIREN_SW(MODE_FWDS);
    } else {
        SIREN_SW(MODE_REV);
    }
#undef SIREN_SW
#undef SIREN_L
}

}  // namespace siren

// tu_w1.hip — the W1 kernel (forward + vjp_x) and its STORE mode (W2 backward stage 1).
#include "launch.h"
#include "w1_kernel.hpp"

namespace siren {

void launch_w1(int mode, dim3 grid, hipStream_t st, const FusedArgs& a) {
#define SIREN_L(LHV, M)                                                                                       \
    hipLaunchKernelGGL((w1_kernel<LHV, M>), grid, dim3(THREADS), 0, st, a.ws, a.x, a.n, a.gy, a.y, a.gx, a.d, a.o, \
                       a.w0, a.w, a.abuf, a.dbuf, a.n_pad, a.ws_bstride)
    if (mode == MODE_STORE) {
        switch (a.lh) {
            case 1: SIREN_L(1, MODE_STORE); break;
            case 2: SIREN_L(2, MODE_STORE); break;
            default: SIREN_L(3, MODE_STORE); break;
        }
    } else if (mode == MODE_REV && a.dbuf == nullptr) {  // gx only
        launch_w1_notile(MODE_REV, grid, st, a);
    } else if (mode == MODE_REV) {  // a.abuf = lane-major cos from MODE_FWDS, a.dbuf = delta tiles
        switch (a.lh) {
            case 1: SIREN_L(1, MODE_REV); break;
            case 2: SIREN_L(2, MODE_REV); break;
            case 3: SIREN_L(3, MODE_REV); break;
            default: launch_w1_deep(MODE_REV, grid, st, a); break;
        }
    } else if (mode == (MODE_W1 | MODE_PROF)) {
        SIREN_L(3, MODE_W1 | MODE_PROF);
    } else if (mode == (MODE_W1 | MODE_O1S | MODE_D(2)) && a.lh == 3) {
        SIREN_L(3, MODE_W1 | MODE_O1S | MODE_D(2));
    } else if (mode == (MODE_W1 | MODE_O1S | MODE_D(3)) && a.lh == 3) {
        SIREN_L(3, MODE_W1 | MODE_O1S | MODE_D(3));
    } else if (mode == (MODE_W1 | MODE_O1S | MODE_D(2) | MODE_PROF) && a.lh == 3) {
        SIREN_L(3, MODE_W1 | MODE_O1S | MODE_D(2) | MODE_PROF);
    } else {
        switch (a.lh) {
            case 1: SIREN_L(1, MODE_W1); break;
            case 2: SIREN_L(2, MODE_W1); break;
            default: SIREN_L(3, MODE_W1); break;
        }
    }
#undef SIREN_L
}

}  // namespace siren

// tu_jet.hip — W4s: backward of the fused Laplacian (jet_kernel.hpp).
#include "jet_kernel.hpp"
#include "launch.h"

namespace siren {

#define NOF ((const float*)nullptr)
#define NUL ((float*)nullptr)

// ph: ws is the phase-scaled image (w1_ws; the jets run in revolutions, jet_kernel.hpp PH), else the unscaled one
void launch_jet_store(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* glap,
                      float* gx, int d, int o, int lh, float w0, float w, float* spill, float* abuf, float* dbuf,
                      int64_t n_pad, bool ph) {
#define SIREN_J(PHV)                                                                                                  \
    hipLaunchKernelGGL((jet_store_kernel<JET_BOTH, false, false, PHV>), grid, dim3(THREADS), 0, st, ws, x, n, glap, gx, \
                       d, o, lh, w0, w, spill, abuf, dbuf, n_pad, (float*)nullptr, (float*)nullptr, NOF, NOF, NOF, NUL, \
                       NUL)
    if (ph)
        SIREN_J(true);
    else
        SIREN_J(false);
#undef SIREN_J
}

// split form: phase 1 = forward jet with stores and outputs (y / gx / lap), phase 2 = seed + reverse from the stores
void launch_jet_phase(int phase, dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n,
                      const float* glap, float* gx, int d, int o, int lh, float w0, float w, float* spill, float* abuf,
                      float* dbuf, int64_t n_pad, float* y, float* lap, bool ph) {
#define SIREN_J(P, PHV)                                                                                               \
    hipLaunchKernelGGL((jet_store_kernel<P, false, false, PHV>), grid, dim3(THREADS), 0, st, ws, x, n, glap, gx, d, o, \
                       lh, w0, w, spill, abuf, dbuf, n_pad, y, lap, NOF, NOF, NOF, NUL, NUL)
    if (phase == JET_FWD) {
        if (ph)
            SIREN_J(JET_FWD, true);
        else
            SIREN_J(JET_FWD, false);
    } else {
        if (ph)
            SIREN_J(JET_REV, true);
        else
            SIREN_J(JET_REV, false);
    }
#undef SIREN_J
}

// third-order adjoint (backward of a Hessian-vector-product node): the mixed jet along (v, g), one launch
void launch_jet_mix(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* v,
                    const float* g, const float* u, float* gx, float* gv, float* gu, int d, int o, int lh, float w0,
                    float w, float* spill, float* abuf, float* dbuf, int64_t n_pad) {
    hipLaunchKernelGGL((jet_store_kernel<JET_BOTH, true>), grid, dim3(THREADS), 0, st, ws, x, n, NOF, gx, d, o, lh, w0,
                       w, spill, abuf, dbuf, n_pad, NUL, NUL, v, g, u, gv, gu);
}

// backward of a Hessian node recomputing its forward jet (QG: quadratic form G (n, d, d) per coordinate, tangents the
// coordinate axes, d <= 2); the kept-forward backward is qf_kernel.hpp (tu_hess.hip)
void launch_jet_quad(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, const float* G,
                     const float* u, float* gx, float* gu, int d, int o, int lh, float w0, float w, float* spill,
                     float* abuf, float* dbuf, int64_t n_pad) {
    hipLaunchKernelGGL((jet_store_kernel<JET_BOTH, true, true>), grid, dim3(THREADS), 0, st, ws, x, n, NOF, gx, d, o,
                       lh, w0, w, spill, abuf, dbuf, n_pad, NUL, NUL, NOF, NOF, u, NUL, gu, G);
}

}  // namespace siren

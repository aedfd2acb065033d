// tu_w4.hip — JET mode of the W1 kernel (W4: y, grad and Laplacian in one forward sweep), 1..5 hidden layers.
#include "launch.h"
#include "w1_kernel.hpp"

namespace siren {

void launch_w4(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, float* y, float* gx, float* lap,
               int d, int o, int lh, float w0, float w) {
#define SIREN_L(LHV)                                                                                             \
    hipLaunchKernelGGL((w1_kernel<LHV, MODE_JET>), grid, dim3(THREADS), 0, st, ws, x, n, (const float*)nullptr, y, \
                       gx, d, o, w0, w, lap, (float*)nullptr, (int64_t)0, (int64_t)0)
    switch (lh) {
        case 1: SIREN_L(1); break;
        case 2: SIREN_L(2); break;
        case 3: SIREN_L(3); break;
        case 4: SIREN_L(4); break;
        default: SIREN_L(5); break;
    }
#undef SIREN_L
}

// W4s split, forward half: W4 + the a-jet tiles (abuf) and the reverse's z-jet scratch (spill) of jet_store_kernel<
// JET_REV, PH>; ws the phase-scaled image; y / gx / lap nullable
void launch_w4s(dim3 grid, hipStream_t st, const float* ws, const float* x, int64_t n, float* y, float* gx, float* lap,
                float* abuf, float* spill, int64_t n_pad, int d, int o, int lh, float w0, float w) {
#define SIREN_L(LHV)                                                                                              \
    hipLaunchKernelGGL((w1_kernel<LHV, MODE_JETS>), grid, dim3(THREADS), 0, st, ws, x, n, (const float*)nullptr, y, \
                       gx, d, o, w0, w, abuf, spill, n_pad, (int64_t)0, lap)
    switch (lh) {
        case 1: SIREN_L(1); break;
        case 2: SIREN_L(2); break;
        case 3: SIREN_L(3); break;
        case 4: SIREN_L(4); break;
        default: SIREN_L(5); break;
    }
#undef SIREN_L
}

}  // namespace siren

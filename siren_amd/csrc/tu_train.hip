// tu_train.hip — split-K weight-gradient, first/last-layer and slab-reduction kernels.
#include "launch.h"
#include "train_kernels.hpp"

namespace siren {

void launch_wgrad(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, int64_t n_pad, int64_t tps,
                  float* partial, int64_t P, int d, int o, int lh, int with_bias, int h, int jet_bias,
                  int64_t bstride_act, int64_t bstride_part) {
#define SIREN_WG(JB)                                                                                           \
    hipLaunchKernelGGL(wgrad_kernel<JB>, grid, dim3(THREADS), 0, st, abuf, dbuf, n_pad, tps, partial, P, d, o, lh, \
                       with_bias, h, bstride_act, bstride_part)
    switch (jet_bias) {
        case 1: SIREN_WG(1); break;
        case 2: SIREN_WG(2); break;
        case 3: SIREN_WG(3); break;
        default: SIREN_WG(0); break;
    }
#undef SIREN_WG
}

#define NOF ((const float*)nullptr)

void launch_small(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x, const float* gy,
                  int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E, int d, int o, int lh, int h,
                  int64_t bstride_act, int64_t bstride_e) {
    hipLaunchKernelGGL(edge_kernel<EDGE_W2>, grid, dim3(edge_threads(EDGE_W2)), 0, st, dbuf,
                       abuf + (int64_t)lh * n_pad * h, NOF, NOF, x, gy, NOF, NOF, n, n_pad / 16, tps, eslab, E, d, o,
                       lh, h, bstride_act, bstride_e);
}

void launch_small_w3(dim3 grid, hipStream_t st, const float* At, const float* D, const float* Dt, const float* AL,
                     const float* x, const float* v, const float* gy, const float* u, int64_t n, int64_t n_pad,
                     int64_t tps, float* eslab, int64_t E, int d, int o, int lh, int64_t bstride_act,
                     int64_t bstride_e) {
    hipLaunchKernelGGL(edge_kernel<EDGE_W3>, grid, dim3(edge_threads(EDGE_W3)), 0, st, D, At + (int64_t)lh * n_pad * H,
                       Dt, AL, x, v, gy, u, n, n_pad / 16, tps, eslab, E, d, o, lh, H, bstride_act, bstride_e);
}

void launch_small_jet(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x,
                      const float* glap, int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E, int d,
                      int o, int lh) {
    hipLaunchKernelGGL(edge_kernel<EDGE_JET>, grid, dim3(edge_threads(EDGE_JET)), 0, st, dbuf,
                       abuf + (int64_t)lh * 4 * n_pad * H, NOF, NOF, x, glap, NOF, NOF, n, n_pad / 4, tps, eslab, E, d,
                       o, lh, H, (int64_t)0, (int64_t)0);
}

void launch_small_mix(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x, const float* v,
                      const float* g, const float* u, int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E,
                      int d, int o, int lh, int h) {
    hipLaunchKernelGGL(edge_kernel<EDGE_MIX>, grid, dim3(edge_threads(EDGE_MIX)), 0, st, dbuf,
                       abuf + (int64_t)lh * 4 * n_pad * h, NOF, NOF, x, v, g, u, n, n_pad / 4, tps, eslab, E, d, o, lh,
                       h, (int64_t)0, (int64_t)0);
}

void launch_small_q8(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x, const float* u,
                     int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E, int d, int o, int lh) {
    hipLaunchKernelGGL(edge_kernel<EDGE_Q8>, grid, dim3(edge_threads(EDGE_Q8)), 0, st, dbuf,
                       abuf + (int64_t)lh * 4 * n_pad * H, NOF, NOF, x, NOF, NOF, u, n, n_pad / 8, tps, eslab, E, d, o,
                       lh, H, (int64_t)0, (int64_t)0);
}

// rows: zb_0 jet (dbuf layer 0), a_L jet (abuf layer L) of the two-stream tiles (2 n_pad columns per layer, h = 512)
void launch_small_j2(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, const float* x, const float* v,
                     const float* gy, const float* u, int64_t n, int64_t n_pad, int64_t tps, float* eslab, int64_t E,
                     int d, int o, int lh) {
    constexpr int WHH = 512;
    hipLaunchKernelGGL(edge_kernel<EDGE_J2>, grid, dim3(edge_threads(EDGE_J2)), 0, st, dbuf,
                       abuf + (int64_t)lh * 2 * n_pad * WHH, NOF, NOF, x, v, gy, u, n, n_pad / 8, tps, eslab, E, d, o,
                       lh, WHH, (int64_t)0, (int64_t)0);
}

void launch_reduce(dim3 grid, hipStream_t st, const float* partial, int64_t S, int64_t P, float* gp, int64_t S2,
                   int64_t lo, int64_t hi, int64_t bstride_part, int64_t begin, int64_t end) {
    hipLaunchKernelGGL(reduce_kernel, grid, dim3(256), 0, st, partial, S, P, gp, S2, lo, hi, bstride_part, begin, end);
}

void launch_edge_reduce(dim3 grid, hipStream_t st, const float* eslab, int64_t SE, int64_t E, int64_t hidden0,
                        int64_t wout, float* gp, int64_t P, int64_t bstride_e) {
    hipLaunchKernelGGL(edge_reduce_kernel, grid, dim3(256), 0, st, eslab, SE, E, hidden0, wout, gp, P, bstride_e);
}

}  // namespace siren

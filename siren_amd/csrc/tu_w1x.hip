// tu_w1x.hip — the split-bf16 W1 kernel (w1x_kernel.hpp) and its weight pack.
#include "launch.h"
#include "w1x_kernel.hpp"
#include "wgradx_kernel.hpp"

namespace siren {

int64_t split_stream_words(int lh) { return (int64_t)x_slices(lh) * X_SLICE; }

void launch_pack_split(const float* p, unsigned* stream, int d, int o, int lh, float s, hipStream_t st) {
    const int64_t total = (int64_t)x_slices(lh) * 3 * X_OBS * 64;
    hipLaunchKernelGGL(pack_split_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, p, stream, d, o, lh,
                       s);
}

void launch_w1x(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x, int64_t n,
                float* y, float* gx, int d, float w0, float w) {
    if (d == 2)
        hipLaunchKernelGGL((w1x_kernel<3, 2, X_W1>), grid, dim3(64 * x_waves<false>()), 0, st, ws_small, stream, x, n,
                           y, gx, w0, w);
    else
        hipLaunchKernelGGL((w1x_kernel<3, 3, X_W1>), grid, dim3(64 * x_waves<false>()), 0, st, ws_small, stream, x, n,
                           y, gx, w0, w);
}

void launch_w1x_store(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x,
                      int64_t n, const float* gy, float* y, float* gx, float* abuf, float* dbuf, int64_t n_pad, int d,
                      float w0, float w) {
    if (d == 2)
        hipLaunchKernelGGL((w1x_kernel<3, 2, X_STORE>), grid, dim3(64 * x_waves<false>()), 0, st, ws_small, stream, x,
                           n, y, gx, w0, w, gy, abuf, dbuf, n_pad);
    else
        hipLaunchKernelGGL((w1x_kernel<3, 3, X_STORE>), grid, dim3(64 * x_waves<false>()), 0, st, ws_small, stream, x,
                           n, y, gx, w0, w, gy, abuf, dbuf, n_pad);
}

void launch_wgradx(dim3 grid, hipStream_t st, const float* abuf, const float* dbuf, int64_t n_pad, int64_t tps,
                   float* partial, int64_t P, int d, int o, int lh) {
    hipLaunchKernelGGL(wgradx_kernel, grid, dim3(THREADS), 0, st, abuf, dbuf, n_pad, tps, partial, P, d, o, lh);
}

// the stored split of the bf16x6 W2 stage: forward (8 waves, 128-coordinate tiles) keeping a_l tiles (abuf) and the
// lane-major cos (cbuf); reverse (4 waves) from them, delta_l tiles into dbuf, gx nullable
void launch_w0xs(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x, int64_t n,
                 float* y, float* abuf, float* cbuf, int64_t n_pad, int d, float w0, float w) {
    if (d == 2)
        hipLaunchKernelGGL((w1x_kernel<3, 2, X_FWDS>), grid, dim3(64 * x_waves<true>()), 0, st, ws_small, stream, x, n,
                           y, (float*)nullptr, w0, w, (const float*)nullptr, abuf, cbuf, n_pad);
    else
        hipLaunchKernelGGL((w1x_kernel<3, 3, X_FWDS>), grid, dim3(64 * x_waves<true>()), 0, st, ws_small, stream, x, n,
                           y, (float*)nullptr, w0, w, (const float*)nullptr, abuf, cbuf, n_pad);
}
void launch_w1xr(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x, int64_t n,
                 const float* gy, float* gx, const float* cbuf, float* dbuf, int64_t n_pad, int d, float w0, float w) {
    if (d == 2)
        hipLaunchKernelGGL((w1x_kernel<3, 2, X_REV>), grid, dim3(64 * x_nw<X_REV>()), 0, st, ws_small, stream, x,
                           n, (float*)nullptr, gx, w0, w, gy, const_cast<float*>(cbuf), dbuf, n_pad);
    else
        hipLaunchKernelGGL((w1x_kernel<3, 3, X_REV>), grid, dim3(64 * x_nw<X_REV>()), 0, st, ws_small, stream, x,
                           n, (float*)nullptr, gx, w0, w, gy, const_cast<float*>(cbuf), dbuf, n_pad);
}

int split_fwd_tile() { return 16 * x_waves<true>(); }
int split_rev_tile() { return 16 * x_nw<X_REV>(); }

void launch_w0x(dim3 grid, hipStream_t st, const float* ws_small, const unsigned* stream, const float* x, int64_t n,
                float* y, int d, float w0, float w) {
    if (d == 2)
        hipLaunchKernelGGL((w1x_kernel<3, 2, X_FWD>), grid, dim3(64 * x_waves<true>()), 0, st, ws_small, stream, x, n,
                           y, (float*)nullptr, w0, w);
    else
        hipLaunchKernelGGL((w1x_kernel<3, 3, X_FWD>), grid, dim3(64 * x_waves<true>()), 0, st, ws_small, stream, x, n,
                           y, (float*)nullptr, w0, w);
}

}  // namespace siren

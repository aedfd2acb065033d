// layered.hip — hidden widths the fused kernels do not hold in registers (any multiple of 64 up to 4096 other than
// 256 / 512; the reference's train_video.py uses SingleBVPNet(hidden_features=1024), experiment_scripts/train_video.py:55).
//
// At hidden 1024 a 16-coordinate activation tile is 64 KiB per wave — more than the register file — so the
// network runs layer by layer over coordinate chunks: each hidden layer's GEMM (z = a W^T, K = H) is a plain library
// GEMM (rocBLAS SGEMM on the fp32 MFMA pipe, atomics off: deterministic), everything else is a fused HIP epilogue
// over the chunk:
//   lay_first   z_0 = x W0^T + b0 (K = d_in), a_0 = sin(w0 z_0), cos_0
//   lay_sine    a_l = sin(w (z_l + b_l)), cos_l                      (in place over the GEMM output)
//   lay_last    the last hidden layer's sine fused with the output layer: y = a_L Wout^T + bout, one wave per row
//   lay_rev     seed u_L = (gy Wout) cos_L w, or u_{l-1} *= cos_{l-1} w_{l-1}, with the bias gradient sum_c u
//               reduced in the same pass into a per-workgroup slab (fixed order: deterministic)
// and the weight gradients are GEMMs over the chunk (dW_l += u_l^T a_{l-1}, beta = 1 after the first chunk).
//   W0  forward:           FWD | Y
//   W1  + vjp_x:           FWD | GX (| Y)
//   W2  + theta:           FWD | GX | THETA                 (forward recomputed per chunk in the scratch)
//   stored split:          FWD | Y | TWS, then GX | THETA | TWS  (a_l / cos_l of all n rows kept in the caller's
//                          buffer: the backward skips the forward GEMMs — the training forward already ran them)
// Row-major C x H buffers are rocBLAS column-major H x C matrices (ld = H). Parameter vectors keep the flat
// state_dict layout (not 16-byte aligned): the epilogues read them with scalar loads.
#include <rocblas/rocblas.h>

#include <mutex>
#include <string>

#include "launch.h"
#include "siren_common.h"
#include "siren_params.h"

namespace siren {

namespace {

// The forward epilogues map like the reverse ones: 4 columns per thread (fixed, so the bias / W0 columns stay in
// registers), 4 row groups per workgroup, grid = (column blocks, row blocks of LAYERED_RPB rows).
// z_0 = x W0^T + b0 -> a = sin(w0 z_0), cs (nullable) = cos(w0 z_0)
__global__ __launch_bounds__(256) void lay_first_kernel(const float* __restrict__ x, const float* __restrict__ W0,
                                                        const float* __restrict__ b0, int C, int d, int H, float w0,
                                                        float* __restrict__ a, float* __restrict__ cs) {
    const int t = threadIdx.x, rg = t >> 6;
    const int g = blockIdx.x * 64 + (t & 63);
    const int h4 = H / 4;
    if (g >= h4) return;
    f32x4 wc[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k)
        wc[k] = k < d ? f32x4{W0[(4 * g) * d + k], W0[(4 * g + 1) * d + k], W0[(4 * g + 2) * d + k],
                              W0[(4 * g + 3) * d + k]}
                      : f32x4{};
    const f32x4 bb = {b0[4 * g], b0[4 * g + 1], b0[4 * g + 2], b0[4 * g + 3]};
    const int r0 = blockIdx.y * LAYERED_RPB;
    const int r1 = r0 + LAYERED_RPB < C ? r0 + LAYERED_RPB : C;
    for (int c = r0 + rg; c < r1; c += 4) {
        f32x4 z = bb;
#pragma unroll
        for (int k = 0; k < MAXD; ++k)
            if (k < d) z += wc[k] * x[c * d + k];
        f32x4 s4, c4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sn, cn;
            sincos_phase(w0 * z[r], sn, cn);
            s4[r] = sn;
            c4[r] = cn;
        }
        ((f32x4*)a)[c * h4 + g] = s4;
        if (cs != nullptr) ((f32x4*)cs)[c * h4 + g] = c4;
    }
}

// z (C x H, in place) -> sin(w (z + b)); cs (nullable) <- cos(w (z + b))
__global__ __launch_bounds__(256) void lay_sine_kernel(float* __restrict__ z, const float* __restrict__ b, int C,
                                                       int H, float w, float* __restrict__ cs) {
    const int t = threadIdx.x, rg = t >> 6;
    const int g = blockIdx.x * 64 + (t & 63);
    const int h4 = H / 4;
    if (g >= h4) return;
    const f32x4 bb = {b[4 * g], b[4 * g + 1], b[4 * g + 2], b[4 * g + 3]};
    const int r0 = blockIdx.y * LAYERED_RPB;
    const int r1 = r0 + LAYERED_RPB < C ? r0 + LAYERED_RPB : C;
    for (int c = r0 + rg; c < r1; c += 4) {
        const int e = c * h4 + g;
        const f32x4 v = ((const f32x4*)z)[e];
        f32x4 s4, c4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sn, cn;
            sincos_phase(w * (v[r] + bb[r]), sn, cn);
            s4[r] = sn;
            c4[r] = cn;
        }
        ((f32x4*)z)[e] = s4;
        if (cs != nullptr) ((f32x4*)cs)[e] = c4;
    }
}

// The last hidden layer's sine fused with the output layer: one wave per row, y[c] = a_L[c] Wout^T + bout (o <= 4,
// a wave-wide butterfly sum per output in a fixed order).
__global__ __launch_bounds__(256) void lay_last_kernel(float* __restrict__ z, const float* __restrict__ b, int64_t C,
                                                       int H, float w, float* __restrict__ cs,
                                                       const float* __restrict__ Wout, const float* __restrict__ bout,
                                                       int o, float* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int h4 = H / 4;
    for (int64_t c = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < C;
         c += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        float acc[MAXO] = {};
        for (int g = lane; g < h4; g += 64) {
            const int64_t e = c * h4 + g;
            const f32x4 v = ((const f32x4*)z)[e];
            const f32x4 bb = {b[4 * g], b[4 * g + 1], b[4 * g + 2], b[4 * g + 3]};
            f32x4 s4, c4;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float sn, cn;
                sincos_phase(w * (v[r] + bb[r]), sn, cn);
                s4[r] = sn;
                c4[r] = cn;
            }
            ((f32x4*)z)[e] = s4;
            if (cs != nullptr) ((f32x4*)cs)[e] = c4;
#pragma unroll
            for (int j = 0; j < MAXO; ++j)
                if (j < o) {
                    const float* wr = Wout + (int64_t)j * H + 4 * g;
                    acc[j] += s4[0] * wr[0] + s4[1] * wr[1] + s4[2] * wr[2] + s4[3] * wr[3];
                }
        }
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            float v = acc[j];
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
            if (j < o && lane == 0) y[c * o + j] = v + bout[j];
        }
    }
}

// Reverse epilogue over rows [blockIdx.y * RPB, +RPB) of a row-major C x H chunk, 4 columns per thread, 4 row groups
// per workgroup:
//   REV_HIDDEN  u *= w cos                                  -> db_l
//   REV_SEED    u = w cos (gy Wout) (gy == NULL: ones)      -> db_L, and dWout[j] = sum_c gy[c][j] a_L[c]
//   REV_FIRST   u *= w0 cos_0                               -> db_0, and dW0[:, k] = sum_c x[c][k] u_0[c]
// Column sums go into per-workgroup slab rows: bslab[blockIdx.y][H] for the bias, xslab[m][blockIdx.y][H] for the
// fused weight gradient (m < o or d) — written on the first chunk, accumulated after: every slab cell has one
// owner, so the sum order is fixed (deterministic).
enum { REV_HIDDEN = 0, REV_SEED = 1, REV_FIRST = 2 };
template <int KIND>
__global__ __launch_bounds__(256) void lay_rev_kernel(float* __restrict__ u, const float* __restrict__ coef, int nm,
                                                      const float* __restrict__ Wout, const float* __restrict__ aL,
                                                      const float* __restrict__ cs, int C, int H, float w, int R,
                                                      float* __restrict__ bslab, float* __restrict__ xslab, int first) {
    __shared__ f32x4 red[4][64];
    const int t = threadIdx.x, rg = t >> 6;
    const int g = blockIdx.x * 64 + (t & 63);
    const int h4 = H / 4;
    const bool col_ok = g < h4;
    constexpr int NX = KIND == REV_HIDDEN ? 0 : (MAXO > MAXD ? MAXO : MAXD);
    f32x4 wo[KIND == REV_SEED ? MAXO : 1];
    if (KIND == REV_SEED) {
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            const float* wr = Wout + (int64_t)j * H + 4 * g;
            wo[j] = (col_ok && j < nm) ? f32x4{wr[0], wr[1], wr[2], wr[3]} : f32x4{};
        }
    }
    f32x4 sum = {0.f, 0.f, 0.f, 0.f};
    f32x4 xs[NX > 0 ? NX : 1];
#pragma unroll
    for (int m = 0; m < (NX > 0 ? NX : 1); ++m) xs[m] = f32x4{};
    const int r0 = blockIdx.y * LAYERED_RPB;
    const int r1 = r0 + LAYERED_RPB < C ? r0 + LAYERED_RPB : C;
    if (col_ok) {
        for (int c = r0 + rg; c < r1; c += 4) {
            const int e = c * h4 + g;
            float cf[NX > 0 ? NX : 1];
#pragma unroll
            for (int m = 0; m < (NX > 0 ? NX : 1); ++m)
                cf[m] = (NX > 0 && m < nm) ? (coef != nullptr ? coef[c * nm + m] : 1.f) : 0.f;
            f32x4 v;
            if (KIND == REV_SEED) {
                v = f32x4{};
#pragma unroll
                for (int j = 0; j < MAXO; ++j) v += wo[j] * cf[j];
            } else {
                v = ((const f32x4*)u)[e];
            }
            v = v * ((const f32x4*)cs)[e] * w;
            ((f32x4*)u)[e] = v;
            sum += v;
            if (KIND == REV_SEED) {
                const f32x4 a = ((const f32x4*)aL)[e];
#pragma unroll
                for (int m = 0; m < NX; ++m) xs[m] += a * cf[m];
            } else if (KIND == REV_FIRST) {
#pragma unroll
                for (int m = 0; m < NX; ++m) xs[m] += v * cf[m];
            }
        }
    }
    auto combine = [&](const f32x4& mine, float* dst_row) {
        red[rg][t & 63] = mine;
        __syncthreads();
        if (rg == 0 && col_ok) {
            const f32x4 s4 = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
            f32x4* dst = (f32x4*)dst_row + g;
            *dst = first ? s4 : *dst + s4;
        }
        __syncthreads();
    };
    combine(sum, bslab + (int64_t)blockIdx.y * H);
#pragma unroll
    for (int m = 0; m < NX; ++m)
        if (m < nm) combine(xs[m], xslab + ((int64_t)m * R + blockIdx.y) * H);
}

// sum over rows of a row-major C x ncols block (ncols <= 64), same slab scheme as lay_rev_kernel
__global__ __launch_bounds__(256) void lay_colsum_kernel(const float* __restrict__ src, int64_t C, int ncols,
                                                         float* __restrict__ slab, int first) {
    __shared__ float red[4][64];
    const int t = threadIdx.x, rg = t >> 6, j = t & 63;
    const int64_t r0 = (int64_t)blockIdx.y * LAYERED_RPB;
    const int64_t r1 = r0 + LAYERED_RPB < C ? r0 + LAYERED_RPB : C;
    float s = 0.f;
    if (j < ncols)
        for (int64_t c = r0 + rg; c < r1; c += 4) s += src[c * ncols + j];
    red[rg][j] = s;
    __syncthreads();
    if (rg == 0 && j < ncols) {
        const float v = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
        float* dst = slab + (int64_t)blockIdx.y * ncols + j;
        *dst = first ? v : *dst + v;
    }
}

// out[j * cs + m * ms] = sum_r slab[m][r][j] over the R slab rows: 4 row groups per workgroup, combined in a fixed
// order
__global__ __launch_bounds__(256) void lay_slab_reduce_kernel(const float* __restrict__ slab, int R, int cols,
                                                              float* __restrict__ out, int cs, int ms) {
    __shared__ float red[4][64];
    const int t = threadIdx.x, rg = t >> 6;
    const int j = blockIdx.x * 64 + (t & 63);
    const float* src = slab + (int64_t)blockIdx.y * R * cols;
    float s = 0.f;
    if (j < cols) {
#pragma unroll 8
        for (int r = rg; r < R; r += 4) s += src[(int64_t)r * cols + j];
    }
    red[rg][t & 63] = s;
    __syncthreads();
    if (rg == 0 && j < cols)
        out[(int64_t)j * cs + (int64_t)blockIdx.y * ms] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

// W^T of one hidden layer (H x H) through a 64 x 65 LDS tile: the forward GEMMs run as N,N on the transposed copy
__global__ __launch_bounds__(256) void lay_transpose_kernel(const float* __restrict__ W, float* __restrict__ WT, int H) {
    __shared__ float tile[64][65];
    const int bx = blockIdx.x * 64, by = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) tile[r][tx] = W[(int64_t)(by + r) * H + bx + tx];
    __syncthreads();
    for (int r = ty; r < 64; r += 4) WT[(int64_t)(bx + r) * H + by + tx] = tile[tx][r];
}

dim3 ew_grid(int64_t work) {
    const int64_t b = (work + 255) / 256;
    return dim3((unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192));
}

// one rocBLAS handle per device, created lazily; calls are serialised (a handle is not thread-safe). The handle is
// that of the device owning the stream (not the caller's current device), and that device is current for the
// duration of the call (restored afterwards)
std::mutex g_blas_mu;
rocblas_handle g_blas[64] = {};

struct Blas {
    std::lock_guard<std::mutex> lock;
    rocblas_handle h = nullptr;
    int prev = -1;
    explicit Blas(hipStream_t st) : lock(g_blas_mu) {
        int dev = 0;
        (void)hipGetDevice(&prev);
        if (st == nullptr || hipStreamGetDevice(st, &dev) != hipSuccess) dev = prev;
        if (dev < 0 || dev >= 64) return;
        if (dev != prev && hipSetDevice(dev) != hipSuccess) return;
        if (g_blas[dev] == nullptr) {
            if (rocblas_create_handle(&g_blas[dev]) != rocblas_status_success) return;
            rocblas_set_atomics_mode(g_blas[dev], rocblas_atomics_not_allowed);
            rocblas_set_pointer_mode(g_blas[dev], rocblas_pointer_mode_host);
        }
        h = g_blas[dev];
        rocblas_set_stream(h, st);
    }
    ~Blas() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

LayeredPlan::LayeredPlan(int d_, int H_, int lh_, int o_, int64_t n) : d(d_), H(H_), lh(lh_), o(o_) {
    const ParamOffsets off(d, o, lh, H);
    P = off.total;
    P_pad = (P + 63) / 64 * 64;  // the buffers after the parameters start 256-byte aligned (float4 epilogues)
    chunk = LAYERED_CHUNK;
    if (n >= 0 && n < chunk) chunk = (n + 63) / 64 * 64 > 0 ? (n + 63) / 64 * 64 : 64;
    buf = chunk * (int64_t)H;
    R = (chunk + LAYERED_RPB - 1) / LAYERED_RPB;
    // packed workspace (immutable after siren_pack): [params][W_1^T .. W_L^T]
    // caller's chunk scratch: [u ping-pong x 2][bias slabs: L + 1 layers x R x H][dWout slab: o x R x H]
    //                         [dW0 slab: d x R x H][output-bias slab: R x o][a_0..a_L][cos_0..cos_L] (the last two
    //                         only without the stored split, whose a_l / cos_l live in the caller's n-row buffers)
    wt = (int64_t)lh * H * H;
    scratch_stored = 2 * buf + (lh + 1 + o + d) * R * H + R * o;
    scratch = scratch_stored + 2 * (lh + 1) * buf;
}

int64_t layered_ws_floats(int d, int H, int lh, int o) {
    const LayeredPlan p(d, H, lh, o, -1);
    return p.P_pad + p.wt;
}

int64_t layered_scratch_floats(int d, int H, int lh, int o, int64_t n, bool stored) {
    const LayeredPlan p(d, H, lh, o, n);
    return stored ? p.scratch_stored : p.scratch;
}

void layered_pack(const LayeredPlan& pl, const float* params, float* ws, hipStream_t st) {
    const ParamOffsets off(pl.d, pl.o, pl.lh, pl.H);
    (void)hipMemcpyAsync(ws, params, pl.P * sizeof(float), hipMemcpyDeviceToDevice, st);
    for (int l = 1; l <= pl.lh; ++l)
        hipLaunchKernelGGL(lay_transpose_kernel, dim3((unsigned)(pl.H / 64), (unsigned)(pl.H / 64)), dim3(256), 0, st,
                           params + off.w(l), ws + pl.P_pad + (int64_t)(l - 1) * pl.H * pl.H, pl.H);
}

int layered_run(int mode, const LayeredPlan& pl, const float* ws, float w0, float w, const float* x, int64_t n,
                const float* gy, float* y, float* gx, float* gparams, float* tws, float* scr, hipStream_t st,
                std::string& err) {
    if (n <= 0) return 0;
    const int d = pl.d, H = pl.H, lh = pl.lh, o = pl.o;
    const ParamOffsets off(d, o, lh, H);
    const float* prm = ws;
    const float* WT = ws + pl.P_pad;                      // W_l^T at WT + (l - 1) H^2 (siren_pack)
    float* U0 = scr;                                      // the caller's chunk scratch (layered_scratch_floats)
    float* U1 = U0 + pl.buf;
    float* bslab = U1 + pl.buf;                          // bias slabs: layer l at bslab + l * R * H
    float* oslab = bslab + (lh + 1) * pl.R * H;           // dWout: o x R x H
    float* fslab = oslab + (int64_t)o * pl.R * H;         // dW0: d x R x H
    float* boslab = fslab + (int64_t)d * pl.R * H;        // dbout: R x o
    float* acs = boslab + pl.R * o;                       // a_l / cos_l of the current chunk (no stored split)
    const bool stored = (mode & LAY_TWS) != 0, fwd = (mode & LAY_FWD) != 0;
    const bool gxm = (mode & LAY_GX) != 0, theta = (mode & LAY_THETA) != 0;
    const bool keep_cos = gxm || theta || stored;  // the forward keeps cos_l for a reverse sweep
    // a_l / cos_l of chunk c0: the caller's n-row buffers (stored split) or the chunk scratch
    auto A = [&](int l, int64_t c0) -> float* {
        return stored ? tws + (int64_t)l * n * H + c0 * H : acs + (int64_t)l * pl.buf;
    };
    auto CS = [&](int l, int64_t c0) -> float* {
        return stored ? tws + (int64_t)(lh + 1 + l) * n * H + c0 * H : acs + (int64_t)(lh + 1 + l) * pl.buf;
    };
    Blas blas(st);
    if (blas.h == nullptr) {
        err = "rocblas_create_handle failed";
        return 3;
    }
    const float one = 1.f, zero = 0.f;
    auto gemm = [&](rocblas_operation ta, rocblas_operation tb, int m, int nn, int k, const float* Am, int lda,
                    const float* Bm, int ldb, float beta, float* Cm, int ldc) -> bool {
        return rocblas_sgemm(blas.h, ta, tb, m, nn, k, &one, Am, lda, Bm, ldb, beta == 0.f ? &zero : &one, Cm, ldc) ==
               rocblas_status_success;
    };
    const rocblas_operation N_ = rocblas_operation_none;
    const int R = (int)pl.R;
    for (int64_t c0 = 0; c0 < n; c0 += pl.chunk) {
        const int C = (int)(n - c0 < pl.chunk ? n - c0 : pl.chunk);
        const float* xc = x + c0 * d;
        const float* gyc = gy != nullptr ? gy + c0 * o : nullptr;
        const int first = c0 == 0;
        const dim3 rgrid((unsigned)((H / 4 + 63) / 64), (unsigned)((C + LAYERED_RPB - 1) / LAYERED_RPB));
        if (fwd) {
            // a_0 (+ cos_0), the hidden layers (lh >= 1, check_cfg; z_l = W_l a_{l-1} as N,N on W_l^T), the last
            // one fused with the output layer (forward-only mode ping-pongs two buffers)
            float* a_prev = A(0, c0);
            hipLaunchKernelGGL(lay_first_kernel, rgrid, dim3(256), 0, st, xc, prm + off.w0, prm + off.b0, C, d, H, w0,
                               a_prev, keep_cos ? CS(0, c0) : nullptr);
            for (int l = 1; l <= lh; ++l) {
                float* a_l = keep_cos ? A(l, c0) : (a_prev == A(0, c0) ? U0 : A(0, c0));
                if (!gemm(N_, N_, H, C, H, WT + (int64_t)(l - 1) * H * H, H, a_prev, H, 0.f, a_l, H)) {
                    err = "rocblas_sgemm (hidden layer) failed";
                    return 3;
                }
                float* cs_l = keep_cos ? CS(l, c0) : nullptr;
                if (l == lh && y != nullptr && (mode & LAY_Y))
                    hipLaunchKernelGGL(lay_last_kernel, ew_grid((int64_t)C * 64), dim3(256), 0, st, a_l,
                                       prm + off.b(l), (int64_t)C, H, w, cs_l, prm + off.wout, prm + off.bout, o,
                                       y + c0 * o);
                else
                    hipLaunchKernelGGL(lay_sine_kernel, rgrid, dim3(256), 0, st, a_l, prm + off.b(l), C, H, w, cs_l);
                a_prev = a_l;
            }
        }
        if (!(gxm || theta)) continue;
        const float beta = first ? 0.f : 1.f;
        if (theta)  // dbout = sum_c gy
            hipLaunchKernelGGL(lay_colsum_kernel, dim3(1, rgrid.y), dim3(256), 0, st, gyc, (int64_t)C, o, boslab, first);
        // seed u_L = (gy Wout) cos_L w (+ db_L, dWout), then the reverse sweep u_{l-1} = (u_l W_l) cos_{l-1}
        // w_{l-1} (+ db_{l-1}; layer 0: + dW0); dW_l += u_l^T a_{l-1} as GEMMs
        float* u = U0;
        hipLaunchKernelGGL(lay_rev_kernel<REV_SEED>, rgrid, dim3(256), 0, st, u, gyc, o, prm + off.wout, A(lh, c0),
                           CS(lh, c0), C, H, w, R, bslab + (int64_t)lh * R * H, oslab, first);
        for (int l = lh; l >= 1; --l) {
            if (theta && !gemm(N_, rocblas_operation_transpose, H, H, C, A(l - 1, c0), H, u, H, beta,
                               gparams + off.w(l), H)) {
                err = "rocblas_sgemm (hidden-layer gradient) failed";
                return 3;
            }
            float* un = u == U0 ? U1 : U0;
            if (!gemm(N_, N_, H, C, H, prm + off.w(l), H, u, H, 0.f, un, H)) {
                err = "rocblas_sgemm (reverse) failed";
                return 3;
            }
            if (l > 1)
                hipLaunchKernelGGL(lay_rev_kernel<REV_HIDDEN>, rgrid, dim3(256), 0, st, un, (const float*)nullptr, 0,
                                   (const float*)nullptr, (const float*)nullptr, CS(l - 1, c0), C, H, w, R,
                                   bslab + (int64_t)(l - 1) * R * H, (float*)nullptr, first);
            else
                hipLaunchKernelGGL(lay_rev_kernel<REV_FIRST>, rgrid, dim3(256), 0, st, un, xc, d, (const float*)nullptr,
                                   (const float*)nullptr, CS(0, c0), C, H, w0, R, bslab, fslab, first);
            u = un;
        }
        // gx = u_0 W0
        if (gx != nullptr && !gemm(N_, N_, d, C, H, prm + off.w0, d, u, H, 0.f, gx + c0 * d, d)) {
            err = "rocblas_sgemm (gx) failed";
            return 3;
        }
    }
    if (theta) {  // bias gradients, dWout and dW0: slab rows summed in order (rows the first chunk wrote)
        const int Rn = (int)(((n < pl.chunk ? n : pl.chunk) + LAYERED_RPB - 1) / LAYERED_RPB);
        const unsigned cb = (unsigned)((H + 63) / 64);
        for (int l = 0; l <= lh; ++l)
            hipLaunchKernelGGL(lay_slab_reduce_kernel, dim3(cb), dim3(256), 0, st, bslab + (int64_t)l * R * H, Rn, H,
                               gparams + (l == 0 ? off.b0 : off.b(l)), 1, 0);
        hipLaunchKernelGGL(lay_slab_reduce_kernel, dim3(cb, (unsigned)o), dim3(256), 0, st, oslab, Rn, H,
                           gparams + off.wout, 1, H);
        hipLaunchKernelGGL(lay_slab_reduce_kernel, dim3(cb, (unsigned)d), dim3(256), 0, st, fslab, Rn, H,
                           gparams + off.w0, d, 1);
        hipLaunchKernelGGL(lay_slab_reduce_kernel, dim3(1), dim3(256), 0, st, boslab, Rn, o, gparams + off.bout, 1, 0);
    }
    return 0;
}

}  // namespace siren

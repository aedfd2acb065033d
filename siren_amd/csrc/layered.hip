// layered.hip — hidden widths the fused kernels do not hold in registers (any multiple of 64 up to 4096 other than
// 256 / 512; the reference's train_video.py uses SingleBVPNet(hidden_features=1024), experiment_scripts/train_video.py:55).
//
// At hidden 1024 a 16-coordinate activation tile is 64 KiB per wave — more than the register file — so the
// network runs layer by layer over coordinate chunks: each hidden layer's GEMM (z = a W^T, K = H) is a plain library
// GEMM (rocBLAS SGEMM on the fp32 MFMA pipe, atomics off: deterministic), everything else is a fused HIP epilogue
// over the chunk (bias + sin / cos, the reverse cos product, the output seed, the first layer's K = d_in product).
// Per chunk of C coordinates the caller's packed workspace holds a_l and cos(w z_l) of every layer and two reverse
// buffers (row-major C x H each), so no entry point needs more than siren_workspace_floats():
//   W0  forward:      z_0 = x W0^T + b0 (epilogue kernel), [z_l = a_{l-1} W_l^T (GEMM), a_l = sin(w(z_l + b_l))]
//                     y = a_L Wout^T (GEMM) + bout
//   W1  + vjp_x:      the forward keeps cos_l; u_L = (gy Wout) cos_L w; [u_{l-1} = (u_l W_l) cos_{l-1} w_{l-1}]
//                     gx = u_0 W0 (GEMM)
//   W2  + theta:      W1's sweep keeping a_l, and per chunk dW_l += u_l^T a_{l-1} (GEMM, beta = 1 after the first
//                     chunk), db_l += u_l^T 1 (GEMV), dW0 += u_0^T x, dWout += gy^T a_L, dbout += gy^T 1.
// Row-major C x H buffers are rocBLAS column-major H x C matrices (ld = H).
#include <rocblas/rocblas.h>

#include <mutex>
#include <string>

#include "launch.h"
#include "siren_common.h"
#include "siren_params.h"

namespace siren {

namespace {

__global__ void lay_first_kernel(const float* __restrict__ x, const float* __restrict__ W0, const float* __restrict__ b0,
                                 int64_t C, int d, int H, float w0, float* __restrict__ a, float* __restrict__ cs) {
    const int64_t total = C * H;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = e / H;
        const int j = (int)(e - c * H);
        float z = b0[j];
        for (int k = 0; k < d; ++k) z = __builtin_fmaf(x[c * d + k], W0[(int64_t)j * d + k], z);
        float sn, cn;
        sincos_phase(w0 * z, sn, cn);
        a[e] = sn;
        if (cs != nullptr) cs[e] = cn;
    }
}

// z (C x H, in place) -> sin(w (z + b)); cs (nullable) <- cos(w (z + b))
__global__ void lay_sine_kernel(float* __restrict__ z, const float* __restrict__ b, int64_t C, int H, float w,
                                float* __restrict__ cs) {
    const int64_t total4 = C * H / 4;
    const int h4 = H / 4;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total4; e += (int64_t)gridDim.x * blockDim.x) {
        const int j4 = (int)(e % h4);
        f32x4 v = ((f32x4*)z)[e];
        const f32x4 bb = ((const f32x4*)b)[j4];
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

// u (C x H, in place) *= cos * w
__global__ void lay_mulcos_kernel(float* __restrict__ u, const float* __restrict__ cs, int64_t total4, float w) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total4; e += (int64_t)gridDim.x * blockDim.x)
        ((f32x4*)u)[e] = ((f32x4*)u)[e] * ((const f32x4*)cs)[e] * w;
}

// u_L[c][k] = w cos_L[c][k] sum_j gy[c][j] Wout[j][k] (gy == NULL: ones)
__global__ void lay_seed_kernel(const float* __restrict__ gy, const float* __restrict__ Wout,
                                const float* __restrict__ cs, int64_t C, int H, int o, float w, float* __restrict__ u) {
    const int64_t total = C * H;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = e / H;
        const int k = (int)(e - c * H);
        float s = 0.f;
        for (int j = 0; j < o; ++j) s = __builtin_fmaf(gy != nullptr ? gy[c * o + j] : 1.f, Wout[(int64_t)j * H + k], s);
        u[e] = s * cs[e] * w;
    }
}

__global__ void lay_bias_kernel(float* __restrict__ y, const float* __restrict__ b, int64_t C, int o) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < C * o; e += (int64_t)gridDim.x * blockDim.x)
        y[e] += b[e % o];
}

__global__ void lay_fill_kernel(float* __restrict__ p, int64_t n, float v) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x)
        p[e] = v;
}

dim3 ew_grid(int64_t work) {
    const int64_t b = (work + 255) / 256;
    return dim3((unsigned)(b < 8192 ? (b > 0 ? b : 1) : 8192));
}

// one rocBLAS handle per device, created lazily; calls are serialised (a handle is not thread-safe)
std::mutex g_blas_mu;
rocblas_handle g_blas[64] = {};

struct Blas {
    std::lock_guard<std::mutex> lock;
    rocblas_handle h = nullptr;
    explicit Blas(hipStream_t st) : lock(g_blas_mu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (dev < 0 || dev >= 64) dev = 0;
        if (g_blas[dev] == nullptr) {
            if (rocblas_create_handle(&g_blas[dev]) != rocblas_status_success) return;
            rocblas_set_atomics_mode(g_blas[dev], rocblas_atomics_not_allowed);
            rocblas_set_pointer_mode(g_blas[dev], rocblas_pointer_mode_host);
        }
        h = g_blas[dev];
        rocblas_set_stream(h, st);
    }
};

}  // namespace

LayeredPlan::LayeredPlan(int d_, int H_, int lh_, int o_, int64_t n) : d(d_), H(H_), lh(lh_), o(o_) {
    const ParamOffsets off(d, o, lh, H);
    P = off.total;
    chunk = LAYERED_CHUNK;
    if (n >= 0 && n < chunk) chunk = (n + 63) / 64 * 64 > 0 ? (n + 63) / 64 * 64 : 64;
    buf = chunk * (int64_t)H;
    // [params][a_0..a_L][cos_0..cos_L][u ping-pong x 2][ones]
    scratch = 2 * (lh + 1) * buf + 2 * buf + chunk;
}

int64_t layered_ws_floats(int d, int H, int lh, int o) {
    const LayeredPlan p(d, H, lh, o, -1);
    return p.P + p.scratch;
}

// mode: 0 = W0 (forward), 1 = W1 (forward + vjp_x), 2 = W2 (+ theta)
int layered_run(int mode, const LayeredPlan& pl, const float* ws, float w0, float w, const float* x, int64_t n,
                const float* gy, float* y, float* gx, float* gparams, hipStream_t st, std::string& err) {
    if (n <= 0) return 0;
    const int d = pl.d, H = pl.H, lh = pl.lh, o = pl.o;
    const ParamOffsets off(d, o, lh, H);
    const float* prm = ws;
    float* scr = const_cast<float*>(ws) + pl.P;  // the packed workspace is the caller's scratch (siren_pack)
    float* A = scr;                               // a_l: A + l * buf
    float* CS = A + (lh + 1) * pl.buf;           // cos_l
    float* U0 = CS + (lh + 1) * pl.buf;
    float* U1 = U0 + pl.buf;
    float* ones = U1 + pl.buf;
    const bool grad = mode >= 1, theta = mode == 2;
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
    const rocblas_operation N_ = rocblas_operation_none, T_ = rocblas_operation_transpose;
    if (theta) hipLaunchKernelGGL(lay_fill_kernel, ew_grid(pl.chunk), dim3(256), 0, st, ones, pl.chunk, 1.f);
    for (int64_t c0 = 0; c0 < n; c0 += pl.chunk) {
        const int C = (int)(n - c0 < pl.chunk ? n - c0 : pl.chunk);
        const float* xc = x + c0 * d;
        const float* gyc = gy != nullptr ? gy + c0 * o : nullptr;
        // forward: a_0 (+ cos_0), then the hidden layers (W0 mode ping-pongs two buffers)
        float* a_prev = A;
        hipLaunchKernelGGL(lay_first_kernel, ew_grid((int64_t)C * H), dim3(256), 0, st, xc, prm + off.w0, prm + off.b0,
                           (int64_t)C, d, H, w0, a_prev, grad ? CS : nullptr);
        for (int l = 1; l <= lh; ++l) {
            float* a_l = grad ? A + (int64_t)l * pl.buf : (a_prev == A ? U0 : A);
            if (!gemm(T_, N_, H, C, H, prm + off.w(l), H, a_prev, H, 0.f, a_l, H)) {
                err = "rocblas_sgemm (hidden layer) failed";
                return 3;
            }
            hipLaunchKernelGGL(lay_sine_kernel, ew_grid((int64_t)C * H / 4), dim3(256), 0, st, a_l, prm + off.b(l),
                               (int64_t)C, H, w, grad ? CS + (int64_t)l * pl.buf : nullptr);
            a_prev = a_l;
        }
        if (y != nullptr) {  // y = a_L Wout^T + bout
            float* yc = y + c0 * o;
            if (!gemm(T_, N_, o, C, H, prm + off.wout, H, a_prev, H, 0.f, yc, o)) {
                err = "rocblas_sgemm (output layer) failed";
                return 3;
            }
            hipLaunchKernelGGL(lay_bias_kernel, ew_grid((int64_t)C * o), dim3(256), 0, st, yc, prm + off.bout,
                               (int64_t)C, o);
        }
        if (!grad) continue;
        const float beta = c0 == 0 ? 0.f : 1.f;
        if (theta) {  // output layer: dWout += gy^T a_L, dbout += gy^T 1
            if (!gemm(N_, T_, H, o, C, a_prev, H, gyc, o, beta, gparams + off.wout, H) ||
                rocblas_sgemv(blas.h, N_, o, C, &one, gyc, o, ones, 1, beta == 0.f ? &zero : &one, gparams + off.bout,
                              1) != rocblas_status_success) {
                err = "rocblas (output-layer gradient) failed";
                return 3;
            }
        }
        // seed u_L = (gy Wout) cos_L w, then the reverse sweep u_{l-1} = (u_l W_l) cos_{l-1} w_{l-1}
        float* u = U0;
        hipLaunchKernelGGL(lay_seed_kernel, ew_grid((int64_t)C * H), dim3(256), 0, st, gyc, prm + off.wout,
                           CS + (int64_t)lh * pl.buf, (int64_t)C, H, o, w, u);
        for (int l = lh; l >= 1; --l) {
            if (theta) {  // dW_l += u_l^T a_{l-1}, db_l += u_l^T 1
                if (!gemm(N_, T_, H, H, C, A + (int64_t)(l - 1) * pl.buf, H, u, H, beta, gparams + off.w(l), H) ||
                    rocblas_sgemv(blas.h, N_, H, C, &one, u, H, ones, 1, beta == 0.f ? &zero : &one,
                                  gparams + off.b(l), 1) != rocblas_status_success) {
                    err = "rocblas (hidden-layer gradient) failed";
                    return 3;
                }
            }
            float* un = u == U0 ? U1 : U0;
            if (!gemm(N_, N_, H, C, H, prm + off.w(l), H, u, H, 0.f, un, H)) {
                err = "rocblas_sgemm (reverse) failed";
                return 3;
            }
            hipLaunchKernelGGL(lay_mulcos_kernel, ew_grid((int64_t)C * H / 4), dim3(256), 0, st, un,
                               CS + (int64_t)(l - 1) * pl.buf, (int64_t)C * H / 4, l - 1 == 0 ? w0 : w);
            u = un;
        }
        // gx = u_0 W0; first layer: dW0 += u_0^T x, db0 += u_0^T 1
        if (gx != nullptr && !gemm(N_, N_, d, C, H, prm + off.w0, d, u, H, 0.f, gx + c0 * d, d)) {
            err = "rocblas_sgemm (gx) failed";
            return 3;
        }
        if (theta) {
            if (!gemm(N_, T_, d, H, C, xc, d, u, H, beta, gparams + off.w0, d) ||
                rocblas_sgemv(blas.h, N_, H, C, &one, u, H, ones, 1, beta == 0.f ? &zero : &one, gparams + off.b0, 1) !=
                    rocblas_status_success) {
                err = "rocblas (first-layer gradient) failed";
                return 3;
            }
        }
    }
    return 0;
}

}  // namespace siren

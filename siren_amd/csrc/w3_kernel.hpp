// w3_kernel.hpp — second-order adjoint of the SIREN (work unit W3) for gfx950.
//
// What autograd asks of the graph node J(x; theta) = dPhi/dx when a loss depends on the gradient
// (loss_functions.py:84-89 gradients_mse, :214-238 sdf; and every divergence() call inside laplace,
// diff_operators.py:27-36): given a per-coordinate cotangent v = gJ (n, d), return
//     gx     = d/dx     sum_c <v_c, J(x_c)>  = H(x_c) v_c        (Hessian-vector product)
//     gtheta = d/dtheta sum_c <v_c, J(x_c)>                       (mixed second derivative; optional)
// Reverse-over-forward: F = sum_c ydot_c where ydot is the forward-mode tangent of y along v_c.
//   forward (per layer, primal + tangent share every weight A operand: 2 MFMAs per ds_read):
//       z_l = W_l a_{l-1} + b_l,   zd_l = W_l ad_{l-1}      (z_0 = W0 x + b0, zd_0 = W0 v on VALU)
//       a_l = sin(w z_l), c_l = cos(w z_l), ad_l = w c_l zd_l
//   reverse (adjoints ab of a and adb of ad; adb_L = Wout^T, ab_L = gy_c Wout^T):
//       zdb_l = w c_l adb_l
//       zb_l  = w c_l ab_l - w^2 a_l zd_l adb_l
//       adb_{l-1} = W_l^T zdb_l,  ab_{l-1} = W_l^T zb_l,  gx = W0^T zb_0
//   weight gradients (THETA): dW_l = zdb_l ad_{l-1}^T + zb_l a_{l-1}^T (the split-K wgrad kernel, K = 2N),
//       db_l = sum zb_l, dW0 = zdb_0 v^T + zb_0 x^T, dWout = sum (ad_L + gy a_L), dbout = sum gy.
// Optional first-order seed gy (n, o): the same sweep then returns the gradient of sum_c gy_c . y_c + <v_c, J(x_c)>
// (the sdf loss's value and gradient terms in ONE backward; the first-order adjoint rides in ab, which is linear).
// Vector outputs (d_out = o > 1, diff_operators.jacobian/hessian, loss_functions.py:112-211): an optional output
// weighting u (n, o) makes the tangent functional sum_c <v_c, J(x_c)^T u_c> (adb_L = Wout^T u_c; u == NULL means
// all ones, i.e. J = sum_j dPhi_j/dx as diff_operators.gradient records it), and the optional output ydot (n, o) is
// the forward tangent J(x_c) v_c = d/du of that functional (the gy-cotangent of a vjp node).
// (c_l, zd_l, a_l) of every layer go to a per-wave spill area in HBM in the forward sweep and come back in the
// reverse sweep (coalesced 1 KiB per block; a WG's 768 KiB usually still sits in the 256 MiB Infinity Cache).
// Same weight stream (packed forward + transposed slices) and 3-slot LDS ring as the W1 kernels.
// KEPT (sdf training after a stored jet forward, siren_forward_grad_store): a_l (wgrad tile layout, kA) and
// cos(w z_l) (lane-major, kC) of every layer come from the forward's workspace, so the hidden layers run the
// tangent GEMMs only (half the forward MFMAs), only zdot is spilled, and kA doubles as the THETA A buffer.
#pragma once
#include "lds_ops.h"
#include "ring.hpp"
#include "siren_common.h"
#include "siren_params.h"

namespace siren {

// The layer GEMMs with the mid-slice ring protocol (ring_mid, lds_ops.h slice_*_mid): slice s is published on entry
// (by the previous GEMM's last mid-slice barrier or the kernel's ring prologue); the operand reads run on across the
// slice seams inside the GEMM.
__device__ __forceinline__ void layer_mma2(const float* __restrict__ stream, float* ring, int& s, int nslices,
                                           int wave, int lane, const f32x4 (&bp)[NB], const f32x4 (&bt)[NB],
                                           f32x4 (&accp)[NB], f32x4 (&acct)[NB]) {
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) {
        accp[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
        acct[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const unsigned rbase = lds_addr(ring) + 16u * lane;
    f32x4 a = lds_read4<0>(rbase + (s % NBUF) * SLICE * 4);
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
        const unsigned va = rbase + (s % NBUF) * SLICE * 4, vn = rbase + ((s + 1) % NBUF) * SLICE * 4;
        auto mid = [&]() { ring_mid(stream, ring, s, nslices, wave, lane); };
        if (kb + 1 < NB)
            slice_mma2_mid<NB, NB / 2, true>(va, vn, bp[kb], bt[kb], accp, acct, a, a, mid);
        else
            slice_mma2_mid<NB, NB / 2, false>(va, vn, bp[kb], bt[kb], accp, acct, a, a, mid);
        ++s;
    }
}

// tangent-only layer GEMM (KEPT): acc = W-slices x B, 16 slices
__device__ __forceinline__ void layer_mma1(const float* __restrict__ stream, float* ring, int& s, int nslices,
                                           int wave, int lane, const f32x4 (&bt)[NB], f32x4 (&acct)[NB]) {
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) acct[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned rbase = lds_addr(ring) + 16u * lane;
    f32x4 a0 = lds_read4<0>(rbase + (s % NBUF) * SLICE * 4);
    f32x4 a1 = lds_read4<1024>(rbase + (s % NBUF) * SLICE * 4);
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
        const unsigned va = rbase + (s % NBUF) * SLICE * 4, vn = rbase + ((s + 1) % NBUF) * SLICE * 4;
        auto mid = [&]() { ring_mid(stream, ring, s, nslices, wave, lane); };
        if (kb + 1 < NB)
            slice_mma_mid<NB, NB / 4, true>(va, vn, bt[kb], acct, a0, a1, a0, a1, mid);
        else
            slice_mma_mid<NB, NB / 4, false>(va, vn, bt[kb], acct, a0, a1, a0, a1, mid);
        ++s;
    }
}

// spill slot of (layer l, quantity q in {c, zd, a}, block b) for this lane: 1 KiB per block, lane-contiguous
__device__ __forceinline__ f32x4* spill_at(float* wave_spill, int l, int q, int b, int lane) {
    return (f32x4*)(wave_spill + ((int64_t)(l * 3 + q) * NB + b) * 256 + lane * 4);
}

// KEPT inputs of (layer l, block rb) for this lane: a_l from the wgrad tile layout (4 strided dwords), cos lane-major
__device__ __forceinline__ f32x4 kept_a(const float* kA, int64_t lstride, int64_t toff, int l, int rb) {
    const float* p = kA + l * lstride + toff + rb * 256;
    return f32x4{p[0], p[16], p[32], p[48]};
}

template <int LH, bool THETA, bool KEPT = false>
__global__ __launch_bounds__(THREADS, 1) void w3_kernel(const float* __restrict__ ws, const float* __restrict__ x,
                                                        const float* __restrict__ v, const float* __restrict__ gy,
                                                        const float* __restrict__ u, float* __restrict__ ydot, int o,
                                                        int64_t n, float* __restrict__ gx,
                                                        float* __restrict__ spill, float* __restrict__ A,
                                                        float* __restrict__ At, float* __restrict__ D,
                                                        float* __restrict__ Dt, int64_t n_pad, int d, float w0,
                                                        float w, const float* __restrict__ kA,
                                                        const float* __restrict__ kC,
                                                        unsigned long long* __restrict__ prof = nullptr,
                                                        int64_t ws_bs = 0, int64_t spill_bs = 0, int64_t buf_bs = 0) {
    __shared__ __attribute__((aligned(16))) float lds[NBUF * SLICE + SMALL_MAX + WAVES * STB_SCRATCH];
    float* ring = lds;
    float* sm = lds + NBUF * SLICE;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15;
    const int nslices = 2 * LH * NB;
    // grouped launch over batched weights (siren_second_order_batched): block (x, element), renumbered XCD-major
    int64_t bx = blockIdx.x;
    if (ws_bs != 0) {
        unsigned rx, ry;
        xcd_remap(rx, ry);
        bx = rx;
        const int64_t b = ry;
        ws += b * ws_bs;
        x += b * n * d;
        v += b * n * d;
        gx += b * n * d;
        if (gy != nullptr) gy += b * n * o;
        if (u != nullptr) u += b * n * o;
        if (ydot != nullptr) ydot += b * n * o;
        spill += b * spill_bs;
        if (THETA) {
            A += b * buf_bs;
            At += b * buf_bs;
            D += b * buf_bs;
            Dt += b * buf_bs;
        }
    }
    const float* stream = ws + small_pad(LH);
    const int64_t tile = bx * WAVES + wave;
    // diagnostics (siren_w3_phase_profile): s_memtime after each phase, workgroups < 256, wave 0
    const bool rec = prof != nullptr && blockIdx.x < 256 && blockIdx.y == 0 && wave == 0;
    int ev = 0;
    auto mark = [&]() {
        if (rec) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (lane == 0) prof[blockIdx.x * 16 + ev] = t;
        }
        ++ev;
    };
    mark();
    float* wsp = spill + tile * (int64_t)(LH + 1) * 3 * NB * 256;
    const int64_t lstride = n_pad * H;
    const int64_t toff = tile * (H * 16) + 4 * g * 16 + c;
    const int64_t tbase = tile * (H * 16);  // the wave's tile (store_block4)
    float* stb = lds + NBUF * SLICE + SMALL_MAX + wave * STB_SCRATCH;
    auto kept_c = [&](int l, int rb) -> f32x4 {
        return *(const f32x4*)(kC + cos_off(bx, wave, LH, l, rb, lane));
    };

    {
        const int nf4 = (small_floats(LH) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t coord = bx * TILE + wave * 16 + c;
    const bool valid = coord < n;
    float xv[MAXD], vv[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        xv[k] = (valid && k < d) ? x[coord * d + k] : 0.f;
        vv[k] = (valid && k < d) ? v[coord * d + k] : 0.f;
    }
    __syncthreads();
    ring_issue(stream, ring, 0, nslices, wave, lane);
    ring_issue(stream, ring, 1, nslices, wave, lane);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // slice 0 (and every earlier load) landed: publish it
    __builtin_amdgcn_s_barrier();

    f32x4 actp[NB], actt[NB], accp[NB], acct[NB];
    // ---- layer 0 (VALU): z0 = W0 x + b0, zd0 = W0 v ----------------------------------------------------
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        const int nb = 16 * rb + 4 * g;
        f32x4 z = *(const f32x4*)(sm + SM_BIAS + nb);
        f32x4 zd = {0.f, 0.f, 0.f, 0.f};
        f32x4 zx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < MAXD; ++k) {
            if (k < d) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + nb);
                // explicit fma chain (w3i_kernel's FIRST epilogue runs the same one over all MAXD rows)
                zx = k == 0 ? xv[0] * wk : fma4(xv[k], wk, zx);
                zd = fma4(vv[k], wk, zd);
            }
        }
        z = zx + z;
        f32x4 sn, cs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a_, c_;
            sincos_fast(w0 * z[r], a_, c_);
            sn[r] = a_;
            cs[r] = c_;
        }
        actp[rb] = sn;
        actt[rb] = (w0 * cs) * zd;
        *spill_at(wsp, 0, 1, rb, lane) = zd;
        if (!KEPT) {
            *spill_at(wsp, 0, 0, rb, lane) = cs;
            if (!THETA) *spill_at(wsp, 0, 2, rb, lane) = sn;  // THETA: a_l comes back from the A tiles
        }
        if (THETA) {
            if (!KEPT) store_block4(A + tbase, rb, actp[rb], stb, lane);
            store_block4(At + tbase, rb, actt[rb], stb, lane);
        }
    }

    mark();
    // ---- hidden layers: primal + tangent GEMMs ------------------------------------------------------------
    int s = 0;
#pragma unroll 1
    for (int l = 1; l <= LH; ++l) {
        if constexpr (KEPT) {
            // primal from the stored forward: tangent GEMM only, zdot_l = W_l adot_{l-1}, adot_l = w cos_l zdot_l
            layer_mma1(stream, ring, s, nslices, wave, lane, actt, acct);
            mark();
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 zd = acct[rb];
                actt[rb] = (w * kept_c(l, rb)) * zd;
                *spill_at(wsp, l, 1, rb, lane) = zd;
                if (THETA) store_block4(At + l * lstride + tbase, rb, actt[rb], stb, lane);
            }
            mark();
            continue;
        }
        layer_mma2(stream, ring, s, nslices, wave, lane, actp, actt, accp, acct);
        mark();
        const float* bl = sm + SM_BIAS + l * H + 4 * g;
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            const f32x4 z = accp[rb] + *(const f32x4*)(bl + 16 * rb);
            const f32x4 zd = acct[rb];
            f32x4 sn, cs;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float a_, c_;
                sincos_fast(w * z[r], a_, c_);
                sn[r] = a_;
                cs[r] = c_;
            }
            actp[rb] = sn;
            actt[rb] = (w * cs) * zd;
            *spill_at(wsp, l, 0, rb, lane) = cs;
            *spill_at(wsp, l, 1, rb, lane) = zd;
            if (!THETA) *spill_at(wsp, l, 2, rb, lane) = sn;
            if (THETA) {
                store_block4(A + l * lstride + tbase, rb, actp[rb], stb, lane);
                store_block4(At + l * lstride + tbase, rb, actt[rb], stb, lane);
            }
        }
        mark();
    }

    // ---- ydot = Wout ad_L (the forward tangent of y along v) ---------------------------------------------------
    if (ydot != nullptr) {
        for (int j = 0; j < o; ++j) {
            float p = 0.f;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + 16 * rb + 4 * g);
                p += wj[0] * actt[rb][0] + wj[1] * actt[rb][1] + wj[2] * actt[rb][2] + wj[3] * actt[rb][3];
            }
            p = sum_groups(p);
            if (valid && g == 0) ydot[coord * o + j] = p;
        }
    }
    // ---- reverse: seed at layer L (adb_L = Wout^T u, ab_L = Wout^T gy; u = ones when NULL, gy = 0 when NULL) ----
    float gyv[MAXO], uv[MAXO];
#pragma unroll
    for (int j = 0; j < MAXO; ++j) {
        gyv[j] = (gy != nullptr && valid && j < o) ? gy[coord * o + j] : 0.f;
        uv[j] = (u != nullptr && valid && j < o) ? u[coord * o + j] : 0.f;
    }
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        f32x4 adb = *(const f32x4*)(sm + SM_SEED + 16 * rb + 4 * g);
        f32x4 abseed = {0.f, 0.f, 0.f, 0.f};
        if (u != nullptr) adb = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + 16 * rb + 4 * g);  // zero rows for j >= o
            abseed = abseed + gyv[j] * wj;
            if (u != nullptr) adb = adb + uv[j] * wj;
        }
        const f32x4 cs = KEPT ? kept_c(LH, rb) : *spill_at(wsp, LH, 0, rb, lane);
        const f32x4 zd = *spill_at(wsp, LH, 1, rb, lane);
        const f32x4 sn = KEPT ? kept_a(kA, lstride, toff, LH, rb)
                              : (THETA ? kept_a(A, lstride, toff, LH, rb) : *spill_at(wsp, LH, 2, rb, lane));
        actt[rb] = (w * cs) * adb;
        actp[rb] = (w * cs) * abseed - (w * w) * sn * zd * adb;
        if (THETA) {
            store_block4(D + LH * lstride + tbase, rb, actp[rb], stb, lane);
            store_block4(Dt + LH * lstride + tbase, rb, actt[rb], stb, lane);
        }
    }
    mark();
#pragma unroll 1
    for (int l = LH; l >= 1; --l) {
        layer_mma2(stream, ring, s, nslices, wave, lane, actp, actt, accp, acct);  // accp = ab, acct = adb (l-1)
        mark();
        const float wl = (l == 1) ? w0 : w;
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            const f32x4 cs = KEPT ? kept_c(l - 1, rb) : *spill_at(wsp, l - 1, 0, rb, lane);
            const f32x4 zd = *spill_at(wsp, l - 1, 1, rb, lane);
            const f32x4 sn = KEPT ? kept_a(kA, lstride, toff, l - 1, rb)
                                  : (THETA ? kept_a(A, lstride, toff, l - 1, rb) : *spill_at(wsp, l - 1, 2, rb, lane));
            const f32x4 wc = wl * cs;
            actt[rb] = wc * acct[rb];
            actp[rb] = wc * accp[rb] - (wl * wl) * sn * zd * acct[rb];
            if (THETA) {
                store_block4(D + (l - 1) * lstride + tbase, rb, actp[rb], stb, lane);
                store_block4(Dt + (l - 1) * lstride + tbase, rb, actt[rb], stb, lane);
            }
        }
        mark();
    }
    // ---- gx = W0^T zb_0 ------------------------------------------------------------------------------------
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (k < d) {
            float p = 0.f;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * g);
                p += wk[0] * actp[rb][0] + wk[1] * actp[rb][1] + wk[2] * actp[rb][2] + wk[3] * actp[rb][3];
            }
            p = sum_groups(p);
            if (valid && g == 0) gx[coord * d + k] = p;
        }
    }
    mark();
}

}  // namespace siren

// w1_kernel.hpp — the headline kernel: fused SIREN forward + coordinate vector-Jacobian product (W1) for
// gfx950, with every sin/cos epilogue interleaved into the NEXT layer's MFMA stream.
//
// Same math and tiling as fused_kernels.hpp (see there and DESIGN.md §3.1): v_mfma_f32_16x16x4_f32,
// weights as A operands from a 3-slot LDS ring of 16 KiB slices, activations as B operands in C/D layout.
// What is different:
//   * The L forward and L reverse GEMMs are fully unrolled (G = 0 .. 2L-1), so every slice index, ring slot
//     and register-array index is a compile-time constant: no branches inside the hot loop at all.
//   * Ping-pong accumulators acc[G & 1]: while GEMM G accumulates into acc[G&1] slice by slice, the epilogue
//     of GEMM G-1 (held in acc[(G+1)&1]) is applied one 16-neuron block ahead: during slice kb the wave
//     turns block kb+1 of the previous pre-activation into the B operand of slice kb+1. The ~25 VALU of each
//     sin/cos thus issue in the MFMA shadow (one wave per SIMD: the matrix pipe runs 32 cycles per MFMA).
//   * Epilogue per GEMM G (L = LH hidden layers):
//       G = 0         FIRST : z0 = x W0^T + b0 (VALU, K = d_in)  -> a_0 = sin(w0 z0), C[0] = cos(w0 z0)
//       1 <= G < L    SINCOS: z_G = acc + b_G                   -> a_G, C[G]
//       G = L         SEED  : z_L = acc + b_L -> y partials (a_L . Wout), delta_L = (gy Wout) . cos . w
//       L < G < 2L    DELTA : delta_{2L-G} = u . C[2L-G] . w
//     then after the last GEMM: delta_0 = u_0 . C[0] . w0 and gx = delta_0 W0.
//   * sincos_fast (siren_common.h) is branch-free: fma Cody-Waite with a full-precision pi/2, valid for
//     |w z| < 1e6 rad (|z| < 3.3e4 at w = 30), ~1e-7 absolute error.
// Requires outermost_linear (SingleBVPNet); the notebook Siren's final sine uses fused_kernel.
#pragma once
#include "siren_common.h"

namespace siren {

enum { EPI_FIRST = 0, EPI_SINCOS = 1, EPI_SEED = 2, EPI_DELTA = 3 };

// cos(w z_l) of layers l >= 1 is parked in AGPRs (the accumulator half of the unified register file): it is
// only read back once, by the reverse epilogue, while the VGPR half holds the B operands and the epilogue
// temporaries. The empty asm statements pin the register class; the moves are v_accvgpr_write/read.
__device__ __forceinline__ f32x4 to_agpr(f32x4 v) {
    f32x4 r;
    asm("; park in agpr" : "=a"(r) : "0"(v));
    return r;
}
// Opaque identity: materialises v here (LLVM would otherwise sink the cos bit-select to its use in the
// reverse sweep and keep ~5 intermediates per element alive across the whole forward pass).
__device__ __forceinline__ f32x4 pin(f32x4 v) {
    asm("; pin" : "+v"(v));
    return v;
}
__device__ __forceinline__ f32x4 from_agpr(f32x4 v) {
    f32x4 r;
    asm("; unpark" : "=v"(r) : "0"(v));
    return r;
}

template <int LH, bool STORE>
struct W1State {
    f32x4 act[NB];        // B operand of the current GEMM (filled one block ahead)
    f32x4 acc[2][NB];     // ping-pong accumulators
    f32x4 C[LH][NB];      // cos(w z_l), l = 0 .. LH-1
    float xv[MAXD];       // this lane's coordinate
    float gyv[MAXO];      // this lane's output cotangent
    float yp[MAXO];       // partial y over this lane's neurons
};

template <int LH, bool STORE>
struct W1Ctx {
    const float* stream;
    float* ring;
    const float* sm;
    int d, o, wave, lane, g;
    float w0, w;
    bool seed_ones;
    float* abuf;      // STORE: tile base (lane-adjusted) of layer 0; layer l at + l * lstride
    float* dbuf;
    int64_t lstride;
};

__device__ __forceinline__ void ring_issue_s(const float* __restrict__ stream, float* ring, int s, int wave, int lane) {
    const float* src = stream + (int64_t)s * SLICE + wave * 1024 + lane * 4;
    float* dst = ring + (s % NBUF) * SLICE + wave * 1024;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        __builtin_amdgcn_global_load_lds((const void*)(src + q * 256),
                                         (__attribute__((address_space(3))) void*)(dst + q * 256), 16, 0, 0);
}

// Epilogue for one 16-neuron block b of GEMM G (see the table at the top).
template <int G, int LH, bool STORE>
__device__ __forceinline__ void w1_epilogue(W1State<LH, STORE>& st, const W1Ctx<LH, STORE>& cx, int b) {
    constexpr int KIND = G == 0 ? EPI_FIRST : (G < LH ? EPI_SINCOS : (G == LH ? EPI_SEED : EPI_DELTA));
    const int nb = 16 * b + 4 * cx.g;
    if constexpr (KIND == EPI_FIRST) {
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < MAXD; ++k) {
            if (k < cx.d) {
                const f32x4 wk = *(const f32x4*)(cx.sm + SM_W0 + k * H + nb);
                z = k == 0 ? st.xv[0] * wk : z + st.xv[k] * wk;
            }
        }
        z += *(const f32x4*)(cx.sm + SM_BIAS + nb);
        f32x4 cs4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sn, cs;
            sincos_fast(cx.w0 * z[r], sn, cs);
            st.act[b][r] = sn;
            cs4[r] = cs;
        }
        st.C[0][b] = pin(cs4);
        if constexpr (STORE) store_block(cx.abuf, b, st.act[b]);
    } else if constexpr (KIND == EPI_SINCOS) {
        const f32x4 z = st.acc[(G + 1) & 1][b] + *(const f32x4*)(cx.sm + SM_BIAS + G * H + nb);
        f32x4 cs4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sn, cs;
            sincos_fast(cx.w * z[r], sn, cs);
            st.act[b][r] = sn;
            cs4[r] = cs;
        }
        st.C[G][b] = to_agpr(cs4);
        if constexpr (STORE) store_block(cx.abuf + G * cx.lstride, b, st.act[b]);
    } else if constexpr (KIND == EPI_SEED) {
        const f32x4 z = st.acc[(G + 1) & 1][b] + *(const f32x4*)(cx.sm + SM_BIAS + LH * H + nb);
        f32x4 sn, cs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a, c;
            sincos_fast(cx.w * z[r], a, c);
            sn[r] = a;
            cs[r] = c;
        }
        if constexpr (STORE) store_block(cx.abuf + LH * cx.lstride, b, sn);
        f32x4 ga = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            if (j < cx.o) {
                const f32x4 wj = *(const f32x4*)(cx.sm + SM_WO + j * H + nb);
                st.yp[j] += wj[0] * sn[0] + wj[1] * sn[1] + wj[2] * sn[2] + wj[3] * sn[3];
                if (!cx.seed_ones) ga += st.gyv[j] * wj;
            }
        }
        if (cx.seed_ones) ga = *(const f32x4*)(cx.sm + SM_SEED + nb);
        st.act[b] = (ga * cs) * cx.w;
        if constexpr (STORE) store_block(cx.dbuf + LH * cx.lstride, b, st.act[b]);
    } else {
        constexpr int L = 2 * LH - G;  // delta_L = u_L . cos(w z_L) . w,  1 <= L < LH
        st.act[b] = (st.acc[(G + 1) & 1][b] * from_agpr(st.C[L][b])) * cx.w;
        if constexpr (STORE) store_block(cx.dbuf + L * cx.lstride, b, st.act[b]);
    }
}

// GEMM G: 16 slices; slice kb multiplies B = act[kb] into acc[G & 1] while block kb+1 of the previous
// epilogue is produced.
template <int G, int LH, bool STORE, int SCHED>
__device__ __forceinline__ void w1_gemm(W1State<LH, STORE>& st, const W1Ctx<LH, STORE>& cx) {
    constexpr int NS = 2 * LH * NB;
    f32x4 (&acc)[NB] = st.acc[G & 1];
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) acc[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    w1_epilogue<G, LH, STORE>(st, cx, 0);
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
        const int s = G * NB + kb;
        // this wave's part of slice s has landed (slice s+1 may be in flight); barrier: all parts landed and
        // every wave is done with slice s-1's slot, which slice s+2 refills
        if (s + 1 < NS)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);  // nothing crosses the barrier (the scheduler would sink epilogues)
        if (s + 2 < NS) {
            const float* sp = cx.stream;
            asm volatile("" : "+s"(sp));  // keep the 96 slice addresses from being hoisted into SGPRs
            ring_issue_s(sp, cx.ring, s + 2, cx.wave, cx.lane);
        }
        const float* sl = cx.ring + (s % NBUF) * SLICE + cx.lane * 4;
        const f32x4 bop = st.act[kb];
        f32x4 a[NB];
#pragma unroll
        for (int ob = 0; ob < NB; ++ob) a[ob] = *(const f32x4*)(sl + ob * 256);
#pragma unroll
        for (int ob = 0; ob < NB; ob += 2) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                acc[ob] = mfma4(a[ob][r], bop[r], acc[ob]);
                acc[ob + 1] = mfma4(a[ob + 1][r], bop[r], acc[ob + 1]);
            }
        }
        if (kb + 1 < NB) w1_epilogue<G, LH, STORE>(st, cx, kb + 1);
        if constexpr (SCHED == 1) {
            // A operands two pairs ahead, then per pair 8 MFMAs each followed by a few epilogue VALU
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // DS_READ: pairs 0, 1
#pragma unroll
            for (int p = 0; p < NB / 2; ++p) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x002, 2, 0);  // VALU
                }
                if (p + 2 < NB / 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS_READ: pair p+2
            }
        }
    }
}

template <int G, int LH, bool STORE, int SCHED>
__device__ __forceinline__ void w1_run(W1State<LH, STORE>& st, const W1Ctx<LH, STORE>& cx) {
    if constexpr (G < 2 * LH) {
        w1_gemm<G, LH, STORE, SCHED>(st, cx);
        w1_run<G + 1, LH, STORE, SCHED>(st, cx);
    }
}

template <int LH, bool STORE, int SCHED = 0>
__global__ __launch_bounds__(THREADS, 1) void w1_kernel(const float* __restrict__ ws, const float* __restrict__ x,
                                                        int64_t n, const float* __restrict__ gy, float* __restrict__ y,
                                                        float* __restrict__ gx, int d, int o, float w0, float w,
                                                        float* __restrict__ abuf, float* __restrict__ dbuf,
                                                        int64_t n_pad) {
    __shared__ __attribute__((aligned(16))) float lds[NBUF * SLICE + SMALL_MAX];
    W1Ctx<LH, STORE> cx;
    W1State<LH, STORE> st;
    cx.ring = lds;
    float* sm = lds + NBUF * SLICE;
    cx.sm = sm;
    cx.lane = threadIdx.x & 63;
    cx.wave = threadIdx.x >> 6;
    cx.g = cx.lane >> 4;
    const int c = cx.lane & 15;
    cx.d = d;
    cx.o = o;
    cx.w0 = w0;
    cx.w = w;
    cx.seed_ones = gy == nullptr;
    cx.stream = ws + small_pad(LH);
    cx.lstride = n_pad * H;
    const int64_t toff = ((int64_t)blockIdx.x * WAVES + cx.wave) * (H * 16) + 4 * cx.g * 16 + c;
    cx.abuf = STORE ? abuf + toff : nullptr;
    cx.dbuf = STORE ? dbuf + toff : nullptr;

    {
        const int nf4 = (small_floats(LH) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t coord = (int64_t)blockIdx.x * TILE + cx.wave * 16 + c;
    const bool valid = coord < n;
#pragma unroll
    for (int k = 0; k < MAXD; ++k) st.xv[k] = (valid && k < d) ? x[coord * d + k] : 0.f;
#pragma unroll
    for (int j = 0; j < MAXO; ++j) {
        st.yp[j] = 0.f;
        st.gyv[j] = (gy != nullptr && valid && j < o) ? gy[coord * o + j] : 0.f;
    }
    __syncthreads();
    ring_issue_s(cx.stream, cx.ring, 0, cx.wave, cx.lane);
    ring_issue_s(cx.stream, cx.ring, 1, cx.wave, cx.lane);

    w1_run<0, LH, STORE, SCHED>(st, cx);

    // y (reduced over the 4 lane groups)
#pragma unroll
    for (int j = 0; j < MAXO; ++j) {
        if (j < o) {
            const float yj = sum_groups(st.yp[j]) + sm[SM_BOUT + j];
            if (y != nullptr && valid && cx.g == 0) y[coord * o + j] = yj;
        }
    }
    // delta_0 = u_0 . cos(w0 z_0) . w0 ;  gx = delta_0 W0
    constexpr int GL = (2 * LH - 1) & 1;
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) st.act[rb] = (st.acc[GL][rb] * st.C[0][rb]) * w0;
    if constexpr (STORE) store_tile(cx.dbuf, st.act);
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (k < d) {
            float p = 0.f;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * cx.g);
                p += wk[0] * st.act[rb][0] + wk[1] * st.act[rb][1] + wk[2] * st.act[rb][2] + wk[3] * st.act[rb][3];
            }
            p = sum_groups(p);
            if (valid && cx.g == 0) gx[coord * d + k] = p;
        }
    }
}

}  // namespace siren

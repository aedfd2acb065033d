#pragma once
// wide_jet_kernel.hpp — second order (W3) at hidden width 512 as a two-stream jet (the backward of
// the dPhi/dx graph node that gradients_mse / sdf / divergence differentiate at hidden_features=512,
// loss_functions.py:84-89, 214-238, diff_operators.py:27-43).
//
// At hidden 512 the W3 kernel's layout (primal and tangent as two separate 16-column tiles, w3_kernel.hpp) needs
// 2 x (activation + accumulator) = 512 registers per lane — more than a wave has. So the tangent rides in the SAME
// tile: a wave's 16 MFMA columns are 8 coordinates x 2 streams (column 2q + s: s = 0 the value z, s = 1 the tangent
// along v), and every weight A operand multiplies both streams at once — the register footprint of the hidden-512
// first-order kernel (wide_kernel.hpp: activation tile in VGPRs, accumulators in AGPRs).
//   forward (per layer):  z = W a + b [value only],  a = sin(w z0),  a' = w cos(w z0) z'        (z0: the pair's
//                         value, broadcast by DPP quad_perm [0,0,2,2]); the z-jet goes to a lane-major scratch and
//                         the a-jet to the wgrad tile layout
//   outputs:              y_j = Wout_j a + b_j (value lanes), ydot_j = Wout_j a' = (J v)_j (tangent lanes)
//   functional:           F = sum_c gy_c . y_c + u_c . ydot_c   (gy: first-order seed, u: output weighting = the
//                         cotangent of J^T u that siren_second_order_ex defines; NULL u = ones, NULL gy = none)
//   reverse seed:         ab_L = sum_j gy_j Wout_j (value), a'b_L = sum_j u_j Wout_j (tangent)
//   sine adjoint:         zb = w c ab - w^2 s z' a'b (value),  z'b = w c a'b (tangent)   (z' and a'b broadcast from
//                         the odd lane by quad_perm [1,1,3,3])
//   linear adjoint:       both streams through W^T (the transposed slices), zb-jets to the wgrad tile layout
//   gx = W0^T zb_0 (value lanes) = H v (+ the first-order gx of gy).
// theta-gradients: the split-K wgrad over 2n columns (dW_l = sum over both streams of zb_l x a_{l-1}, bias from the
// value columns: jet_bias 2) and edge_kernel<EDGE_J2> (dW0 = zb_0 x^T + z'b_0 v^T, dWout = gy a_L + u a'_L).
// One launch runs the forward and the reverse (like jet_store_kernel JET_BOTH), 32 KiB slices in the 3-slot ring of
// the hidden-512 kernels, operand reads by lds_ops.h.
#include "lds_ops.h"
#include "siren_common.h"
#include "siren_params.h"
#include "wide_kernel.hpp"

namespace siren {

template <int SEL>
__device__ __forceinline__ float pair_bcast(float v) {  // quad_perm [SEL, SEL, SEL + 2, SEL + 2]
    constexpr int ctrl = SEL | (SEL << 2) | ((SEL + 2) << 4) | ((SEL + 2) << 6);
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xf, 0xf, false));
}

// a-jet of z-jet (this lane's stream): ka = [value lane], kb = w [tangent lane]
__device__ __forceinline__ f32x4 jet2_sin(const f32x4& z, float w, float ka, float kb) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float sn, cs;
        sincos_fast(w * pair_bcast<0>(z[r]), sn, cs);
        out[r] = __builtin_fmaf(ka, sn, (kb * cs) * z[r]);
    }
    return out;
}

// cotangent of the z-jet from the cotangent u of the a-jet: m0 = [value lane]
__device__ __forceinline__ f32x4 jet2_sin_adjoint(const f32x4& u, const f32x4& z, float w, float m0) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float z0 = pair_bcast<0>(z[r]), zt = pair_bcast<1>(z[r]), ut = pair_bcast<1>(u[r]);
        float sn, cs;
        sincos_fast(w * z0, sn, cs);
        out[r] = __builtin_fmaf(w * cs, u[r], -(m0 * (w * w * sn)) * (zt * ut));
    }
    return out;
}

// NS = 4 (MIX): the third-order adjoint at hidden 512 (jet_kernel.hpp's mixed jet: streams value, tangent along v,
// tangent along g, mixed second order; 4 coordinates per wave): the backward of the Hessian-vector-product node
// h = sum_j u_j H_j v given its cotangent g (siren_hvp_backward); outputs gx (value lanes), gv = W0^T zb_0,v (out2)
// and gu_j = D2 y_j[v, g] (out3), seed sum_j u_j Wout_j on the second-order stream.
//
// grid.x = tiles of 64 / NS coordinates (4 waves x 16 / NS); abuf / dbuf: a- / zb-jets of layers 0..L as 16-column
// tiles [l][tile][neuron][16] with NS n_pad columns per layer; spill: z-jets lane-major, layer stride NS n_pad * 512.
// NS = 2: tg unused, out2 = ydot (n, o), out3 unused. NS = 4: gy unused, out2 = gv (n, d), out3 = gu (n, o).
template <int NS>
__global__ __launch_bounds__(THREADS, 1) void wide_jet_kernel(
    const float* __restrict__ ws, const float* __restrict__ x, const float* __restrict__ v,
    const float* __restrict__ tg, const float* __restrict__ gy, const float* __restrict__ u, int64_t n, int d, int o,
    int lh, float w0, float w, float* __restrict__ gx, float* __restrict__ out2, float* __restrict__ out3,
    float* __restrict__ spill, float* __restrict__ abuf, float* __restrict__ dbuf, int64_t n_pad) {
    static_assert(NS == 2 || NS == 4, "two-stream (W3) or four-stream (mixed) jets");
    constexpr int CPW = 16 / NS;  // coordinates per wave
    __shared__ __attribute__((aligned(16))) float lds[WNBUF * WSLICE + WSMALL_MAX];
    const SmallLayout L(WH);
    float* ring = lds;
    float* sm = lds + WNBUF * WSLICE;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15, js = c % NS;
    const int npass = 2 * lh;
    const int nslices = npass * WNB;
    const float* stream = ws + L.pad(lh);
    {
        const int nf4 = (L.floats(lh) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t coord = (int64_t)blockIdx.x * (WAVES * CPW) + wave * CPW + c / NS;
    const bool valid = coord < n;
    const int64_t wt = (int64_t)blockIdx.x * WAVES + wave;  // this wave's 16-column tile
    const int64_t lstride = NS * n_pad * WH;                  // floats per layer (NS n_pad columns)
    const int64_t toff = wt * (WH * 16) + 4 * g * 16 + c;     // tile layout: tile + lane
    float* sp = spill + wt * (WH * 16) + lane * 4;            // scratch: lane-major blocks
    const float val = js == 0 ? 1.f : 0.f;
    // per-lane jet coefficients: first-layer coefficient of W0[:, k] (x_k on the value stream, the tangent's
    // components on the tangent streams), the sine's stream factors and the adjoint's stream masks
    float jcf[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        const float* tp = (NS == 4 && js == 2) ? tg : v;
        jcf[k] = (valid && k < d && js < 3) ? (js == 0 ? x[coord * d + k] : tp[coord * d + k]) : 0.f;
    }
    const float kb0 = js == 0 ? 0.f : w0, kb = js == 0 ? 0.f : w;
    const float kg0 = (NS == 4 && js == 3) ? w0 * w0 : 0.f, kg = (NS == 4 && js == 3) ? w * w : 0.f;
    const float m12 = (js == 1 || js == 2) ? 1.f : 0.f;
    const bool s1 = js == 1;
    auto jsin = [&](const f32x4& z, float wl, float kbl, float kgl) -> f32x4 {
        if constexpr (NS == 2) return jet2_sin(z, wl, val, kbl);
        else return jet_sin<true>(z, wl, val, kbl, kgl);
    };
    auto jadj = [&](const f32x4& uu, const f32x4& z, float wl) -> f32x4 {
        if constexpr (NS == 2) return jet2_sin_adjoint(uu, z, wl, val);
        else return jet_sin_adjoint<true>(uu, z, wl, val, m12, s1);
    };
    __syncthreads();
    int s = 0;
    wring_issue(stream, ring, s, nslices, wave, lane);
    wring_issue(stream, ring, s + 1, nslices, wave, lane);

    // ---- first layer (K = d_in) on VALU: z_0 jet -> scratch, a_0 jet -> abuf -------------------------------------
    f32x4 act[WNB], acc[WNB];
#pragma unroll
    for (int rb = 0; rb < WNB; ++rb) {
        const int nb = 16 * rb + 4 * g;
        f32x4 z = val * *(const f32x4*)(sm + L.bias + nb);
#pragma unroll
        for (int k = 0; k < MAXD; ++k)
            if (k < d) z += jcf[k] * *(const f32x4*)(sm + L.w0 + k * WH + nb);
        *(f32x4*)(sp + rb * 256) = z;
        act[rb] = jsin(z, w0, kb0, kg0);
    }
    wstore_tile(abuf + toff, act);

#pragma unroll 1
    for (int p = 0; p < npass; ++p) {
#pragma unroll
        for (int ob = 0; ob < WNB; ++ob) acc[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
        // reverse passes: the stored z-jet block kb of the epilogue's layer goes into act[kb] once slice kb has
        // consumed it (as wide_kernel's cos prefetch; the ring's vmcnt(8) only waits for more)
        const bool rev_pass = p >= lh;
        const float* zpre = rev_pass ? sp + (int64_t)(2 * lh - p - 1) * lstride : sp;
#pragma unroll
        for (int kb2 = 0; kb2 < WNB; ++kb2) {
            wring_wait(s, nslices);
            wring_issue(stream, ring, s + 2, nslices, wave, lane);
            slice_mma<WNB>(lds_addr(ring + (s % WNBUF) * WSLICE) + 16u * lane, act[kb2], acc);
            if (rev_pass) act[kb2] = *(const f32x4*)(zpre + kb2 * 256);
            ++s;
        }
        if (p < lh) {
            // forward layer l = p + 1: z_l jet -> scratch, a_l jet -> abuf
            const int l = p + 1;
            const float* bl = sm + L.bias + l * WH + 4 * g;
            float* zp = sp + (int64_t)l * lstride;
#pragma unroll
            for (int rb = 0; rb < WNB; ++rb) {
                const f32x4 z = acc[rb] + val * *(const f32x4*)(bl + 16 * rb);
                *(f32x4*)(zp + rb * 256) = z;
                act[rb] = jsin(z, w, kb, kg);
            }
            wstore_tile(abuf + (int64_t)l * lstride + toff, act);
            if (l == lh) {
                // outputs per stream: NS = 2 ydot_j = (J v)_j on tangent lanes; NS = 4 gu_j = D2 y_j[v, g] on the
                // second-order lanes; then the reverse seed with this lane's output weights
                float wj_lane[MAXO];
                constexpr int OUT_STREAM = NS == 2 ? 1 : 3;
                float* outp = NS == 2 ? out2 : out3;
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    float pj = 0.f;
                    if (j < o) {
#pragma unroll
                        for (int rb = 0; rb < WNB; ++rb) {
                            const f32x4 wv = *(const f32x4*)(sm + L.wo + j * WH + 16 * rb + 4 * g);
                            pj += wv[0] * act[rb][0] + wv[1] * act[rb][1] + wv[2] * act[rb][2] + wv[3] * act[rb][3];
                        }
                        pj = sum_groups(pj);
                        if (valid && g == 0 && js == OUT_STREAM && outp != nullptr) outp[coord * o + j] = pj;
                    }
                    const float uj = (j < o) ? (u != nullptr ? (valid ? u[coord * o + j] : 0.f) : (valid ? 1.f : 0.f)) : 0.f;
                    if constexpr (NS == 2) {
                        const float gj = (gy != nullptr && valid && j < o) ? gy[coord * o + j] : 0.f;
                        wj_lane[j] = js == 0 ? gj : uj;
                    } else {
                        wj_lane[j] = js == 3 ? uj : 0.f;
                    }
                }
#pragma unroll
                for (int rb = 0; rb < WNB; ++rb) {
                    const float* wo = sm + L.wo + 16 * rb + 4 * g;  // rows j >= o are zero padded
                    const f32x4 ua = wj_lane[0] * *(const f32x4*)wo + wj_lane[1] * *(const f32x4*)(wo + WH) +
                                     wj_lane[2] * *(const f32x4*)(wo + 2 * WH) + wj_lane[3] * *(const f32x4*)(wo + 3 * WH);
                    const f32x4 z = acc[rb] + val * *(const f32x4*)(bl + 16 * rb);  // z_L jet, still in acc
                    act[rb] = jadj(ua, z, w);
                }
                wstore_tile(dbuf + (int64_t)lh * lstride + toff, act);
            }
        } else {
            // reverse through W_l (l = 2L - p): acc = cotangent of the a_{l-1} jet; act holds the z_{l-1} jet
            const int lm = 2 * lh - p - 1;
            const float wl = lm == 0 ? w0 : w;
#pragma unroll
            for (int rb = 0; rb < WNB; ++rb) act[rb] = jadj(acc[rb], act[rb], wl);
            wstore_tile(dbuf + (int64_t)lm * lstride + toff, act);
        }
    }

    // ---- gx = W0^T zb_0 (value lanes); NS = 4: gv = W0^T zb_0,v (stream-1 lanes) ------------------------------------
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (k < d) {
            float q = 0.f;
#pragma unroll
            for (int rb = 0; rb < WNB; ++rb) {
                const f32x4 wk = *(const f32x4*)(sm + L.w0 + k * WH + 16 * rb + 4 * g);
                q += wk[0] * act[rb][0] + wk[1] * act[rb][1] + wk[2] * act[rb][2] + wk[3] * act[rb][3];
            }
            q = sum_groups(q);
            if (valid && g == 0 && js == 0) gx[coord * d + k] = q;
            if (NS == 4 && out2 != nullptr && valid && g == 0 && js == 1) out2[coord * d + k] = q;
        }
    }
}

}  // namespace siren

#pragma once
// jet_kernel.hpp — W4s: the backward of the fused Laplacian (laplace_mse training, loss_functions.py:104-109).
//
// The forward is the W4 jet (w1_kernel MODE_JET): per coordinate, 4 jet streams (value, d/dx_1, d/dx_2,
// sum_i d2/dx_i2) of every layer, packed as 4 coordinates x 4 streams into the 16 MFMA columns of a wave. Its
// reverse is again a 16-column MFMA sweep: the cotangent of a layer's output jet goes back through W_l^T for all
// streams at once, and the elementwise coupling between the streams (jet_sin_adjoint, siren_common.h) runs in
// the epilogue with the quad's values exchanged by DPP. The weight gradient of layer l is then
//   dW_l = sum over all 16 columns of zb_l (jet of the layer-l pre-activation cotangent) x a_{l-1} (jet)
// i.e. wgrad_kernel over K = 4 N columns (bias: value columns only), and the first / output layers are reduced
// by edge_kernel<EDGE_JET> (train_kernels.hpp):
//   dW_0[:, k] = sum zb_0,value x_k + zb_0,tangent k     db_0 = sum zb_0,value     (z_0 = W0 x + b0, dz_0/dx_k = W0[:, k])
//   dWout[j]   = sum glap a_L,second                                               (lap = sum_j Wout_j a_L,second)
//   gx         = W0^T zb_0,value
//
// jet_store_kernel: forward jet (stores a-jets to abuf and, per stream lane, the reverse's combinations of the z jet —
// siren_common.h jet_sin_d; MIX / QG: the z jet itself — to a lane-major scratch), seed
// u_L,second = (sum_j Wout_j) glap, then the reverse sweep storing zb-jets to dbuf; one layer body for all 2L
// GEMM passes (runtime loop), 3-slot ring of 16 KiB slices (ring.hpp). Tiles are 16 columns = 4 coordinates.
// Split (laplace_mse training, SirenLaplace with a stored forward): PHASE JET_FWD runs the forward passes only —
// stores as above, plus the outputs y / grad / Laplacian from the last a-jet (the W4 forward's results) — and
// PHASE JET_REV the seed + reverse passes only from the stored z-jets; JET_BOTH is the single-launch form.
//
// MIX = true: the third-order adjoint (the backward of a Hessian-vector-product node h = sum_j u_j H_j(x) v, i.e.
// SirenHVP: laplace_mse through the reference's unfused divergence(gradient()), diff_operators.py:27-36, and the
// second jacobian() of helmholtz_pml / wave_pml, loss_functions.py:112-211). With g the cotangent of h,
//   S = sum_c <g_c, h_c> = sum_c sum_j u_j D2 y_j(x_c)[v_c, g_c]
// is the mixed second derivative of the network along two per-coordinate tangents, so the same 4-stream jet carries
// it: stream 0 value, stream 1 along v, stream 2 along g, stream 3 the mixed second order (jet_sin<true>). Its
// reverse gives every cotangent of the node at once:
//   gx = W0^T zb_0,value   gv = W0^T zb_0,v   gu_j = D2 y_j[v, g] (the forward's last jet)   dtheta as for W4s
// with the first layer's tangents W0 v / W0 g (per coordinate) and the output seed sum_j u_j Wout_j.
//
// QG = true (with MIX): the backward of a Hessian node Hm = sum_j u_j H_j(x) (n, d, d), d <= 2 — the node that every
// divergence() / hessian() column of one gradient node shares, so autograd sums all their cotangents into ONE
// cotangent G (n, d, d) and calls ONE backward. S = sum_c <G_c, Hm_c> = sum_c sum_j u_j D2 y_j(x_c)[Q_c] with
// Q = sym(G): the tangents are the coordinate axes (as the W4 jet) and the second-order stream follows the
// per-coordinate quadratic form Q (jet_sin_q / jet_sin_adjoint_q); tq (n, d, d) = G; gu_j = D2 y_j[Q].
#include <type_traits>

#include "lds_ops.h"
#include "ring.hpp"
#include "siren_common.h"
#include "siren_params.h"



namespace siren {

// Tile / scratch accessors that step their pointer through an opaque register: the compiler would otherwise
// hoist one 64-bit address per 16-neuron block (the offsets exceed the 12-bit immediate) and run out of VGPRs
// at 2 waves per SIMD.
__device__ __forceinline__ void jstore_tile(float* p, const f32x4 (&v)[NB]) {
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        store_block(p, 0, v[rb]);
        p += 256;
        asm volatile("" : "+v"(p));
    }
}
struct LaneBlocks {  // lane-major scratch: block rb of this lane at p + rb * 256
    float* p;
    __device__ __forceinline__ f32x4 next_load() {
        const f32x4 v = *gmem4(p);
        p += 256;
        asm volatile("" : "+v"(p));
        return v;
    }
    __device__ __forceinline__ void next_store(const f32x4& v) {
        *gmem4(p) = v;
        p += 256;
        asm volatile("" : "+v"(p));
    }
};

enum { JET_BOTH = 0, JET_FWD = 1, JET_REV = 2 };

// JET_FWD: glap is unused and the outputs go to y (n, o) / gx (n, d) / lap (n) (each nullable)
// MIX: tv / tg (n, d) the tangents v / g, tu (n, o) the output weighting (NULL = ones); gv (n, d) and gu (n, o)
// nullable outputs; glap unused (JET_BOTH only)
// (The backward of a Hessian node that kept its forward jets is qf_kernel.hpp: reverse GEMMs only, on the node's own
// 8-coordinate layout.)
// PH (!MIX): ws is the phase-scaled image (w1_ws: weights and biases carry w / 2 pi, W0 and b0 w0 / 2 pi), the jets are
// in revolutions (jet_sin_d_rev) and the reverse GEMMs return s u (s = w / 2 pi): the scratch holds D / s, the seed is
// s u_L, and gx undoes W0's scale (the zb / a-jet tiles are the true ones either way)
template <int PHASE, bool MIX = false, bool QG = false, bool PH = false>
__global__ __launch_bounds__(THREADS, 2) void jet_store_kernel(
    const float* __restrict__ ws, const float* __restrict__ x, int64_t n, const float* __restrict__ glap,
    float* __restrict__ gx, int d, int o, int lh, float w0, float w, float* __restrict__ spill,
    float* __restrict__ abuf, float* __restrict__ dbuf, int64_t n_pad, float* __restrict__ y,
    float* __restrict__ lap, const float* __restrict__ tv, const float* __restrict__ tg,
    const float* __restrict__ tu, float* __restrict__ gv, float* __restrict__ gu, const float* __restrict__ tq = nullptr) {
    static_assert(!MIX || PHASE == JET_BOTH, "the mixed jet runs as one launch");
    static_assert(!QG || MIX, "the quadratic-form jet is the mixed jet's variant");
    __shared__ __attribute__((aligned(16))) float lds[NBUF * SLICE + SMALL_MAX];
    float* ring = lds;
    float* sm = lds + NBUF * SLICE;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15, js = c & 3;
    const int nslices = (PHASE == JET_FWD ? 1 : 2) * lh * NB;  // JET_FWD never issues the reverse slices
    const float* stream = ws + small_pad(lh);
    {
        const int nf4 = (small_floats(lh) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t coord = (int64_t)blockIdx.x * 16 + wave * 4 + (c >> 2);
    const bool valid = coord < n;
    const int64_t wt = (int64_t)blockIdx.x * WAVES + wave;      // 16-column tile (4 coordinates)
    const int64_t lstride = 4 * n_pad * H;                      // floats per layer (n_pad coordinates)
    const int64_t toff = wt * (H * 16) + 4 * g * 16 + c;
    float* sp = spill + wt * (H * 16) + lane * 4;
    float xv[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) xv[k] = (valid && k < d) ? x[coord * d + k] : 0.f;
    const float val = js == 0 ? 1.f : 0.f;
    float jcf[MAXD];  // first-layer coefficients of W0[:, k] per stream
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if constexpr (QG) {  // tangents along the coordinate axes (d <= 2)
            jcf[k] = val * xv[k] + (js == k + 1 ? 1.f : 0.f);
        } else if constexpr (MIX) {
            const float* tp = js == 1 ? tv : tg;
            jcf[k] = (valid && k < d && (js == 1 || js == 2)) ? tp[coord * d + k] : val * xv[k];
        } else {
            jcf[k] = val * xv[k] + (js == k + 1 ? 1.f : 0.f);
        }
    }
    static_assert(!(PH && MIX), "the phase-scaled jets cover the Laplacian's jet only");
    constexpr float two_pi = 6.28318530717958648f, four_pi2 = 39.4784176043574344f;
    const float s_h = w * 0.159154943091895336f;  // PH: the hidden layers' pack scale s = w / 2 pi
    const float rw0 = w0 / s_h;                   // PH: layer 0's w0 over the reverse scale
    const float kb0 = js == 0 ? 0.f : (PH ? two_pi : w0), kg0 = js == 3 ? (PH ? four_pi2 : w0 * w0) : 0.f;
    const float kb = js == 0 ? 0.f : (PH ? two_pi : w), kg = js == 3 ? (PH ? four_pi2 : w * w) : 0.f;
    // !MIX: the scratch holds the reverse's combinations of the z jet (jet_sin_d), per layer scale w0 / w; PH: in
    // revolutions and over s (layer l's dA, dB, dC = (w_l / s) (1, 2 pi, 4 pi^2): 2 pi (1, 2 pi, 4 pi^2) for l >= 1)
    const float dA0 = js == 0 ? (PH ? rw0 : w0) : 0.f, dB0 = js == 0 ? 0.f : (PH ? two_pi * rw0 : w0 * w0),
                dC0 = js == 3 ? (PH ? four_pi2 * rw0 : w0 * w0 * w0) : 0.f;
    const float dA = js == 0 ? (PH ? two_pi : w) : 0.f, dB = js == 0 ? 0.f : (PH ? four_pi2 : w * w),
                dC = js == 3 ? (PH ? two_pi * four_pi2 : w * w * w) : 0.f;
    const float m12 = (js == 1 || js == 2) ? 1.f : 0.f;
    const float gl = (PHASE != JET_FWD && valid && js == 3) ? (MIX ? 1.f : (PH ? s_h : 1.f) * glap[coord]) : 0.f;
    const bool s1 = js == 1;
    // QG: this lane's row of 2 Q (streams 1, 2; Q = sym(G), G (n, d, d), d <= 2) for jet_sin_q / jet_sin_adjoint_q
    f32x2 qreg = {0.f, 0.f};
    if constexpr (QG) {
        if (valid && (js == 1 || js == 2)) {
            const float* gq = tq + coord * d * d;
            const float q12x2 = d > 1 ? gq[1] + gq[2] : 0.f;
            qreg[0] = js == 1 ? 2.f * gq[0] : q12x2;
            qreg[1] = js == 1 ? q12x2 : (d > 1 ? 2.f * gq[3] : 0.f);
        }
    }
    auto qload = [&]() -> f32x2 { return qreg; };
    __syncthreads();
    const int p0 = PHASE == JET_REV ? lh : 0, p1 = PHASE == JET_FWD ? lh : 2 * lh;
    int s = p0 * NB;
    ring_issue(stream, ring, s, nslices, wave, lane);
    ring_issue(stream, ring, s + 1, nslices, wave, lane);
    // slice s0 published before the first pass (its successors are published by the mid-slice barriers)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    // ---- first layer: z_0 jet (VALU, K = d_in) ---------------------------------------------------------------
    f32x4 act[NB], acc[NB];
    if (PHASE == JET_REV) {
        // seed from the stored z_L jet (the JET_FWD launch's scratch)
        LaneBlocks zl{sp + (int64_t)lh * lstride};
        f32x4 dv[NB];  // every block in flight at once (as the reverse epilogues below)
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) dv[rb] = zl.next_load();
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            const f32x4 u = gl * *(const f32x4*)(sm + SM_SEED + 16 * rb + 4 * g);
            act[rb] = jet_sin_adjoint_d(u, dv[rb], val, m12);
        }
        jstore_tile(dbuf + (int64_t)lh * lstride + toff, act);
    } else {
        LaneBlocks zs{sp};
        const f32x2 qc = qload();
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            const int nb = 16 * rb + 4 * g;
            f32x4 z = val * *(const f32x4*)(sm + SM_BIAS + nb);
#pragma unroll
            for (int k = 0; k < MAXD; ++k)
                if (k < d) z += jcf[k] * *(const f32x4*)(sm + SM_W0 + k * H + nb);
            if constexpr (QG) {
                f32x4 kz;
                act[rb] = jet_sin_q(z, w0, val, kb0, kg0, qc[0], qc[1], js == 3, kz);
                zs.next_store(kz);
            } else if constexpr (MIX) {
                zs.next_store(z);
                act[rb] = jet_sin<MIX>(z, w0, val, kb0, kg0);
            } else {
                f32x4 dz;
                act[rb] = PH ? jet_sin_d_rev(z, val, kb0, kg0, dA0, dB0, dC0, dz)
                             : jet_sin_d(z, w0, val, kb0, kg0, dA0, dB0, dC0, dz);
                zs.next_store(dz);
            }
        }
        jstore_tile(abuf + toff, act);
    }

#pragma unroll 1
    for (int p = p0; p < p1; ++p) {
        {
#pragma unroll
            for (int ob = 0; ob < NB; ++ob) acc[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
            // mid-slice ring protocol (ring_mid / slice_mma_mid): the operand reads run on across the slice seams
            const unsigned rbase = lds_addr(ring) + 16u * lane;
            f32x4 a0 = lds_read4<0>(rbase + (s % NBUF) * SLICE * 4);
            f32x4 a1 = lds_read4<1024>(rbase + (s % NBUF) * SLICE * 4);
#pragma unroll
            for (int kb2 = 0; kb2 < NB; ++kb2) {
                const unsigned va = rbase + (s % NBUF) * SLICE * 4, vn = rbase + ((s + 1) % NBUF) * SLICE * 4;
                auto mid = [&]() { ring_mid(stream, ring, s, nslices, wave, lane); };
                if (kb2 + 1 < NB)
                    slice_mma_mid<NB, 4, true>(va, vn, act[kb2], acc, a0, a1, a0, a1, mid);
                else
                    slice_mma_mid<NB, 4, false>(va, vn, act[kb2], acc, a0, a1, a0, a1, mid);
                ++s;
            }
        }
        if (p < lh) {
            // forward layer l = p + 1: z_l jet -> scratch, a_l jet -> abuf
            const int l = p + 1;
            const float* bl = sm + SM_BIAS + l * H + 4 * g;
            float* zp = sp + (int64_t)l * lstride;
            LaneBlocks zs{zp};
            const f32x2 qc = qload();
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 z = acc[rb] + val * *(const f32x4*)(bl + 16 * rb);
                if constexpr (QG) {
                    f32x4 kz;
                    act[rb] = jet_sin_q(z, w, val, kb, kg, qc[0], qc[1], js == 3, kz);
                    zs.next_store(kz);
                } else if constexpr (MIX) {
                    zs.next_store(z);
                    act[rb] = jet_sin<MIX>(z, w, val, kb, kg);
                } else {
                    f32x4 dz;
                    act[rb] = PH ? jet_sin_d_rev(z, val, kb, kg, dA, dB, dC, dz)
                                 : jet_sin_d(z, w, val, kb, kg, dA, dB, dC, dz);
                    zs.next_store(dz);
                }
            }
            jstore_tile(abuf + (int64_t)l * lstride + toff, act);
            if (PHASE == JET_FWD && l == lh) {
                // outputs per stream (the W4 forward's): y_j (value), sum_j dy_j/dx_k (tangent k), sum_j Lap y_j
                float tot = 0.f;
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    if (j < o) {
                        float pj = 0.f;
#pragma unroll
                        for (int rb = 0; rb < NB; ++rb) {
                            const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + 16 * rb + 4 * g);
                            pj += wj[0] * act[rb][0] + wj[1] * act[rb][1] + wj[2] * act[rb][2] + wj[3] * act[rb][3];
                        }
                        const float vj = sum_groups(pj) + val * sm[SM_BOUT + j];
                        if (y != nullptr && valid && g == 0 && js == 0) y[coord * o + j] = vj;
                        tot += vj;
                    }
                }
                if (valid && g == 0) {
                    if (js == 3) {
                        if (lap != nullptr) lap[coord] = tot;
                    } else if (js >= 1 && js <= d && gx != nullptr) {
                        gx[coord * d + js - 1] = tot;
                    }
                }
            }
            if (MIX && gu != nullptr && l == lh) {
                // gu_j = D2 y_j[v, g] = Wout_j . a_L,second (stream 3 lanes; the bias only enters stream 0)
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    if (j < o) {
                        float pj = 0.f;
#pragma unroll
                        for (int rb = 0; rb < NB; ++rb) {
                            const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + 16 * rb + 4 * g);
                            pj += wj[0] * act[rb][0] + wj[1] * act[rb][1] + wj[2] * act[rb][2] + wj[3] * act[rb][3];
                        }
                        pj = sum_groups(pj);
                        if (valid && g == 0 && js == 3) gu[coord * o + j] = pj;
                    }
                }
            }
            if (PHASE == JET_BOTH && l == lh) {
                // seed: u_L (cotangent of the a_L jet) = (sum_j Wout_j) glap on the second-order stream only
                // (MIX: sum_j u_j Wout_j), then zb_L = adjoint of the last sine layer
                LaneBlocks zl{zp};
                const f32x2 qc = qload();
                float uw[MAXO];  // MIX: this coordinate's output weighting (the seed is sum_j u_j Wout_j)
#pragma unroll
                for (int j = 0; j < MAXO; ++j)
                    uw[j] = (MIX && j < o) ? (tu != nullptr ? (valid ? tu[coord * o + j] : 0.f) : 1.f) : 0.f;
#pragma unroll
                for (int rb = 0; rb < NB; ++rb) {
                    f32x4 sd;
                    if constexpr (MIX) {  // WoT rows j >= o are zero padded: branch-free sum over all 4
                        const float* wo = sm + SM_WO + 16 * rb + 4 * g;
                        sd = uw[0] * *(const f32x4*)wo + uw[1] * *(const f32x4*)(wo + H) +
                             uw[2] * *(const f32x4*)(wo + 2 * H) + uw[3] * *(const f32x4*)(wo + 3 * H);
                    } else {
                        sd = *(const f32x4*)(sm + SM_SEED + 16 * rb + 4 * g);
                    }
                    act[rb] = QG    ? jet_sin_adjoint_q(gl * sd, zl.next_load(), w, val, m12, qc[0], qc[1])
                              : MIX ? jet_sin_adjoint<MIX>(gl * sd, zl.next_load(), w, val, m12, s1)
                                    : jet_sin_adjoint_d(gl * sd, zl.next_load(), val, m12);
                }
                jstore_tile(dbuf + (int64_t)lh * lstride + toff, act);
            }
        } else {
            // reverse through W_l (l = 2L - p): acc = u_{l-1}, zb_{l-1} = adjoint of sine layer l-1
            const int lm = 2 * lh - p - 1;
            LaneBlocks zl{sp + (int64_t)lm * lstride};
            const float wl = lm == 0 ? w0 : w;
            const f32x2 qc = qload();
            if constexpr (!MIX) {
                // all 16 blocks of the combinations in flight at once (a load per block one block ahead waited out
                // 16 memory latencies per layer; the linear adjoint leaves the registers for it)
                f32x4 dv[NB];
#pragma unroll
                for (int rb = 0; rb < NB; ++rb) dv[rb] = zl.next_load();
#pragma unroll
                for (int rb = 0; rb < NB; ++rb) act[rb] = jet_sin_adjoint_d(acc[rb], dv[rb], val, m12);
            } else {
#pragma unroll
                for (int rb = 0; rb < NB; ++rb) {
                    act[rb] = QG ? jet_sin_adjoint_q(acc[rb], zl.next_load(), wl, val, m12, qc[0], qc[1])
                                 : jet_sin_adjoint<MIX>(acc[rb], zl.next_load(), wl, val, m12, s1);
                }
            }
            jstore_tile(dbuf + (int64_t)lm * lstride + toff, act);
        }
    }

    if (PHASE == JET_FWD) return;
    // ---- gx = W0^T zb_0 (value stream); MIX: gv = W0^T zb_0 (stream 1, the cotangent of v) ----------------------
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (k < d) {
            float q = 0.f;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * g);
                q += wk[0] * act[rb][0] + wk[1] * act[rb][1] + wk[2] * act[rb][2] + wk[3] * act[rb][3];
            }
            q = sum_groups(q) * (PH ? two_pi / w0 : 1.f);  // PH: LDS W0^T carries w0 / 2 pi
            if (valid && g == 0 && js == 0) gx[coord * d + k] = q;
            if (MIX && gv != nullptr && valid && g == 0 && js == 1) gv[coord * d + k] = q;
        }
    }
}

}  // namespace siren

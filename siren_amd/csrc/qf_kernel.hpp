#pragma once
// qf_kernel.hpp — the backward of the Hessian node reading its forward jets from the node's KEEP scratch
// (siren_hessian_backward_kept) with its epilogues BETWEEN the reverse GEMMs (round 4; the A/B baseline of
// qfi_kernel.hpp, SIREN_FLAG_QF_SERIAL). Math and layout: qf_common.hpp.
#include "lds_ops.h"
#include "qf_common.hpp"
#include "ring.hpp"
#include "siren_params.h"

namespace siren {

constexpr int QF_PREFETCH = 3;  // kept blocks loaded ahead of the epilogue element that consumes them

// gx (n, d) = W0^T zb_0,value; gu (n, o) nullable = D2 y_j[Q]; tu (n, o) nullable output weighting (NULL = ones);
// G (n, d, d); kept = the Hessian node's KEEP scratch of the same (ws, x, n); abuf / dbuf: a- / zb-jet tiles of layers
// 0..L. Grid: hess_groups(n) / 4 workgroups of 4 waves (8 coordinates each).
__global__ __launch_bounds__(THREADS, 1) void qf_rev_kernel(const float* __restrict__ ws, const float* __restrict__ x,
                                                            int64_t n, const float* __restrict__ G,
                                                            const float* __restrict__ tu,
                                                            const float* __restrict__ kept, float* __restrict__ gx,
                                                            float* __restrict__ gu, int d, int o, int lh, float w0,
                                                            float w, float* __restrict__ abuf, float* __restrict__ dbuf,
                                                            int64_t n_pad) {
    __shared__ __attribute__((aligned(16))) float lds[NBUF * SLICE + SMALL_MAX];
    float* ring = lds;
    float* sm = lds + NBUF * SLICE;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR): never a spilled VGPR
    const int g = lane >> 4, c = lane & 15;
    const bool hi = c >= 8;
    const int nslices = 2 * lh * NB;
    const float* stream = ws + small_pad(lh);
    {
        const int nf4 = (small_floats(lh) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t ngroups = hess_groups(n);
    const int64_t grp = (int64_t)blockIdx.x * WAVES + wave;
    const int64_t coord = grp * 8 + (c & 7);
    const bool valid = coord < n;
    const int64_t lstride = 4 * n_pad * H;                  // floats per layer of abuf / dbuf
    const int64_t toff = 2 * grp * (H * 16) + 4 * g * 16 + c;  // tile 0 of the pair; tile 1 at + H * 16
    const float* kp = kept + hess_kept_off(ngroups, lh, 1, grp, 0, 0, lane);  // layer 1 (layer 0 is rebuilt)
    const int64_t kl = hess_kept_lstride(ngroups);  // floats between layers of the kept scratch
    QfCoef q;
    {
        const float* gq = G + coord * d * d;
        q.q11 = valid ? gq[0] : 0.f;
        q.q12 = (valid && d > 1) ? gq[1] + gq[2] : 0.f;
        q.q22 = (valid && d > 1) ? gq[3] : 0.f;
        q.e1 = hi ? q.q11 : 0.f;
        q.e2 = hi ? q.q22 : q.q12;
        q.ca = hi ? 2.f * q.q11 : q.q12;
        q.cb = hi ? q.q12 : 2.f * q.q22;
        q.mlo = hi ? 0.f : 1.f;
    }
    __syncthreads();
    // the ring starts at the first reverse slice (the stream's transposed layers)
    int s = lh * NB;
    ring_issue(stream, ring, s, nslices, wave, lane);
    ring_issue(stream, ring, s + 1, nslices, wave, lane);

    f32x4 act[2][NB], acc[2][NB];
    // one layer's epilogue: acc (cotangent of the a-jet of layer lm) + kept z-jet -> a-jet (abuf) and zb (act, dbuf);
    // the kept blocks are loaded QF_PREFETCH blocks ahead
    auto epilogue = [&](int lm, auto seed) {
        constexpr bool SEED = decltype(seed)::value;
        const float wl = lm == 0 ? w0 : w, wl2 = wl * wl;
        const bool rebuild = lm == 0;  // wave-uniform: layer 0's jet comes from x, not from the kept scratch
        const float* kr = kp + (rebuild ? 0 : lm - 1) * kl;
        float* ap = abuf + (int64_t)lm * lstride + toff;
        float* dp = dbuf + (int64_t)lm * lstride + toff;
        QfKept kq[QF_PREFETCH];
        float x0 = 0.f, x1 = 0.f;  // (loaded here, not held across the kernel: the register budget is full)
        if (!rebuild) {
#pragma unroll
            for (int i = 0; i < QF_PREFETCH; ++i) kq[i] = qf_load(kr + i * 768);
        } else {
            x0 = valid ? x[coord * d] : 0.f;
            x1 = (valid && d > 1) ? x[coord * d + 1] : 0.f;
        }
        float uw[MAXO], gup[MAXO];
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            uw[j] = (SEED && valid && j < o) ? (tu != nullptr ? tu[coord * o + j] : 1.f) : 0.f;
            gup[j] = 0.f;
        }
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            const QfKept kc = rebuild ? qf_layer0(sm, rb, g, hi, x0, x1) : kq[rb % QF_PREFETCH];
            asm volatile("" ::: "memory");  // keep the prefetch distance: no hoisting of the layer's 48 loads
            if (!rebuild && rb + QF_PREFETCH < NB) kq[rb % QF_PREFETCH] = qf_load(kr + (rb + QF_PREFETCH) * 768);
            f32x4 ua, ub;
            if constexpr (SEED) {
                // the cotangent of the a_L jet lives on the Q stream only: u_3 = sum_j u_j Wout_j (hi lanes, tile 1)
                const float* wo = sm + SM_WO + 16 * rb + 4 * g;  // WoT rows j >= o are zero padded
                const f32x4 sd = uw[0] * *(const f32x4*)wo + uw[1] * *(const f32x4*)(wo + H) +
                                 uw[2] * *(const f32x4*)(wo + 2 * H) + uw[3] * *(const f32x4*)(wo + 3 * H);
                const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
                ua = zero;
                ub = hi ? sd : zero;
            } else {
                ua = acc[0][rb];
                ub = acc[1][rb];
            }
            f32x4 aa, ab;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float ea, eb, za, zb;
                qf_elem(kc.k[0][r], kc.k[1][r], kc.k[2][r], ua[r], ub[r], wl, wl2, q, hi, ea, eb, za, zb, !rebuild);
                aa[r] = ea;
                ab[r] = eb;
                act[0][rb][r] = za;
                act[1][rb][r] = zb;
            }
            if constexpr (!SEED) qf_store_block(ap, aa);  // a_L's value / d/dx_1 streams feed no gradient
            qf_store_block(ap + H * 16, ab);
            qf_store_block(dp, act[0][rb]);
            qf_store_block(dp + H * 16, act[1][rb]);
            ap += 256;
            dp += 256;
            asm volatile("" : "+v"(ap), "+v"(dp));
            if constexpr (SEED) {  // gu_j = Wout_j . a_L,3 (hi lanes' tile-1 a-jet)
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + 16 * rb + 4 * g);
                    gup[j] += wj[0] * ab[0] + wj[1] * ab[1] + wj[2] * ab[2] + wj[3] * ab[3];
                }
            }
        }
        if constexpr (SEED) {
            if (gu != nullptr) {
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    const float pj = sum_groups(gup[j]);
                    if (j < o && valid && g == 0 && hi) gu[coord * o + j] = pj;
                }
            }
        }
    };

    // seed at layer L from the kept z_L jet (no forward sweep), then the L reverse GEMMs
    epilogue(lh, std::true_type{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // slice s landed (and the seed's stores): publish it
    __builtin_amdgcn_s_barrier();
#pragma unroll 1
    for (int p = lh; p < 2 * lh; ++p) {
#pragma unroll
        for (int ob = 0; ob < NB; ++ob) acc[0][ob] = acc[1][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
        {
            const unsigned rbase = lds_addr(ring) + 16u * lane;
            f32x4 a = lds_read4<0>(rbase + (s % NBUF) * SLICE * 4);
#pragma unroll
            for (int kb = 0; kb < NB; ++kb) {
                const unsigned va = rbase + (s % NBUF) * SLICE * 4, vn = rbase + ((s + 1) % NBUF) * SLICE * 4;
                auto mid = [&]() { ring_mid(stream, ring, s, nslices, wave, lane); };
                if (kb + 1 < NB)
                    slice_mma2_mid<NB, NB / 2, true>(va, vn, act[0][kb], act[1][kb], acc[0], acc[1], a, a, mid);
                else
                    slice_mma2_mid<NB, NB / 2, false>(va, vn, act[0][kb], act[1][kb], acc[0], acc[1], a, a, mid);
                ++s;
            }
        }
        epilogue(2 * lh - p - 1, std::false_type{});
    }

    // ---- gx = W0^T zb_0,value (tile 0, lo lanes) ---------------------------------------------------------------
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (k < d) {
            float qk = 0.f;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * g);
                qk += wk[0] * act[0][rb][0] + wk[1] * act[0][rb][1] + wk[2] * act[0][rb][2] + wk[3] * act[0][rb][3];
            }
            qk = sum_groups(qk);
            if (valid && g == 0 && !hi) gx[coord * d + k] = qk;
        }
    }
}

}  // namespace siren

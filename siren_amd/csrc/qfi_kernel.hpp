#pragma once
// qfi_kernel.hpp — the kept backward of the Hessian node (siren_hessian_backward_kept) with every epilogue interleaved
// into the NEXT reverse GEMM's MFMA stream: qf_common.hpp's math and Q8 layout on w3i_kernel.hpp's schedule.
//
// qf_rev_kernel ran each layer's epilogue (kept z-jet loads, the quadratic-form jet adjoint, four tile stores per
// block) between two reverse GEMMs. At one wave per SIMD nothing covered it, and with every CU in the same phase the
// GPU moved its HBM traffic in bursts while the matrix pipe idled: 0.51 MFMA busy. Here, as in w1 / w3i:
//   * The L reverse GEMMs are fully unrolled (G = 0 .. L-1: G carries the cotangent of layer L - G down through
//     W_{L-G}^T). GEMM G accumulates both column tiles of the Q8 pair into acc[G & 1]; the epilogue that turns GEMM
//     G-1's output (the a-jet cotangent of layer L - G) into GEMM G's B operands (the z-jet cotangent zb of that layer)
//     runs one 16-neuron block ahead, inside slice kb for block kb + 1, as one VALU cluster after the last operand pair.
//     G = 0's epilogue is the seed (the output weighting u on the Q stream of layer L, no GEMM before it).
//   * B operands are built just in time: a two-slot register ring (block kb & 1) instead of a whole tile, so the two
//     accumulator sets (256 registers) fit beside the kept-jet reloads and the staged tile blocks at one wave per SIMD
//     (round 4's interleaved attempt kept a full B tile and spilled 93-177 VGPRs).
//   * Epilogue E = G NB + b reads the kept z-jet of layer L - G, block b (3 x 16 B per lane, saddr-form loads issued at
//     the mid-slice barrier three slices ahead, retired by that slice's counted vmcnt) and stages its four tile blocks
//     (a-jet pair, zb pair; the seed's a-jet value stream feeds no gradient and is skipped) through a per-wave LDS
//     transpose into one coalesced 1 KiB store each, issued early in the slice that consumes the block.
//   * Every mid-slice s_waitcnt vmcnt(N) counts the vector-memory ops issued after the ring slice it publishes (a load's
//     data waits for every older load AND store: they retire in issue order), compile-time per slice.
//   * After the last GEMM, the layer-0 epilogue (the jet rebuilt from x, qf_layer0) runs serially: a_0 / zb_0 tiles and
//     gx = W0^T zb_0,value.
// Results are bitwise those of qf_rev_kernel (same per-element arithmetic, qf_elem; tests/test_gpu_third_order.py).
#include "qf_common.hpp"
#include "w3i_kernel.hpp"

#ifndef QFI_EPI_PAIR
#define QFI_EPI_PAIR 7  // operand pair after which the epilogue cluster runs (>= 4: after the mid-slice reload wait)
#endif
// operand pair after whose wait the previous epilogue's tile blocks are stored (< QFI_EPI_PAIR, which restages them;
// >= 4: behind the mid-slice ring refill). Measured (profiles/r05c_qfi_probes.log, r05d): pair 0 5.14 ms, behind the
// refill 5.50 ms
#ifndef QFI_STORE_PAIR
#define QFI_STORE_PAIR 0
#endif
static_assert(QFI_EPI_PAIR >= 4 && QFI_EPI_PAIR < siren::NB / 2, "the kept reloads land at the mid-slice wait");
static_assert(QFI_STORE_PAIR >= 0 && QFI_STORE_PAIR < QFI_EPI_PAIR, "the epilogue restages the tile blocks");

namespace siren {

// vector-memory ops of epilogue E: kept reloads (3 per block) and tile stores (4; 3 for the seed, G = 0)
template <int E, int LH>
constexpr int qfi_nrl() {
    return (E < 0 || E >= LH * NB) ? 0 : 3;
}
template <int E, int LH>
constexpr int qfi_nst() {
    return (E < 0 || E >= LH * NB) ? 0 : (E < NB ? 3 : 4);
}

template <int LH>
struct QfiState {
    f32x4 b[2][2];           // B operands [block & 1][tile] of the current slice and the next
    f32x4 acc[2][2][NB];     // ping-pong accumulators [G & 1][tile][output block]
    f32x4 pa0, pa1;          // the next slice's first operand pair (in flight)
    f32x4 pk[3][3];          // kept z-jet of epilogue E in slot E % 3: this lane's three streams
    f32x4 tq[4];             // the last epilogue's tile blocks, transposed (stored at the start of the next slice)
    float uw[MAXO], gup[MAXO];  // seed: this coordinate's output weighting u_j, partial D2 y_j[Q]
};

struct QfiCtx {
    const float* stream;
    float* ring;
    const float* sm;
    int wave, lane, g;
    bool hi;
    float w, w2;
    QfCoef q;
    unsigned ring_vaddr, sm_vaddr;
    const char* kb;          // kept scratch of this wave's group, layer 1 (wave-uniform); layer l at + (l - 1) kl
    int64_t kl;              // bytes between the layers of the kept scratch
    const char* ta;          // a-jet / zb-jet tile pair of this wave's group, layer 0 (wave-uniform); layer l at + l lb
    const char* td;
    int64_t lb;              // bytes between the layers of the tile buffers
    unsigned vl;             // 16 lane
    unsigned tw, tr;         // LDS transpose scratch of the wave: this lane's write / read address
};

template <int E, int LH>
__device__ __forceinline__ void qfi_reload_issue(QfiState<LH>& st, const QfiCtx& cx) {
    if constexpr (E < LH * NB) {
        constexpr int G = E / NB, B = E % NB, L = LH - G;
#pragma unroll
        for (int t = 0; t < 3; ++t)
            w3_load16_once(st.pk[E % 3][t], w3_at(cx.kb, (int64_t)(L - 1) * cx.kl + (B * 3 + t) * 1024), cx.vl);
    }
}
template <int E, int LH>
__device__ __forceinline__ void qfi_reload_landed(QfiState<LH>& st) {
    if constexpr (E < LH * NB) asm volatile("" : "+v"(st.pk[E % 3][0]), "+v"(st.pk[E % 3][1]), "+v"(st.pk[E % 3][2]));
}

// stores of the tile blocks epilogue E staged (staging order: [a-jet tile 0 unless seed], a-jet tile 1, zb tile 0, 1)
template <int E, int LH>
__device__ __forceinline__ void qfi_tile_flush(QfiState<LH>& st, const QfiCtx& cx) {
    if constexpr (E < LH * NB) {
        constexpr int G = E / NB, B = E % NB, L = LH - G;
        constexpr int NT = qfi_nst<E, LH>();
#pragma unroll
        for (int i = 0; i < NT; ++i) asm volatile("" : "+v"(st.tq[i]));  // landed (the caller's lgkmcnt wait)
        const int64_t off = (int64_t)L * cx.lb + B * 1024;
        constexpr int A0 = NT == 4 ? 1 : 0;
        if constexpr (NT == 4) w3_store16(w3_at(cx.ta, off), cx.vl, st.tq[0]);
        w3_store16(w3_at(cx.ta, off + 16384), cx.vl, st.tq[A0]);
        w3_store16(w3_at(cx.td, off), cx.vl, st.tq[A0 + 1]);
        w3_store16(w3_at(cx.td, off + 16384), cx.vl, st.tq[A0 + 2]);
    }
}

// seed parameters of block b: the output layer's rows Wout_j (zero padded for j >= d_out)
struct QfiSeed {
    f32x4 wo[MAXO];
};
template <int B>
__device__ __forceinline__ void qfi_seed_issue(QfiSeed& sp, unsigned sm_vaddr) {
    static_for<0, MAXO>([&](auto J) {
        constexpr int j = decltype(J)::value;
        sp.wo[j] = lds_read4<4 * (SM_WO + j * H + 16 * B)>(sm_vaddr);
    });
}
__device__ __forceinline__ void qfi_seed_load(QfiSeed& sp, const QfiCtx& cx, int b) {
#pragma unroll
    for (int j = 0; j < MAXO; ++j) sp.wo[j] = *(const f32x4*)(cx.sm + SM_WO + j * H + 16 * b + 4 * cx.g);
}

// The epilogue that builds block b of GEMM G's B operands from the kept z-jet in slot `slot` and (G > 0) GEMM G-1's
// output, and stages its four tile blocks (qf_rev_kernel's epilogue for one block, same arithmetic: qf_elem).
template <int G, int LH>
__device__ __forceinline__ void qfi_epilogue(QfiState<LH>& st, const QfiCtx& cx, int b, int slot,
                                             const QfiSeed& sp) {
    constexpr bool SEED = G == 0;
    f32x4 ua, ub;
    if constexpr (SEED) {
        // the cotangent of the a_L jet lives on the Q stream only: u_3 = sum_j u_j Wout_j (hi lanes, tile 1)
        const f32x4 sd = opaque(st.uw[0]) * sp.wo[0] + opaque(st.uw[1]) * sp.wo[1] + opaque(st.uw[2]) * sp.wo[2] +
                         opaque(st.uw[3]) * sp.wo[3];
        const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
        ua = zero;
        ub = cx.hi ? sd : zero;
    } else {
        ua = st.acc[(G + 1) & 1][0][b];
        ub = st.acc[(G + 1) & 1][1][b];
    }
    const f32x4* kc = st.pk[slot];
    f32x4 aa, ab, za, zb;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float ea, eb, ga, gb;
        qf_elem(kc[0][r], kc[1][r], kc[2][r], ua[r], ub[r], cx.w, cx.w2, cx.q, cx.hi, ea, eb, ga, gb);
        aa[r] = ea;
        ab[r] = eb;
        za[r] = ga;
        zb[r] = gb;
    }
    st.b[b & 1][0] = za;
    st.b[b & 1][1] = zb;
    int nt = 0;
    if constexpr (!SEED) w3_stage(st.tq[nt++], aa, cx.tw, cx.tr);  // a_L's value / d/dx_1 streams feed no gradient
    w3_stage(st.tq[nt++], ab, cx.tw, cx.tr);
    w3_stage(st.tq[nt++], za, cx.tw, cx.tr);
    w3_stage(st.tq[nt++], zb, cx.tw, cx.tr);
    if constexpr (SEED) {  // gu_j = Wout_j . a_L,3 (hi lanes' tile-1 a-jet)
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            const f32x4 wj = sp.wo[j];
            st.gup[j] += wj[0] * ab[0] + wj[1] * ab[1] + wj[2] * ab[2] + wj[3] * ab[3];
            asm volatile("" : "+v"(st.gup[j]));  // materialised here, not sunk past the reverse sweep
        }
    }
}

// One slice S = G NB + KB of reverse GEMM G: 8 operand pairs x 16 MFMAs (two column tiles per A operand), the mid-slice
// ring barrier after pair 3 (epilogue S+3's kept reloads issued ahead of the ring refill), epilogue S's tile blocks
// stored after pair QFI_STORE_PAIR's wait, and epilogue block KB+1 as one VALU cluster after pair QFI_EPI_PAIR.
template <int G, int KB, int LH>
__device__ __forceinline__ void qfi_slice(QfiState<LH>& st, const QfiCtx& cx) {
    constexpr int NS = LH * NB;
    constexpr int S = G * NB + KB;
    constexpr int SLOT = (S % W1_NBUF) * SLICE * 4;
    constexpr int NSLOT = ((S + 1) % W1_NBUF) * SLICE * 4;
    constexpr bool EPI = KB + 1 < NB;
    f32x4(&acc0)[NB] = st.acc[G & 1][0];
    f32x4(&acc1)[NB] = st.acc[G & 1][1];
    const f32x4 b0 = st.b[KB & 1][0], b1 = st.b[KB & 1][1];
    QfiSeed sp;
    if constexpr (EPI && G == 0) qfi_seed_issue<KB + 1>(sp, cx.sm_vaddr);
    f32x4 a0 = st.pa0, a1 = st.pa1;
    static_for<0, NB / 2>([&](auto P) {
        constexpr int p = decltype(P)::value;
        if constexpr (p == 4 && S + 1 < NS) {
            // publish slice S+1 (issued at the mid-slice of S-2, after epilogue S+1's reloads) and free the slot of
            // slice S-1 for slice S+3. Younger and allowed outstanding: the tile stores of the last two epilogues
            // issued after that ring slice (S-1 and S with the stores before the mid-slice wait, S-2 and S-1 after
            // it), epilogue S+2's reloads and slice S+2's ring loads (mid-slice of S-1)
            constexpr bool EARLY = QFI_STORE_PAIR < 4;
            constexpr int ALLOW = (EARLY ? qfi_nst<S - 1, LH>() + qfi_nst<S, LH>()
                                         : qfi_nst<S - 2, LH>() + qfi_nst<S - 1, LH>()) +
                                  qfi_nrl<S + 2, LH>() + (S + 2 < NS ? 4 : 0);
            static_assert(ALLOW < 64, "vmcnt is 6 bits");
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(ALLOW) : "memory");
            qfi_reload_landed<S + 1, LH>(st);
            qfi_reload_issue<S + 3, LH>(st, cx);  // two slices ahead of its use
            __builtin_amdgcn_s_barrier();
            if constexpr (S + 3 < NS) {
                const float* spp = cx.stream;
                asm volatile("" : "+s"(spp));  // keep slice addresses from being hoisted into SGPRs
                ring_issue4(spp, cx.ring, S + 3, cx.wave, 16u * cx.lane);
            }
        }
        f32x4 n0, n1;
        constexpr bool NEXT_IN_SLICE = p + 1 < NB / 2;
        constexpr bool NEXT_SLICE = !NEXT_IN_SLICE && S + 1 < NS;
        if constexpr (NEXT_IN_SLICE) {
            n0 = lds_read4<SLOT + (2 * p + 2) * 1024>(cx.ring_vaddr);
            n1 = lds_read4<SLOT + (2 * p + 3) * 1024>(cx.ring_vaddr);
        } else if constexpr (NEXT_SLICE) {
            n0 = lds_read4<NSLOT>(cx.ring_vaddr);
            n1 = lds_read4<NSLOT + 1024>(cx.ring_vaddr);
        }
        if constexpr (NEXT_IN_SLICE || NEXT_SLICE)
            lgkm_wait<2>(a0, a1);
        else
            lgkm_wait<0>(a0, a1);
        if constexpr (p == 0 && EPI && G == 0) {
            // the seed parameters were issued before pair 1's reads: the wait above covered them
#pragma unroll
            for (int j = 0; j < MAXO; ++j) asm volatile("" : "+v"(sp.wo[j]));
        }
        // the tile blocks epilogue S staged (end of the previous slice / before the GEMM): their LDS transpose was
        // retired by pair 0's wait; stored after this pair's wait
        if constexpr (p == QFI_STORE_PAIR) qfi_tile_flush<S, LH>(st, cx);
        if constexpr (p == QFI_EPI_PAIR && EPI) {
            __builtin_amdgcn_sched_barrier(0);
            qfi_epilogue<G, LH>(st, cx, KB + 1, (S + 1) % 3, sp);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            acc0[2 * p] = mfma4(a0[r], b0[r], acc0[2 * p]);
            acc1[2 * p] = mfma4(a0[r], b1[r], acc1[2 * p]);
            acc0[2 * p + 1] = mfma4(a1[r], b0[r], acc0[2 * p + 1]);
            acc1[2 * p + 1] = mfma4(a1[r], b1[r], acc1[2 * p + 1]);
        }
        if constexpr (NEXT_IN_SLICE || NEXT_SLICE) {
            a0 = n0;
            a1 = n1;
        }
    });
    st.pa0 = a0;
    st.pa1 = a1;
    __builtin_amdgcn_sched_barrier(0);
}

template <int G, int LH>
__device__ __forceinline__ void qfi_gemm(QfiState<LH>& st, const QfiCtx& cx) {
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) st.acc[G & 1][0][ob] = st.acc[G & 1][1][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
        // block 0 of the input (its kept reloads, epilogue G NB, were covered by the previous slice's wait)
        QfiSeed sp;
        if constexpr (G == 0) qfi_seed_load(sp, cx, 0);
        qfi_epilogue<G, LH>(st, cx, 0, (G * NB) % 3, sp);
    }
    static_for<0, NB>([&](auto KB) { qfi_slice<G, decltype(KB)::value, LH>(st, cx); });
}

template <int G, int LH>
__device__ __forceinline__ void qfi_run(QfiState<LH>& st, const QfiCtx& cx) {
    if constexpr (G < LH) {
        qfi_gemm<G, LH>(st, cx);
        qfi_run<G + 1, LH>(st, cx);
    }
}

// Arguments and workspace exactly as qf_rev_kernel (launch_qf_rev): grid hess_groups(n) / 4 workgroups of 4 waves,
// 8 coordinates per wave.
template <int LH>
__global__ __launch_bounds__(THREADS, 1) void qfi_rev_kernel(const float* __restrict__ ws, const float* __restrict__ x,
                                                             int64_t n, const float* __restrict__ G,
                                                             const float* __restrict__ tu,
                                                             const float* __restrict__ kept, float* __restrict__ gx,
                                                             float* __restrict__ gu, int d, int o, float w0, float w,
                                                             float* __restrict__ abuf, float* __restrict__ dbuf,
                                                             int64_t n_pad) {
    constexpr int SMALL4 = (small_floats_ct(LH) + 3) / 4 * 4;
    __shared__ __attribute__((aligned(16))) float lds[W1_NBUF * SLICE + SMALL4 + WAVES * STB_SCRATCH];
    QfiCtx cx;
    QfiState<LH> st;
    cx.ring = lds;
    float* sm = lds + W1_NBUF * SLICE;
    cx.sm = sm;
    cx.lane = threadIdx.x & 63;
    cx.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    cx.g = cx.lane >> 4;
    const int c = cx.lane & 15;
    cx.hi = c >= 8;
    cx.w = w;
    cx.w2 = w * w;
    cx.stream = ws + small_pad(LH) + (int64_t)LH * NB * SLICE;  // the transposed (reverse) slices
    const unsigned lds_base = lds_addr(lds);
    cx.ring_vaddr = lds_base + cx.lane * 16;
    cx.sm_vaddr = lds_base + W1_NBUF * SLICE * 4 + 16 * cx.g;
    {
        const unsigned scr = lds_base + 4u * (W1_NBUF * SLICE + SMALL4 + cx.wave * STB_SCRATCH);
        cx.tw = scr + 4u * (4 * cx.g * STB_ROW + c);                      // row 4 g + r (r by the offsets), column c
        cx.tr = scr + 4u * ((cx.lane >> 2) * STB_ROW + 4 * (cx.lane & 3));  // row lane / 4, columns 4 (lane & 3)
    }
    const int64_t ngroups = hess_groups(n);
    const int64_t grp = (int64_t)blockIdx.x * WAVES + cx.wave;
    const int64_t coord = grp * 8 + (c & 7);
    const bool valid = coord < n;
    cx.kb = (const char*)(kept + hess_kept_off(ngroups, LH, 1, grp, 0, 0, 0));
    cx.kl = hess_kept_lstride(ngroups) * 4;
    cx.ta = (const char*)(abuf + 2 * grp * (H * 16));
    cx.td = (const char*)(dbuf + 2 * grp * (H * 16));
    cx.lb = 4 * n_pad * H * 4;
    cx.vl = 16u * cx.lane;
    {
        const float* gq = G + coord * d * d;
        QfCoef& q = cx.q;
        q.q11 = valid ? gq[0] : 0.f;
        q.q12 = (valid && d > 1) ? gq[1] + gq[2] : 0.f;
        q.q22 = (valid && d > 1) ? gq[3] : 0.f;
        q.e1 = cx.hi ? q.q11 : 0.f;
        q.e2 = cx.hi ? q.q22 : q.q12;
        q.ca = cx.hi ? 2.f * q.q11 : q.q12;
        q.cb = cx.hi ? q.q12 : 2.f * q.q22;
        q.mlo = cx.hi ? 0.f : 1.f;
    }
#pragma unroll
    for (int j = 0; j < MAXO; ++j) {
        st.uw[j] = (valid && j < o) ? (tu != nullptr ? tu[coord * o + j] : 1.f) : 0.f;
        st.gup[j] = 0.f;
    }
    {
        const int nf4 = (small_floats(LH) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    __syncthreads();
    // prologue, in the order the mid-slice counts assume: epilogues 0 and 1's reloads, ring slices 0 and 1, epilogue
    // 2's reloads, ring slice 2; then slice 0 and epilogue 0 / 1's reloads landed (all but the last 11 ops)
    qfi_reload_issue<0, LH>(st, cx);
    qfi_reload_issue<1, LH>(st, cx);
    ring_issue4(cx.stream, cx.ring, 0, cx.wave, 16u * cx.lane);
    ring_issue4(cx.stream, cx.ring, 1, cx.wave, 16u * cx.lane);
    qfi_reload_issue<2, LH>(st, cx);
    ring_issue4(cx.stream, cx.ring, 2, cx.wave, 16u * cx.lane);
    asm volatile("s_waitcnt vmcnt(11)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    qfi_reload_landed<0, LH>(st);
    st.pa0 = lds_read4<0>(cx.ring_vaddr);
    st.pa1 = lds_read4<1024>(cx.ring_vaddr);

    qfi_run<0, LH>(st, cx);

    // gu_j = D2 y_j[Q] (the seed epilogues accumulated this lane's neurons)
    if (gu != nullptr) {
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            const float pj = sum_groups(st.gup[j]);
            if (j < o && valid && cx.g == 0 && cx.hi) gu[coord * o + j] = pj;
        }
    }
    // ---- layer 0 (serial): the jet rebuilt from x, the last GEMM's output -> a_0 / zb_0 tiles, gx = W0^T zb_0,value --
    {
        constexpr int GL = (LH - 1) & 1;
        const float x0 = valid ? x[coord * d] : 0.f;
        const float x1 = (valid && d > 1) ? x[coord * d + 1] : 0.f;
        const float wl = w0, wl2 = w0 * w0;
        float qk[2] = {0.f, 0.f};
        // tile blocks as four dword stores each (store_block): no LDS transpose, so no LDS wait between the blocks
        float* pa0 = (float*)cx.ta + 4 * cx.g * 16 + c;
        float* pd0 = (float*)cx.td + 4 * cx.g * 16 + c;
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            const int nb = 16 * rb + 4 * cx.g;
            const f32x4 wa = *(const f32x4*)(sm + SM_W0 + nb);
            const f32x4 wb = *(const f32x4*)(sm + SM_W0 + H + nb);  // zero padded row when d == 1
            const f32x4 zv = layer0_z(*(const f32x4*)(sm + SM_BIAS + nb), wa, wb, x0, x1);
            const f32x4 ua = st.acc[GL][0][rb], ub = st.acc[GL][1][rb];
            f32x4 aa, ab, za, zb;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float ea, eb, ga, gb;
                qf_elem0(zv[r], wa[r], wb[r], ua[r], ub[r], wl, wl2, cx.q, cx.hi, ea, eb, ga, gb);
                aa[r] = ea;
                ab[r] = eb;
                za[r] = ga;
                zb[r] = gb;
            }
            store_block(pa0, rb, aa);
            store_block(pa0 + H * 16, rb, ab);
            store_block(pd0, rb, za);
            store_block(pd0 + H * 16, rb, zb);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * cx.g);  // zero row when d == 1
                qk[k] += wk[0] * za[0] + wk[1] * za[1] + wk[2] * za[2] + wk[3] * za[3];
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (k < d) {
                const float s = sum_groups(qk[k]);
                if (valid && cx.g == 0 && !cx.hi) gx[coord * d + k] = s;
            }
        }
    }
}

}  // namespace siren

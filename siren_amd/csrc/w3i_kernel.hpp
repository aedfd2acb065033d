// w3i_kernel.hpp — the second-order adjoint (work unit W3, w3_kernel.hpp) with every epilogue interleaved into the
// NEXT GEMM's MFMA stream, the way w1_kernel.hpp does it for W1.
//
// Same math, weight stream (the unscaled pack), spill buffer, tile stores and outputs as w3_kernel — the results are
// bitwise those of w3_kernel (tests/test_gpu_w3i.py); see w3_kernel.hpp for the derivation. What changes is the
// schedule:
//   * The L forward and L reverse GEMMs are fully unrolled (G = 0 .. 2L-1). GEMM G accumulates the primal and the
//     tangent column tiles into acc[G & 1] (two MFMAs per A operand read; KEPT forward GEMMs run the tangent only),
//     while the epilogue that turns GEMM G-1's output into GEMM G's B operands runs one 16-neuron block ahead: in slice
//     kb the wave builds block kb+1, so the sincos VALU, the spill / tile stores and the reverse sweep's spill reloads
//     sit between the MFMAs instead of in a store burst between two GEMMs (w3_kernel spends 28-34 % of a tile there,
//     every CU in the same phase, profiles/r02_w3_phases.log).
//   * Epilogue kinds, named by the GEMM whose input they produce:
//       G = 0        FIRST: layer 0 on VALU from x, v (K = d_in)
//       0 < G < L    FWD  : layer G (sin / cos of the primal, tangent a-dot)
//       G = L        SEED : layer L's forward epilogue fused with the reverse seed (layer L is never spilled), and
//                           the ydot partials
//       G > L        REV  : adjoints of layer 2L - G from reverse GEMM G-1, with (cos, zdot, a) reloaded
//     then, after the last GEMM, the layer-0 adjoint and gx (serial).
//   * The forward spills (z, zdot) per layer — not (cos, zdot, a): the reverse recomputes sin / cos of w z, bitwise
//     what the forward computed, instead of reloading two of three blocks (a KEPT launch reloads the stored
//     forward's cos and a, as w3_kernel).
//   * The inputs a REV epilogue (or a KEPT FWD / SEED one) reloads are issued by saddr-form asm loads at the mid-slice
//     barrier two slices before the slice that uses them, ahead of the ring refill; the mid-slice s_waitcnt vmcnt(N)
//     counts every vector-memory op issued after the ring slice it publishes (stores, reloads, the next slices), so
//     nothing younger is waited for.
//   * THETA tile blocks go out as one coalesced 1 KiB store each, transposed through LDS (w3_stage).
//   * 4-slot LDS ring with one mid-slice barrier per slice, the next slice's first operand pair read during the last
//     pair, counted lgkmcnt waits: w1_kernel's slice machinery (ring_issue4, lds_read4, lgkm_wait).
#pragma once
#include "w1_kernel.hpp"
// The epilogue block runs as one VALU cluster after operand pair W3I_EPI_PAIR (>= 4: after the mid-slice wait its
// reloads land at; A/B pairs 4 / 5 / 6 / 7 / slice end interleaved by hipcc: pair 5 -1.4 % on w3_theta, pair 7 the
// same there and -1.4 % more on the sdf step, profiles/r03x_epilogue_placement.log; cf. w1_kernel.hpp w1_epi_pair)
#ifndef W3I_EPI_PAIR
#define W3I_EPI_PAIR 7
#endif
static_assert(W3I_EPI_PAIR >= 4 && W3I_EPI_PAIR < siren::NB / 2, "the REV reloads land at the mid-slice wait (pair 4)");

namespace siren {

enum { W3E_FIRST = 0, W3E_FWD = 1, W3E_SEED = 2, W3E_REV = 3 };

template <int G, int LH>
constexpr int w3_epi_kind() {
    return G == 0 ? W3E_FIRST : (G < LH ? W3E_FWD : (G == LH ? W3E_SEED : W3E_REV));
}
// column tiles of GEMM G: the KEPT forward GEMMs run the tangent only (the primal comes from the stored forward)
template <int G, int LH, bool KEPT>
constexpr int w3_streams() {
    return (KEPT && G < LH) ? 1 : 2;
}
// LDS parameter reads an epilogue block needs: FIRST W0T[0..3] + b0; FWD b_G; SEED b_L + WoT[0..3] + seed
template <int KIND>
constexpr int w3_nparams() {
    return KIND == W3E_FIRST ? 5 : (KIND == W3E_FWD ? 1 : (KIND == W3E_SEED ? 6 : 0));
}
template <int KIND, int G, int LH>
constexpr int w3_param_off(int i, int b) {
    return 4 * (16 * b) + 4 * (KIND == W3E_FIRST ? (i < 4 ? SM_W0 + i * H : SM_BIAS)
                               : KIND == W3E_FWD ? SM_BIAS + G * H
                                                 : (i == 0 ? SM_BIAS + LH * H : (i < 5 ? SM_WO + (i - 1) * H : SM_SEED)));
}
// reloaded inputs of an epilogue: (cos, zdot, a) for REV; cos for a KEPT FWD; (cos, a) for a KEPT SEED
template <int KIND, bool KEPT>
constexpr bool w3_reloads() {
    return KIND == W3E_REV || (KEPT && (KIND == W3E_FWD || KIND == W3E_SEED));
}

// vector-memory stores an epilogue issues (all saddr-form asm, issued after the ring refill of its slice's mid-slice
// barrier): the next mid-slice wait leaves them outstanding instead of waiting for them (s_waitcnt counts stores too)
template <int KIND, bool THETA, bool KEPT>
constexpr int w3_nstores() {
    return KIND == W3E_FIRST ? (KEPT ? 1 : 2) + (THETA ? (KEPT ? 1 : 2) : 0)
         : KIND == W3E_FWD   ? (KEPT ? 1 + (THETA ? 1 : 0) : 2 + (THETA ? 2 : 0))
         : KIND == W3E_SEED  ? (THETA ? (KEPT ? 3 : 4) : 0)
                             : (THETA ? 2 : 0);
}

// vector-memory loads of an epilogue's reloads (w3_reload_issue): REV reloads (z, zdot) — or (cos, zdot, a) from the
// stored forward when KEPT, a being 4 dword loads from the tile layout —, a KEPT FWD cos, a KEPT SEED (cos, a)
template <int KIND, bool KEPT>
constexpr int w3_nreloads() {
    return KIND == W3E_REV ? (KEPT ? 6 : 2)
         : (KEPT && KIND == W3E_FWD) ? 1 : ((KEPT && KIND == W3E_SEED) ? 5 : 0);
}
template <int E, int LH, bool THETA, bool KEPT>
constexpr int w3_nvmem_st() {  // stores of epilogue E (0 past either end)
    return (E < 0 || E >= 2 * LH * NB) ? 0 : w3_nstores<w3_epi_kind<E / NB, LH>(), THETA, KEPT>();
}
template <int E, int LH, bool KEPT>
constexpr int w3_nvmem_rl() {
    return (E < 0 || E >= 2 * LH * NB) ? 0 : w3_nreloads<w3_epi_kind<E / NB, LH>(), KEPT>();
}

template <int LH>
struct W3iState {
    f32x4 ap[NB], at[NB];              // B operands (primal, tangent) of the current GEMM, built one block ahead
    f32x4 accp[2][NB], acct[2][NB];    // ping-pong accumulators
    f32x4 pa0, pa1;                    // the next slice's first operand pair (in flight)
    f32x4 pc[3], pz[3], ps[3];         // reloads of epilogue E in slot E % 3: (z, zdot) or, KEPT, (cos, zdot, a)
    f32x4 tq[4];                       // THETA: the last epilogue's tile blocks, transposed (stored next slice)
    float xv[MAXD], vv[MAXD], gyv[MAXO], uv[MAXO], ydp[MAXO];
};

struct W3iCtx {
    const float* stream;
    float* ring;
    const float* sm;
    int wave, lane, g;
    float w0, w, useed;        // useed = 1 when u == NULL (the all-ones output weighting: adb_L = seed)
    unsigned ring_vaddr, sm_vaddr;
    const char* wsp;           // this wave's spill area (wave-uniform)
    const char* kc;            // KEPT: this wave's lane-major cos base (wave-uniform)
    const char* sa;            // reverse source of a_l in the wgrad tile layout (A or kA) at the wave's tile (uniform)
    const char* tA;            // THETA tile bases of the wave's tile (wave-uniform): layer l at + l * lbytes
    const char* tAt;
    const char* tD;
    const char* tDt;
    int64_t lstride, lbytes;   // floats / bytes between the layers of a tile buffer
    unsigned vl, vt;           // this lane's byte offset: 16 lane (lane-major blocks), 4 (4 g 16 + c) (tile layout)
    unsigned tw, tr;           // LDS transpose scratch of the wave: this lane's write / read address
};

// a_l block from the wgrad tile layout (kept_a: 4 dwords 64 B apart at the lane's (4 g 16 + c) offset)
__device__ __forceinline__ void w3_load_tile(f32x4& r, const char* base, unsigned voff) {
    asm volatile(
        "global_load_dword %0, %4, %5\n\t"
        "global_load_dword %1, %4, %5 offset:64\n\t"
        "global_load_dword %2, %4, %5 offset:128\n\t"
        "global_load_dword %3, %4, %5 offset:192"
        : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
        : "v"(voff), "s"(base));
}
// spill slot (layer l, quantity q in {c, zd, a}, block b): 1 KiB per block, lane-contiguous (w3_kernel spill_at)
__device__ __forceinline__ int64_t w3_spill_off(int l, int q, int b) { return ((int64_t)(l * 3 + q) * NB + b) * 1024; }

// issue the reloads of epilogue E (block b of GEMM G's input)
template <int E, int LH, bool THETA, bool KEPT>
__device__ __forceinline__ void w3_reload_issue(W3iState<LH>& st, const W3iCtx& cx) {
    constexpr int G = E / NB, B = E % NB;
    constexpr int KIND = w3_epi_kind<G, LH>();
    if constexpr (G < 2 * LH && w3_reloads<KIND, KEPT>()) {
        constexpr int M = KIND == W3E_REV ? 2 * LH - G : G;  // the layer whose forward values are reloaded
        if constexpr (KEPT)
            w3_load16(st.pc[E % 3], w3_at(cx.kc, (int64_t)(M * NB + B) * 1024), cx.vl);
        else
            w3_load16(st.pc[E % 3], w3_at(cx.wsp, w3_spill_off(M, 0, B)), cx.vl);  // z
        if constexpr (KIND == W3E_REV) w3_load16(st.pz[E % 3], w3_at(cx.wsp, w3_spill_off(M, 1, B)), cx.vl);
        if constexpr (KEPT && (KIND == W3E_REV || KIND == W3E_SEED))
            w3_load_tile(st.ps[E % 3], w3_at(cx.sa, M * cx.lbytes + B * 1024), cx.vt);
    }
}
// epilogue E's reloads have landed (the caller's vmcnt wait covered them): redefine them after the wait
template <int E, int LH, bool KEPT>
__device__ __forceinline__ void w3_reload_landed(W3iState<LH>& st) {
    constexpr int G = E / NB;
    constexpr int KIND = w3_epi_kind<G, LH>();
    if constexpr (G < 2 * LH && w3_reloads<KIND, KEPT>()) {
        asm volatile("" : "+v"(st.pc[E % 3]));
        if constexpr (KIND == W3E_REV) asm volatile("" : "+v"(st.pz[E % 3]));
        if constexpr (KEPT && (KIND == W3E_REV || KIND == W3E_SEED)) asm volatile("" : "+v"(st.ps[E % 3]));
    }
}

// THETA: the tile blocks epilogue E staged (w3i_epilogue), in its staging order: A (primal a_l, unless KEPT), At
// (tangent a-dot), then for SEED / REV the adjoints D, Dt
template <int KIND, bool KEPT>
constexpr int w3_ntiles() {
    return KIND == W3E_SEED ? (KEPT ? 3 : 4) : (KIND == W3E_REV ? 2 : (KEPT ? 1 : 2));
}
template <int E, int LH, bool THETA, bool KEPT>
__device__ __forceinline__ void w3_tile_flush(W3iState<LH>& st, const W3iCtx& cx) {
    constexpr int G = E / NB, B = E % NB;
    constexpr int KIND = w3_epi_kind<G, LH>();
    if constexpr (THETA && G < 2 * LH) {
        constexpr int NT = w3_ntiles<KIND, KEPT>();
#pragma unroll
        for (int i = 0; i < NT; ++i) asm volatile("" : "+v"(st.tq[i]));  // landed
        constexpr int L = KIND == W3E_REV ? 2 * LH - G : (KIND == W3E_SEED ? LH : G);  // FIRST: G = 0
        auto put = [&](int k, const char* base) { w3_store16(w3_at(base, L * cx.lbytes + B * 1024), cx.vl, st.tq[k]); };
        if constexpr (KIND == W3E_REV) {
            put(0, cx.tD);
            put(1, cx.tDt);
        } else {
            constexpr int A0 = KEPT ? 0 : 1;
            if constexpr (!KEPT) put(0, cx.tA);
            put(A0, cx.tAt);
            if constexpr (KIND == W3E_SEED) {
                put(A0 + 1, cx.tD);
                put(A0 + 2, cx.tDt);
            }
        }
    }
}

template <int KIND, int G, int LH>
struct W3iParams {
    f32x4 v[w3_nparams<KIND>() > 0 ? w3_nparams<KIND>() : 1];
};
template <int KIND, int G, int LH, int B>
__device__ __forceinline__ void w3_param_issue(W3iParams<KIND, G, LH>& ep, unsigned sm_vaddr) {
    static_for<0, w3_nparams<KIND>()>([&](auto I) {
        ep.v[decltype(I)::value] = lds_read4<w3_param_off<KIND, G, LH>(decltype(I)::value, B)>(sm_vaddr);
    });
}
template <int KIND, int G, int LH>
__device__ __forceinline__ void w3_param_load(W3iParams<KIND, G, LH>& ep, const W3iCtx& cx, int b) {
#pragma unroll
    for (int i = 0; i < w3_nparams<KIND>(); ++i)
        ep.v[i] = *(const f32x4*)((const char*)cx.sm + w3_param_off<KIND, G, LH>(i, b) + 16 * cx.g);
}

__device__ __forceinline__ void w3_sincos4(const f32x4& t, f32x4& sn, f32x4& cs) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float a_, c_;
        sincos_fast(t[r], a_, c_);
        sn[r] = a_;
        cs[r] = c_;
    }
}

// The epilogue that builds block b of GEMM G's B operands (the table at the top); E = G NB + b its reload slot.
template <int G, int LH, bool THETA, bool KEPT>
__device__ __forceinline__ void w3i_epilogue(W3iState<LH>& st, const W3iCtx& cx, int b,
                                             const W3iParams<w3_epi_kind<G, LH>(), G, LH>& ep, int slot) {
    constexpr int KIND = w3_epi_kind<G, LH>();
    const f32x4* accp = st.accp[(G + 1) & 1];
    const f32x4* acct = st.acct[(G + 1) & 1];
    auto spill = [&](int l, int q, const f32x4& val) { w3_store16(w3_at(cx.wsp, w3_spill_off(l, q, b)), cx.vl, val); };
    int nt = 0;  // tile blocks staged so far (w3_tile_flush stores them in this order)
    auto tile = [&](const f32x4& val) {
        w3_stage(st.tq[nt], val, cx.tw, cx.tr);
        ++nt;
    };
    if constexpr (KIND == W3E_FIRST) {
        // z0 = W0 x + b0, zd0 = W0 v (rows k >= d_in of W0T are zero, as are x_k / v_k there)
        f32x4 zx = st.xv[0] * ep.v[0];
        f32x4 zd = fma4(st.vv[0], ep.v[0], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int k = 1; k < MAXD; ++k) {  // fma(0, 0, z) = z: the rows past d_in change nothing
            zx = fma4(st.xv[k], ep.v[k], zx);
            zd = fma4(st.vv[k], ep.v[k], zd);
        }
        const f32x4 z = zx + ep.v[4];
        f32x4 sn, cs;
        w3_sincos4(opaque(cx.w0) * z, sn, cs);
        st.ap[b] = sn;
        st.at[b] = (opaque(cx.w0) * cs) * zd;
        spill(0, 1, zd);
        if constexpr (!KEPT) spill(0, 0, z);  // the reverse recomputes sin / cos of w0 z (bitwise the same)
        if constexpr (THETA) {
            if constexpr (!KEPT) tile(sn);
            tile(st.at[b]);
        }
    } else if constexpr (KIND == W3E_FWD) {
        const f32x4 zd = acct[b];
        if constexpr (KEPT) {
            st.at[b] = (opaque(cx.w) * st.pc[slot]) * zd;
        } else {
            const f32x4 z = accp[b] + ep.v[0];
            f32x4 sn, cs;
            w3_sincos4(opaque(cx.w) * z, sn, cs);
            st.ap[b] = sn;
            st.at[b] = (opaque(cx.w) * cs) * zd;
            spill(G, 0, z);
            if constexpr (THETA) tile(sn);
        }
        spill(G, 1, zd);
        if constexpr (THETA) tile(st.at[b]);
    } else if constexpr (KIND == W3E_SEED) {
        // layer L's forward epilogue, then the seed adb_L = Wout^T u (u = ones: the seed row), ab_L = Wout^T gy
        const f32x4 zd = acct[b];
        f32x4 sn, cs;
        if constexpr (KEPT) {
            cs = st.pc[slot];
            sn = st.ps[slot];
        } else {
            const f32x4 z = accp[b] + ep.v[0];
            w3_sincos4(opaque(cx.w) * z, sn, cs);
        }
        const f32x4 atl = (opaque(cx.w) * cs) * zd;
        if constexpr (THETA) {
            if constexpr (!KEPT) tile(sn);
            tile(atl);
        }
        f32x4 adb = opaque(cx.useed) * ep.v[5];
        f32x4 abseed = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            const f32x4 wj = ep.v[1 + j];  // zero rows for j >= d_out
            st.ydp[j] += wj[0] * atl[0] + wj[1] * atl[1] + wj[2] * atl[2] + wj[3] * atl[3];
            // materialised here: hipcc would sink the sum into the ydot branch after the last GEMM and keep every
            // block's a-dot and Wout rows alive across the reverse sweep
            asm volatile("" : "+v"(st.ydp[j]));
            abseed = abseed + st.gyv[j] * wj;
            adb = adb + st.uv[j] * wj;
        }
        st.at[b] = (opaque(cx.w) * cs) * adb;
        st.ap[b] = (opaque(cx.w) * cs) * abseed - (opaque(cx.w) * opaque(cx.w)) * sn * zd * adb;
        if constexpr (THETA) {
            tile(st.ap[b]);
            tile(st.at[b]);
        }
    } else {
        constexpr int M = 2 * LH - G;  // 1 <= M < L
        f32x4 sn, cs;
        if constexpr (KEPT) {
            cs = st.pc[slot];
            sn = st.ps[slot];
        } else {
            w3_sincos4(opaque(cx.w) * st.pc[slot], sn, cs);
        }
        const f32x4 wc = opaque(cx.w) * cs;
        st.at[b] = wc * acct[b];
        st.ap[b] = wc * accp[b] - (opaque(cx.w) * opaque(cx.w)) * sn * st.pz[slot] * acct[b];
        if constexpr (THETA) {
            tile(st.ap[b]);
            tile(st.at[b]);
        }
    }
}

// One slice s = 16 G + KB: 8 operand pairs x (8 or 16) MFMAs, the mid-slice ring barrier after pair 3 (with the
// reloads of epilogue s + 2 issued ahead of the ring refill), and epilogue block KB+1 of GEMM G's input in the shadow.
template <int G, int KB, int LH, bool THETA, bool KEPT>
__device__ __forceinline__ void w3i_slice(W3iState<LH>& st, const W3iCtx& cx) {
    constexpr int NS = 2 * LH * NB;
    constexpr int S = G * NB + KB;
    constexpr int SLOT = (S % W1_NBUF) * SLICE * 4;
    constexpr int NSLOT = ((S + 1) % W1_NBUF) * SLICE * 4;
    constexpr int KIND = w3_epi_kind<G, LH>();
    constexpr bool EPI = KB + 1 < NB;
    constexpr bool TWO = w3_streams<G, LH, KEPT>() == 2;
    f32x4(&accp)[NB] = st.accp[G & 1];
    f32x4(&acct)[NB] = st.acct[G & 1];
    const f32x4 bp = st.ap[KB], bt = st.at[KB];
    W3iParams<KIND, G, LH> ep;
    if constexpr (EPI && w3_nparams<KIND>() > 0) w3_param_issue<KIND, G, LH, KB + 1>(ep, cx.sm_vaddr);
    f32x4 a0 = st.pa0, a1 = st.pa1;
    static_for<0, NB / 2>([&](auto P) {
        constexpr int p = decltype(P)::value;
        if constexpr (p == 4 && S + 1 < NS) {
            // publish slice S+1 and free the slot of slice S-1 for slice S+3; epilogue S+1's reloads (issued one
            // slice ago, before slice S+2's ring loads) have landed; issue epilogue S+2's ahead of the refill
            // slice S+1 (issued at the mid-slice of S-2, after epilogue S+1's reloads) must have landed; younger and
            // allowed outstanding: epilogue S-1's stores, epilogue S+2's reloads and slice S+2's ring loads (both
            // issued at the mid-slice of S-1), epilogue S's stores
            constexpr int ALLOW = w3_nvmem_st<S - 1, LH, THETA, KEPT>() + w3_nvmem_rl<S + 2, LH, KEPT>() +
                                  (S + 2 < NS ? 4 : 0) + w3_nvmem_st<S, LH, THETA, KEPT>();
            static_assert(ALLOW < 64, "vmcnt is 6 bits");
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(ALLOW) : "memory");
            w3_reload_landed<S + 1, LH, KEPT>(st);
            w3_reload_issue<S + 3, LH, THETA, KEPT>(st, cx);  // two slices ahead of its use
            __builtin_amdgcn_s_barrier();
            if constexpr (S + 3 < NS) {
                const float* sp = cx.stream;
                asm volatile("" : "+s"(sp));  // keep slice addresses from being hoisted into SGPRs
                ring_issue4(sp, cx.ring, S + 3, cx.wave, 16u * cx.lane);
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
        if constexpr (p == 0 && EPI) {
            // the epilogue parameters were issued before pair 1's reads: the wait above covered them
#pragma unroll
            for (int i = 0; i < w3_nparams<KIND>(); ++i) asm volatile("" : "+v"(ep.v[i]));
        }
        // the tile blocks epilogue S staged at the end of the previous slice: retired by the same wait
        if constexpr (p == 0) w3_tile_flush<S, LH, THETA, KEPT>(st, cx);
        if constexpr (p == W3I_EPI_PAIR && EPI) {  // the epilogue block as one VALU cluster after this pair's wait
            __builtin_amdgcn_sched_barrier(0);
            w3i_epilogue<G, LH, THETA, KEPT>(st, cx, KB + 1, ep, (S + 1) % 3);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if constexpr (TWO) {
                accp[2 * p] = mfma4(a0[r], bp[r], accp[2 * p]);
                acct[2 * p] = mfma4(a0[r], bt[r], acct[2 * p]);
                accp[2 * p + 1] = mfma4(a1[r], bp[r], accp[2 * p + 1]);
                acct[2 * p + 1] = mfma4(a1[r], bt[r], acct[2 * p + 1]);
            } else {
                acct[2 * p] = mfma4(a0[r], bt[r], acct[2 * p]);
                acct[2 * p + 1] = mfma4(a1[r], bt[r], acct[2 * p + 1]);
            }
        }
        if constexpr (NEXT_IN_SLICE || NEXT_SLICE) {
            a0 = n0;
            a1 = n1;
        }
    });
    st.pa0 = a0;
    st.pa1 = a1;

    // one scheduling region per slice: the epilogue interleaves with this slice's MFMAs, but hipcc may not hoist later
    // blocks' epilogue arithmetic (whose inputs are all ready when the GEMM starts) into it
    __builtin_amdgcn_sched_barrier(0);
}

template <int G, int LH, bool THETA, bool KEPT>
__device__ __forceinline__ void w3i_gemm(W3iState<LH>& st, const W3iCtx& cx) {
    constexpr int KIND = w3_epi_kind<G, LH>();
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) {
        st.accp[G & 1][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
        st.acct[G & 1][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    {
        // block 0 of the input (its reloads, epilogue G NB, were covered by the previous slice's wait)
        W3iParams<KIND, G, LH> ep;
        w3_param_load<KIND, G, LH>(ep, cx, 0);
        w3i_epilogue<G, LH, THETA, KEPT>(st, cx, 0, ep, (G * NB) % 3);
    }
    static_for<0, NB>([&](auto KB) { w3i_slice<G, decltype(KB)::value, LH, THETA, KEPT>(st, cx); });
}

template <int G, int LH, bool THETA, bool KEPT>
__device__ __forceinline__ void w3i_run(W3iState<LH>& st, const W3iCtx& cx) {
    if constexpr (G < 2 * LH) {
        w3i_gemm<G, LH, THETA, KEPT>(st, cx);
        w3i_run<G + 1, LH, THETA, KEPT>(st, cx);
    }
}

// Arguments and workspace exactly as w3_kernel (launch_w3); one 64-coordinate tile per workgroup.
template <int LH, bool THETA, bool KEPT>
__global__ __launch_bounds__(THREADS, 1) void w3i_kernel(const float* __restrict__ ws, const float* __restrict__ x,
                                                         const float* __restrict__ v, const float* __restrict__ gy,
                                                         const float* __restrict__ u, float* __restrict__ ydot, int o,
                                                         int64_t n, float* __restrict__ gx, float* __restrict__ spill,
                                                         float* __restrict__ A, float* __restrict__ At,
                                                         float* __restrict__ D, float* __restrict__ Dt, int64_t n_pad,
                                                         int d, float w0, float w, const float* __restrict__ kA,
                                                         const float* __restrict__ kC, int64_t ws_bs = 0,
                                                         int64_t spill_bs = 0, int64_t buf_bs = 0) {
    constexpr int NS = 2 * LH * NB;
    constexpr int SMALL4 = (small_floats_ct(LH) + 3) / 4 * 4;
    __shared__ __attribute__((aligned(16))) float lds[W1_NBUF * SLICE + SMALL4 + WAVES * STB_SCRATCH];
    W3iCtx cx;
    W3iState<LH> st;
    cx.ring = lds;
    float* sm = lds + W1_NBUF * SLICE;
    cx.sm = sm;
    cx.lane = threadIdx.x & 63;
    cx.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    cx.g = cx.lane >> 4;
    const int c = cx.lane & 15;
    int64_t bx = blockIdx.x;
    if (ws_bs != 0) {  // grouped launch over batched weights (siren_second_order_batched), renumbered XCD-major
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
    cx.stream = ws + small_pad(LH);
    cx.w0 = w0;
    cx.w = w;
    cx.useed = u == nullptr ? 1.f : 0.f;
    cx.lstride = n_pad * H;
    const unsigned lds_base = lds_addr(lds);
    cx.ring_vaddr = lds_base + cx.lane * 16;
    cx.sm_vaddr = lds_base + W1_NBUF * SLICE * 4 + 16 * cx.g;
    const int64_t tile = bx * WAVES + cx.wave;
    cx.wsp = (const char*)(spill + tile * (int64_t)(LH + 1) * 3 * NB * 256);
    cx.kc = KEPT ? (const char*)(kC + cos_off(bx, cx.wave, LH, 0, 0, 0)) : nullptr;
    const int64_t tbase = tile * (H * 16);
    cx.sa = (const char*)((KEPT ? kA : A) + tbase);
    cx.tA = (const char*)(A + tbase);
    cx.tAt = (const char*)(At + tbase);
    cx.tD = (const char*)(D + tbase);
    cx.tDt = (const char*)(Dt + tbase);
    cx.lbytes = cx.lstride * 4;
    cx.vl = 16u * cx.lane;
    cx.vt = 4u * (4 * cx.g * 16 + c);
    {
        const unsigned scr = lds_base + 4u * (W1_NBUF * SLICE + SMALL4 + cx.wave * STB_SCRATCH);
        cx.tw = scr + 4u * (4 * cx.g * STB_ROW + c);                      // row 4 g + r (r by the offsets), column c
        cx.tr = scr + 4u * ((cx.lane >> 2) * STB_ROW + 4 * (cx.lane & 3));  // row lane / 4, columns 4 (lane & 3)
    }
    {
        const int nf4 = (small_floats(LH) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t coord = bx * TILE + cx.wave * 16 + c;
    const bool valid = coord < n;
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        st.xv[k] = (valid && k < d) ? x[coord * d + k] : 0.f;
        st.vv[k] = (valid && k < d) ? v[coord * d + k] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < MAXO; ++j) {
        st.gyv[j] = (gy != nullptr && valid && j < o) ? gy[coord * o + j] : 0.f;
        st.uv[j] = (u != nullptr && valid && j < o) ? u[coord * o + j] : 0.f;
        st.ydp[j] = 0.f;
    }
    __syncthreads();
    // ring prologue: slices 0..2 in flight, slice 0 published, its first operand pair read
    ring_issue4(cx.stream, cx.ring, 0, cx.wave, 16u * cx.lane);
    ring_issue4(cx.stream, cx.ring, 1, cx.wave, 16u * cx.lane);
    ring_issue4(cx.stream, cx.ring, 2, cx.wave, 16u * cx.lane);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    st.pa0 = lds_read4<0>(cx.ring_vaddr);
    st.pa1 = lds_read4<1024>(cx.ring_vaddr);

    w3i_run<0, LH, THETA, KEPT>(st, cx);

    // ydot = Wout ad_L (the SEED epilogue accumulated this lane's neurons)
    if (ydot != nullptr) {
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            if (j < o) {
                const float p = sum_groups(st.ydp[j]);
                if (valid && cx.g == 0) ydot[coord * o + j] = p;
            }
        }
    }
    // layer-0 adjoints from the last reverse GEMM (serial), then gx = W0^T zb_0
    {
        constexpr int GL = (2 * LH - 1) & 1;
        const char* sa0 = cx.sa;
        // The blocks' spill / kept loads run PD blocks ahead of their use (issued before the previous blocks'
        // stores, which pin the order): loaded at the use, each block waited for its own loads behind the stores of
        // the block before, one memory latency per block of every tile's serial tail (round 6)
        constexpr int PD = 4;
        f32x4 tz[NB], tc[NB], ts[NB];
        auto tail_load = [&](int rb) {
            tz[rb] = *(const f32x4*)(cx.wsp + w3_spill_off(0, 1, rb) + 16 * cx.lane);
            if constexpr (KEPT) {
                tc[rb] = *(const f32x4*)(cx.kc + rb * 1024 + 16 * cx.lane);
                const float* p = (const float*)sa0 + rb * 256 + 4 * cx.g * 16 + c;
                ts[rb] = f32x4{p[0], p[16], p[32], p[48]};
            } else {
                tc[rb] = *(const f32x4*)(cx.wsp + w3_spill_off(0, 0, rb) + 16 * cx.lane);  // z_0 (sin / cos at use)
            }
        };
#pragma unroll
        for (int rb = 0; rb < PD; ++rb) tail_load(rb);
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            if (rb + PD < NB) tail_load(rb + PD);
            const f32x4 zd = tz[rb];
            f32x4 sn, cs;
            if constexpr (KEPT) {
                cs = tc[rb];
                sn = ts[rb];
            } else {
                w3_sincos4(w0 * tc[rb], sn, cs);
            }
            const f32x4 wc = w0 * cs;
            const f32x4 adb = st.acct[GL][rb];
            st.at[rb] = wc * adb;
            st.ap[rb] = wc * st.accp[GL][rb] - (w0 * w0) * sn * zd * adb;
            if constexpr (THETA) {
                w3_stage_store(w3_at(cx.tD, rb * 1024), st.ap[rb], cx.tw, cx.tr, cx.vl);
                w3_stage_store(w3_at(cx.tDt, rb * 1024), st.at[rb], cx.tw, cx.tr, cx.vl);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (k < d) {
            float p = 0.f;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * cx.g);
                p += wk[0] * st.ap[rb][0] + wk[1] * st.ap[rb][1] + wk[2] * st.ap[rb][2] + wk[3] * st.ap[rb][3];
            }
            p = sum_groups(p);
            if (valid && cx.g == 0) gx[coord * d + k] = p;
        }
    }
}

}  // namespace siren

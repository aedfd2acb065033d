#pragma once
// widei_kernel.hpp — the hidden-512 stored-forward training split (MODE_FWDS / MODE_REV of wide_kernel.hpp; BASELINE
// config 4, SingleBVPNet(hidden_features=512) under image_mse) with every epilogue interleaved into the NEXT GEMM's MFMA
// stream, the schedule of w1_kernel.hpp / qfi_kernel.hpp at hidden 512.
//
// wide_kernel runs each layer's epilogue between two GEMMs: per wave and layer 32 KiB of a_l tile and 32 KiB of
// lane-major cos(w z_l) (FWDS) or 32 KiB of delta tile (REV) leave in one burst while the matrix pipe idles, and with
// every CU in the same phase the GPU writes at the HBM roofline during the burst and not at all during the GEMM
// (FWDS: 17 GB per 2^20-coordinate launch; 0.71 MFMA busy). Here:
//   * The L GEMMs of the pass (forward W_1..W_L; reverse W_L^T..W_1^T) are fully unrolled. GEMM G accumulates into
//     acc[G & 1] (32 blocks, AGPRs); the epilogue that turns GEMM G-1's output into GEMM G's B operand runs one
//     16-neuron block ahead: inside slice kb for block kb + 1, as one VALU cluster after the last operand pair. B
//     operands are built just in time (a two-block register ring), so the two accumulator sets fit at one wave per
//     SIMD next to everything else.
//   * Epilogue kinds: FWDS G = 0 FIRST (layer 0 from x, K = d_in on VALU), G > 0 SINCOS (a_G = sin(w z_G), cos(w z_G)
//     to the scratch); REV G = 0 SEED (delta_L = (gy Wout) . cos(w z_L) . w from the stored cos), G > 0 DELTA
//     (delta = u . cos . w). After the last GEMM the final epilogue runs serially (FWDS: a_L, cos_L and y; REV: delta_0
//     and gx = W0^T delta_0).
//   * Each epilogue block's tile block (a_l or delta_l, the wgrad layout) is transposed through a per-wave LDS scratch
//     into ONE coalesced 1 KiB store, issued at the start of the slice that consumes the block; the lane-major cos
//     block goes out directly (FWDS) or is reloaded NBUF - 1 mid-slices ahead of its epilogue (REV). The mid-slice
//     s_waitcnt vmcnt(N) counts exactly the vector-memory ops issued after the ring slice it publishes.
//   * Ring of 32 KiB slices, 4 slots at 1..3 hidden layers (3 beyond, where the small block leaves no room): the barrier
//     after operand pair 7 of 16 publishes slice s + 1 and frees slot s - 1 for slice s + NBUF - 1; the next slice's
//     first operand pair is read during the last pair.
// Same arithmetic as wide_kernel (sincos_fast on the unscaled pack), so the results are bitwise those of wide_kernel
// (tests/test_gpu_wide.py).
#include "w3i_kernel.hpp"
#include "wide_kernel.hpp"

#ifndef WIDEI_EPI_PAIR
#define WIDEI_EPI_PAIR 15  // operand pair (of 16) after which the epilogue cluster runs (>= 8: after the mid-slice wait)
#endif
static_assert(WIDEI_EPI_PAIR >= 8 && WIDEI_EPI_PAIR < siren::WNB / 2, "REV's cos reload lands at the mid-slice wait");

namespace siren {

constexpr int wsmall_floats_ct(int lh) { return 9 * WH + 4 + (lh + 1) * WH; }
// ring slots: 4 x 32 KiB while the small block fits beside them in the 160 KiB of LDS (1..3 hidden layers: the slice for
// S + 3 is issued at the mid-slice of S, two slices of lead), else 3 (one slice of lead)
constexpr int widei_nbuf(int lh) { return lh <= 3 ? 4 : 3; }

template <int E, int LH>
constexpr bool widei_has(int) { return E >= 0 && E < LH * WNB; }

// the vector-memory ops issued after ring slice S + 1 (issued at the mid-slice of S + 2 - NBUF, right after epilogue
// S + 1's reload) up to the mid-slice wait of slice S: the reloads and ring slices of the mid-slices in between, and the
// stores of the epilogues run after it (FWDS: the direct cos store and the tile flush; REV: the tile flush)
template <int S, int LH, int MODE>
constexpr int widei_allow() {
    constexpr int ahead = widei_nbuf(LH) - 1, NS = LH * WNB;
    int n = 0;
    for (int m = S + 2 - ahead; m < S; ++m) {
        const int e = m + ahead;  // reload and ring slice issued at the mid-slice of m
        n += (MODE == MODE_REV && e >= 0 && e < NS) ? 1 : 0;
        n += e < NS ? 8 : 0;
    }
    for (int e = S + 2 - ahead; e <= S; ++e)
        n += (e >= 0 && e < NS) ? ((MODE == MODE_FWDS ? 1 : 0) + 1) : 0;
    return n;
}

template <int LH, int MODE>
struct WideiState {
    f32x4 b[2];          // B operands [block & 1] of the current slice and the next
    f32x4 acc[2][WNB];   // ping-pong accumulators [G & 1][output block]
    f32x4 pa0, pa1;      // the next slice's first operand pair (in flight)
    f32x4 pc[3];         // REV: cos reload of epilogue E in slot E % 3
    f32x4 tq;            // the last epilogue's tile block, transposed (stored at the start of the next slice)
    float xv[MAXD], gyv[MAXO], yp[MAXO];
};

struct WideiCtx {
    const float* stream;
    float* ring;
    const float* sm;
    int wave, lane, g;
    float w0, w;
    unsigned ring_vaddr, sm_vaddr;  // LDS byte addresses: this lane's 16 B of ring slot 0; small block + 16 g
    const char* cs;      // this wave's lane-major cos scratch, layer 0 (wave-uniform); layer l at + l * lb
    const char* tb;      // this wave's tile (abuf for FWDS, dbuf for REV), layer 0 (wave-uniform)
    int64_t lb;          // bytes between layers (tiles and scratch)
    unsigned vl;         // 16 lane
    unsigned tw, tr;     // LDS transpose scratch: this lane's write / read address
};

// LDS parameters an epilogue block reads: FWDS FIRST W0T[0..3] + b0, SINCOS b_G; REV SEED WoT[0..3]
template <int G, int MODE>
constexpr int widei_nparams() {
    return MODE == MODE_FWDS ? (G == 0 ? 5 : 1) : (G == 0 ? 4 : 0);
}
template <int G, int MODE>
constexpr int widei_param_off(int i, int b) {  // bytes from the small block + 16 g
    return 4 * (16 * b) + 4 * (MODE == MODE_FWDS ? (G == 0 ? (i < 4 ? i * WH : 9 * WH + 4) : 9 * WH + 4 + G * WH)
                                                 : 4 * WH + i * WH);
}
template <int G, int MODE>
struct WideiParams {
    f32x4 v[widei_nparams<G, MODE>() > 0 ? widei_nparams<G, MODE>() : 1];
};
template <int G, int MODE, int B>
__device__ __forceinline__ void widei_param_issue(WideiParams<G, MODE>& ep, unsigned sm_vaddr) {
    static_for<0, widei_nparams<G, MODE>()>([&](auto I) {
        ep.v[decltype(I)::value] = lds_read4<widei_param_off<G, MODE>(decltype(I)::value, B)>(sm_vaddr);
    });
}
template <int G, int MODE>
__device__ __forceinline__ void widei_param_load(WideiParams<G, MODE>& ep, const WideiCtx& cx, int b) {
#pragma unroll
    for (int i = 0; i < widei_nparams<G, MODE>(); ++i)
        ep.v[i] = *(const f32x4*)((const char*)cx.sm + widei_param_off<G, MODE>(i, b) + 16 * cx.g);
}

// this wave's 8 KiB of the 32 KiB slice s (8 saddr-form 1 KiB global_load_lds pieces) into ring slot s % NBUF
template <int NBUF>
__device__ __forceinline__ void widei_ring_issue(const float* __restrict__ stream, float* ring, int s, int wave,
                                                 int lane) {
    const char* src = (const char*)(stream + (int64_t)s * WSLICE + wave * 2048);
    const unsigned dst = lds_addr(ring + (s % NBUF) * WSLICE + wave * 2048);
#pragma unroll
    for (int q = 0; q < 8; ++q) glds_x4(src + q * 1024, 16u * lane, dst + q * 1024);
}

// the layer whose cos epilogue E reads (REV: SEED layer L, then L - G) or writes (FWDS: layer G)
template <int E, int LH, int MODE>
constexpr int widei_layer() { return MODE == MODE_FWDS ? E / WNB : LH - E / WNB; }

template <int E, int LH, int MODE>
__device__ __forceinline__ void widei_reload_issue(WideiState<LH, MODE>& st, const WideiCtx& cx) {
    if constexpr (MODE == MODE_REV && widei_has<E, LH>(0)) {
        constexpr int L = widei_layer<E, LH, MODE>(), B = E % WNB;
        w3_load16(st.pc[E % 3], w3_at(cx.cs, (int64_t)L * cx.lb + B * 1024), cx.vl);
    }
}
template <int E, int LH, int MODE>
__device__ __forceinline__ void widei_reload_landed(WideiState<LH, MODE>& st) {
    if constexpr (MODE == MODE_REV && widei_has<E, LH>(0)) asm volatile("" : "+v"(st.pc[E % 3]));
}
template <int E, int LH, int MODE>
__device__ __forceinline__ void widei_tile_flush(WideiState<LH, MODE>& st, const WideiCtx& cx) {
    if constexpr (widei_has<E, LH>(0)) {
        constexpr int L = widei_layer<E, LH, MODE>(), B = E % WNB;
        asm volatile("" : "+v"(st.tq));  // landed (the caller's lgkmcnt wait)
        w3_store16(w3_at(cx.tb, (int64_t)L * cx.lb + B * 1024), cx.vl, st.tq);
    }
}

// The epilogue that builds block b of GEMM G's B operand (E = G WNB + b); it stages the tile block for the flush at the
// start of slice E and (FWDS) stores the cos block.
template <int G, int LH, int MODE>
__device__ __forceinline__ void widei_epilogue(WideiState<LH, MODE>& st, const WideiCtx& cx, int b,
                                               const WideiParams<G, MODE>& ep, int slot) {
    if constexpr (MODE == MODE_FWDS) {
        f32x4 z;
        float wl;
        if constexpr (G == 0) {
            z = ep.v[4];
#pragma unroll
            for (int k = 0; k < MAXD; ++k) z += st.xv[k] * ep.v[k];  // rows k >= d_in of W0T and x_k are zero
            wl = cx.w0;
        } else {
            z = st.acc[(G + 1) & 1][b] + ep.v[0];
            wl = cx.w;
        }
        f32x4 sn, cs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a, c;
            sincos_fast(opaque(wl) * z[r], a, c);
            sn[r] = a;
            cs[r] = c;
        }
        st.b[b & 1] = sn;
        w3_stage(st.tq, sn, cx.tw, cx.tr);
        w3_store16(w3_at(cx.cs, (int64_t)G * cx.lb + b * 1024), cx.vl, cs);
    } else {
        const f32x4 cs = st.pc[slot];
        f32x4 d;
        if constexpr (G == 0) {
            f32x4 ga = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < MAXO; ++j) ga += opaque(st.gyv[j]) * ep.v[j];  // zero rows / gy_j for j >= d_out
            d = (ga * cs) * opaque(cx.w);
        } else {
            d = (st.acc[(G + 1) & 1][b] * cs) * opaque(cx.w);
        }
        st.b[b & 1] = d;
        w3_stage(st.tq, d, cx.tw, cx.tr);
    }
}

// One slice S = G WNB + KB: 16 operand pairs x 8 MFMAs, the mid-slice ring barrier after pair 7 (REV: epilogue S+2's
// cos reload issued ahead of the ring refill), the tile block of epilogue S stored at its start, and epilogue block
// KB+1 as one VALU cluster after pair WIDEI_EPI_PAIR.
template <int G, int KB, int LH, int MODE>
__device__ __forceinline__ void widei_slice(WideiState<LH, MODE>& st, const WideiCtx& cx) {
    constexpr int NS = LH * WNB;
    constexpr int NBUF = widei_nbuf(LH);
    constexpr int S = G * WNB + KB;
    constexpr int SLOT = (S % NBUF) * WSLICE * 4;
    constexpr int NSLOT = ((S + 1) % NBUF) * WSLICE * 4;
    constexpr bool EPI = KB + 1 < WNB;
    f32x4(&acc)[WNB] = st.acc[G & 1];
    const f32x4 bop = st.b[KB & 1];
    WideiParams<G, MODE> ep;
    if constexpr (EPI && widei_nparams<G, MODE>() > 0) widei_param_issue<G, MODE, KB + 1>(ep, cx.sm_vaddr);
    f32x4 a0 = st.pa0, a1 = st.pa1;
    const unsigned rv = cx.ring_vaddr + SLOT, nv = cx.ring_vaddr + NSLOT;  // ds offsets above 64 KiB: base per slot
    static_for<0, WNB / 2>([&](auto P) {
        constexpr int p = decltype(P)::value;
        if constexpr (p == 8 && S + 1 < NS) {
            // publish slice S+1 (issued behind epilogue S+1's reload) and free the slot of slice S-1 for slice
            // S+NBUF-1; the vector-memory ops issued after slice S+1 stay outstanding (widei_allow)
            constexpr int ALLOW = widei_allow<S, LH, MODE>();
            static_assert(ALLOW < 64, "vmcnt is 6 bits");
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(ALLOW) : "memory");
            widei_reload_landed<S + 1, LH, MODE>(st);
            widei_reload_issue<S + NBUF - 1, LH, MODE>(st, cx);
            __builtin_amdgcn_s_barrier();
            if constexpr (S + NBUF - 1 < NS) {
                const float* spp = cx.stream;
                asm volatile("" : "+s"(spp));  // keep slice addresses from being hoisted into SGPRs
                widei_ring_issue<NBUF>(spp, cx.ring, S + NBUF - 1, cx.wave, cx.lane);
            }
        }
        f32x4 n0, n1;
        constexpr bool NEXT_IN_SLICE = p + 1 < WNB / 2;
        constexpr bool NEXT_SLICE = !NEXT_IN_SLICE && S + 1 < NS;
        if constexpr (NEXT_IN_SLICE) {
            n0 = lds_read4<(2 * p + 2) * 1024>(rv);
            n1 = lds_read4<(2 * p + 3) * 1024>(rv);
        } else if constexpr (NEXT_SLICE) {
            n0 = lds_read4<0>(nv);
            n1 = lds_read4<1024>(nv);
        }
        if constexpr (NEXT_IN_SLICE || NEXT_SLICE)
            lgkm_wait<2>(a0, a1);
        else
            lgkm_wait<0>(a0, a1);
        if constexpr (p == 0 && EPI) {
            // the epilogue parameters were issued before pair 1's reads: the wait above covered them
#pragma unroll
            for (int i = 0; i < widei_nparams<G, MODE>(); ++i) asm volatile("" : "+v"(ep.v[i]));
        }
        // the tile block epilogue S staged (end of the previous slice / before the GEMM): retired by this wait
        if constexpr (p == 0) widei_tile_flush<S, LH, MODE>(st, cx);
        if constexpr (p == WIDEI_EPI_PAIR && EPI) {
            __builtin_amdgcn_sched_barrier(0);
            widei_epilogue<G, LH, MODE>(st, cx, KB + 1, ep, (S + 1) % 3);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            acc[2 * p] = mfma4(a0[r], bop[r], acc[2 * p]);
            acc[2 * p + 1] = mfma4(a1[r], bop[r], acc[2 * p + 1]);
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

template <int G, int LH, int MODE>
__device__ __forceinline__ void widei_gemm(WideiState<LH, MODE>& st, const WideiCtx& cx) {
#pragma unroll
    for (int ob = 0; ob < WNB; ++ob) st.acc[G & 1][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
        WideiParams<G, MODE> ep;
        widei_param_load<G, MODE>(ep, cx, 0);
        widei_epilogue<G, LH, MODE>(st, cx, 0, ep, (G * WNB) % 3);
    }
    static_for<0, WNB>([&](auto KB) { widei_slice<G, decltype(KB)::value, LH, MODE>(st, cx); });
}

template <int G, int LH, int MODE>
__device__ __forceinline__ void widei_run(WideiState<LH, MODE>& st, const WideiCtx& cx) {
    if constexpr (G < LH) {
        widei_gemm<G, LH, MODE>(st, cx);
        widei_run<G + 1, LH, MODE>(st, cx);
    }
}

// Arguments, workspace and grid exactly as wide_kernel<MODE_FWDS / MODE_REV> (launch_wide): FWDS writes y, the a_l
// tiles (abuf) and cos(w z_l) of layers 0..L (spill); REV reads that cos and writes the delta tiles (dbuf) and gx.
template <int LH, int MODE>
__global__ __launch_bounds__(THREADS, 1) void widei_kernel(const float* __restrict__ ws, const float* __restrict__ x,
                                                           int64_t n, const float* __restrict__ gy,
                                                           float* __restrict__ y, float* __restrict__ gx, int d, int o,
                                                           float w0, float w, float* __restrict__ spill,
                                                           float* __restrict__ abuf, float* __restrict__ dbuf,
                                                           int64_t n_pad) {
    static_assert(MODE == MODE_FWDS || MODE == MODE_REV, "the stored-forward split");
    constexpr bool REV = MODE == MODE_REV;
    constexpr int NS = LH * WNB;
    constexpr int SMALL4 = (wsmall_floats_ct(LH) + 3) / 4 * 4;
    constexpr int NBUF = widei_nbuf(LH);
    __shared__ __attribute__((aligned(16))) float lds[NBUF * WSLICE + SMALL4 + WAVES * STB_SCRATCH];
    WideiCtx cx;
    WideiState<LH, MODE> st;
    cx.ring = lds;
    float* sm = lds + NBUF * WSLICE;
    cx.sm = sm;
    cx.lane = threadIdx.x & 63;
    cx.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    cx.g = cx.lane >> 4;
    const int c = cx.lane & 15;
    cx.w0 = w0;
    cx.w = w;
    const SmallLayout L(WH);
    cx.stream = ws + L.pad(LH) + (REV ? (int64_t)LH * WNB * WSLICE : 0);
    const unsigned lds_base = lds_addr(lds);
    cx.ring_vaddr = lds_base + cx.lane * 16;
    cx.sm_vaddr = lds_base + NBUF * WSLICE * 4 + 16 * cx.g;
    {
        const unsigned scr = lds_base + 4u * (NBUF * WSLICE + SMALL4 + cx.wave * STB_SCRATCH);
        cx.tw = scr + 4u * (4 * cx.g * STB_ROW + c);
        cx.tr = scr + 4u * ((cx.lane >> 2) * STB_ROW + 4 * (cx.lane & 3));
    }
    const int64_t wt = (int64_t)blockIdx.x * WAVES + cx.wave;  // this wave's 16-coordinate tile
    cx.lb = n_pad * WH * 4;
    cx.cs = (const char*)(spill + wt * (WH * 16));
    cx.tb = (const char*)((REV ? dbuf : abuf) + wt * (WH * 16));
    cx.vl = 16u * cx.lane;
    const int64_t coord = (int64_t)blockIdx.x * TILE + cx.wave * 16 + c;
    const bool valid = coord < n;
#pragma unroll
    for (int k = 0; k < MAXD; ++k) st.xv[k] = (valid && k < d) ? x[coord * d + k] : 0.f;
#pragma unroll
    for (int j = 0; j < MAXO; ++j) {
        st.gyv[j] = (j < o) ? (gy == nullptr ? 1.f : (valid ? gy[coord * o + j] : 0.f)) : 0.f;
        st.yp[j] = 0.f;
    }
    {
        const int nf4 = (L.floats(LH) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    __syncthreads();
    // prologue: the NBUF - 1 mid-slices before slice 0, in the order the mid-slice counts assume (epilogue e's reload,
    // then ring slice e, for e = 0 .. NBUF - 2); then slice 0 and epilogue 0's reload landed
    static_for<0, NBUF - 1>([&](auto E) {
        widei_reload_issue<decltype(E)::value, LH, MODE>(st, cx);
        widei_ring_issue<NBUF>(cx.stream, cx.ring, decltype(E)::value, cx.wave, cx.lane);
    });
    constexpr int PRO = (NBUF - 2) * (8 + (REV ? 1 : 0));  // ops issued after ring slice 0
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(PRO) : "memory");
    __builtin_amdgcn_s_barrier();
    widei_reload_landed<0, LH, MODE>(st);
    st.pa0 = lds_read4<0>(cx.ring_vaddr);
    st.pa1 = lds_read4<1024>(cx.ring_vaddr);

    widei_run<0, LH, MODE>(st, cx);

    constexpr int GL = (LH - 1) & 1;
    // the final epilogue (serial): its tile blocks go out as four dword stores each (store_block), with no LDS
    // transpose and so no LDS wait between the blocks' arithmetic (measured: the staged form kept the tail serial)
    float* tp = (float*)cx.tb + (int64_t)(REV ? 0 : LH) * (cx.lb / 4) + 4 * cx.g * 16 + c;
    if constexpr (!REV) {
        // last hidden layer: a_L and cos(w z_L) (the reverse pass's seed) out, y = a_L Wout^T + bout
        const float* bl = sm + L.bias + LH * WH + 4 * cx.g;
#pragma unroll
        for (int rb = 0; rb < WNB; ++rb) {
            const f32x4 z = st.acc[GL][rb] + *(const f32x4*)(bl + 16 * rb);
            f32x4 sn, cs;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float a, cc;
                sincos_fast(w * z[r], a, cc);
                sn[r] = a;
                cs[r] = cc;
            }
            store_block(tp, rb, sn);
            w3_store16(w3_at(cx.cs, (int64_t)LH * cx.lb + rb * 1024), cx.vl, cs);
#pragma unroll
            for (int j = 0; j < MAXO; ++j) {
                if (j < o) {
                    const f32x4 wj = *(const f32x4*)(sm + L.wo + j * WH + 16 * rb + 4 * cx.g);
                    st.yp[j] += wj[0] * sn[0] + wj[1] * sn[1] + wj[2] * sn[2] + wj[3] * sn[3];
                }
            }
        }
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            if (j < o) {
                const float yj = sum_groups(st.yp[j]) + sm[L.bout + j];
                if (y != nullptr && valid && cx.g == 0) y[coord * o + j] = yj;
            }
        }
    } else {
        // delta_0 = u_0 . cos(w0 z_0) . w0 (cos_0 from the scratch), its tile, gx = delta_0 W0
        // cos_0 blocks loaded PD blocks ahead of their use (issued before the previous blocks' tile stores): loaded at
        // the use, every block waited for its own load behind the stores, 32 serial memory latencies in every tile's
        // tail (round 6)
        float q[MAXD] = {0.f, 0.f, 0.f, 0.f};
        constexpr int PD = 8;
        f32x4 c0s[WNB];
#pragma unroll
        for (int rb = 0; rb < PD; ++rb) c0s[rb] = *(const f32x4*)(cx.cs + rb * 1024 + 16 * cx.lane);
#pragma unroll
        for (int rb = 0; rb < WNB; ++rb) {
            if (rb + PD < WNB) c0s[rb + PD] = *(const f32x4*)(cx.cs + (rb + PD) * 1024 + 16 * cx.lane);
            const f32x4 c0 = c0s[rb];
            const f32x4 dl = (st.acc[GL][rb] * c0) * w0;
            store_block(tp, rb, dl);
#pragma unroll
            for (int k = 0; k < MAXD; ++k) {
                if (k < d) {
                    const f32x4 wk = *(const f32x4*)(sm + L.w0 + k * WH + 16 * rb + 4 * cx.g);
                    q[k] = dot4_acc(wk, dl, q[k]);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < MAXD; ++k) {
            if (k < d) {
                const float qk = sum_groups(q[k]);
                if (valid && cx.g == 0) gx[coord * d + k] = qk;
            }
        }
    }
}

}  // namespace siren

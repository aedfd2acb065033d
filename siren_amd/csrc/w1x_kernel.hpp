// w1x_kernel.hpp — W1 (fused SIREN forward + coordinate vector-Jacobian product, gy = ones) with the hidden-layer
// GEMMs on the bf16 matrix pipe in fp32-equivalent precision ("bf16x6").
//
// Every fp32 operand is split exactly into three bf16 pieces by truncation, v = hi + mid + lo (hi = the top 8
// significand bits, mid the next 8, lo the last 8; both subtractions are exact), and each K-step of a layer GEMM
// sums the six products whose magnitude is at or above 2^-16 of hi*hi:
//     lo(W) hi(a) + mid(W) mid(a) + hi(W) lo(a) + mid(W) hi(a) + hi(W) mid(a) + hi(W) hi(a)
// in fp32 on v_mfma_f32_16x16x32_bf16 (bf16 x bf16 products are exact in fp32). The dropped terms are 2^-24 of the
// leading one, the fp32 rounding level: against the fp64 goldens this matches the fp32 kernel (G1 gradient
// 1.4e-6 vs 2.0e-6, G2 8.6e-6 vs 8.3e-6 relative; a three-product split lands at 9e-5 / 2.2e-4 and is not used).
// The bf16 pipe issues a 16x16x32 MFMA every 16 cycles against 32 cycles for the fp32 16x16x4, i.e. 8x the K per
// cycle, so six of them cost 2.67x less matrix time than the fp32 K-step.
//
// Tiling (one wave = 16 coordinates = the MFMA columns, as in w1_kernel.hpp):
//   * A = weights. The pack (pack_split_kernel) pre-splits the phase-scaled weights of the 2 L layer GEMMs into
//     slices of half a K-step: 8 output blocks x (hi, mid, lo) x 1 KiB, lane (g, m) holding the 8 bf16 of row
//     16 ob + m at K positions kn(s, g, j) = 32 s + 16 (j >> 2) + 4 g + (j & 3), j = 0..7.
//   * B = activations. After a layer's epilogue, lane (g, c) holds rows 16 b + 4 g + r of column c (the C/D layout);
//     blocks 2s and 2s+1 give exactly the 8 values kn(s, g, 0..7) of K-step s, so the split pieces of the next
//     layer's B operand are built in place (v_perm of the upper halves), with no lane exchange.
//   * A 4-slot LDS ring of 24 KiB slices (global_load_lds), one barrier per slice placed mid-slice (it publishes
//     slice S+1 and frees slot S-1 for slice S+3); the A pieces of the next output block are read one block ahead
//     with a counted lgkmcnt.
//   * The epilogue producing K-step s+1's B operand (two blocks) runs in the MFMA shadow of K-step s; cos(w z_l)
//     of the forward layers is parked in AGPRs for the reverse sweep; the ring streams across the coordinate tiles
//     of a persistent grid.
// Epilogues (phase-scaled pack, as w1_kernel.hpp): FIRST a_0 = sin(x W0^T + b0), SINCOS a_G, SEED (y partials and
// delta_L = seed . cos . w), DELTA delta_l = u_l . cos_l . 2 pi; then delta_0 and gx = delta_0 W0 (VALU).
#pragma once
#include <type_traits>

#include "lds_ops.h"
#include "siren_common.h"
#include "tile_io.h"

namespace siren {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// kernel modes: W1 (y, gx with gy = ones), FWD (the forward-only W0, 8 waves), STORE (the W2 stage of the bf16x6
// training leg: the forward recomputed, the reverse seeded with a per-coordinate gy (d_out 1), and a_l / delta_l written
// as 16-coordinate tiles in the wgrad layout, as w1_kernel MODE_STORE)
// FWDS / REV: the stored-forward split of that W2 stage (as w1_kernel MODE_FWDS / MODE_REV): FWDS is the forward-only
// W0 (8 waves) plus the a_l tiles and the lane-major cos(w z_l), l >= 1; REV runs the reverse GEMMs only, each
// epilogue's cos block reloaded from that buffer (layer 0's recomputed from x, as every mode does), and writes the
// delta_l tiles.
enum { X_W1 = 0, X_FWD = 1, X_STORE = 2, X_FWDS = 3, X_REV = 4 };
constexpr bool x_fwd_like(int xm) { return xm == X_FWD || xm == X_FWDS; }  // forward GEMMs only, two waves per SIMD
// lane-major cos buffer of X_FWDS / X_REV: per 16-coordinate wave tile wt, (L + 1) layers x NB blocks x 64 lanes x f32x4
// (w1_kernel's cos_off with tile WAVES + wave = wt)
__host__ __device__ constexpr int64_t x_cos_off(int64_t wt, int lh) { return wt * (lh + 1) * NB * 256; }
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int X_OBS = 8;                            // output blocks per slice (half a K-step)
constexpr int X_SLICE = 3 * X_OBS * 256;            // 32-bit words per slice: 8 blocks x (hi, mid, lo) x 1 KiB
constexpr int X_NBUF = 4;                           // ring slots (96 KiB)
#ifndef X_EPI_AT
#define X_EPI_AT 7                                  // slice block after which the slice's epilogue block is issued
#endif
#ifndef X_EPI_FENCE
#define X_EPI_FENCE 0  // 1: the epilogue block as one VALU cluster (scheduling barriers around it; A/B probe)
#endif
constexpr int X_KSTEPS = H / 32;                    // K-steps of one 256-wide GEMM
constexpr int X_SPG = 2 * X_KSTEPS;                 // slices per GEMM
constexpr int x_slices(int lh) { return 2 * lh * X_SPG; }  // slices per coordinate tile

__device__ __forceinline__ f32x4 mfma_x(const u32x4& a, const u32x4& b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                    0, 0, 0);
}

// exact 3-way bf16 split of two values into the (lo half, hi half) of one word per piece; the subtractions run as
// one packed v_pk_add_f32 per pair
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 trunc_bf16x2(f32x2 v) {
    return f32x2{__uint_as_float(__float_as_uint(v[0]) & 0xffff0000u),
                 __uint_as_float(__float_as_uint(v[1]) & 0xffff0000u)};
}
__device__ __forceinline__ void split_pair(float v0, float v1, unsigned& h, unsigned& m, unsigned& l) {
    const f32x2 v = {v0, v1};
    h = __builtin_amdgcn_perm(__float_as_uint(v1), __float_as_uint(v0), 0x07060302u);
    const f32x2 r = v - trunc_bf16x2(v);
    m = __builtin_amdgcn_perm(__float_as_uint(r[1]), __float_as_uint(r[0]), 0x07060302u);
    const f32x2 q = r - trunc_bf16x2(r);
    l = __builtin_amdgcn_perm(__float_as_uint(q[1]), __float_as_uint(q[0]), 0x07060302u);
}

// block b of a layer's output (lane: rows 16 b + 4 g + r) -> words 2 (b & 1), 2 (b & 1) + 1 of the K-step's pieces
template <int HALF>
__device__ __forceinline__ void split_block(const f32x4& v, u32x4 (&p)[3]) {
    unsigned h0, m0, l0, h1, m1, l1;
    split_pair(v[0], v[1], h0, m0, l0);
    split_pair(v[2], v[3], h1, m1, l1);
    p[0][2 * HALF] = h0;
    p[0][2 * HALF + 1] = h1;
    p[1][2 * HALF] = m0;
    p[1][2 * HALF + 1] = m1;
    p[2][2 * HALF] = l0;
    p[2][2 * HALF + 1] = l1;
}

// X_REV: cos reload slots (see x_cos_n)
#ifndef X_CQ
#define X_CQ 8
#endif
template <int LH>
struct XState {
    float gyv;         // X_STORE / X_REV: this lane's output cotangent
    f32x4 cq[X_CQ < 6 ? 6 : X_CQ];  // X_REV: reloaded cos blocks, block u of a tile's consumption order in cq[u % X_CQ]
    u32x4 bx[2][3];    // B operand pieces (hi, mid, lo) of K-step s in bx[s & 1]
    f32x4 acc[2][NB];  // ping-pong accumulators (GEMM G in acc[G & 1])
    f32x4 C[LH][NB];   // cos(w z_l), 1 <= l < LH (layer 0's is recomputed at the end: 64 fewer live registers)
    u32x4 pa[3][3];    // A pieces of output blocks b, b + 1, b + 2 of the tile's block sequence (b % 3)
    float xv[4];
    float yp;
    float xn[4], gn;   // X_REV: the next tile's coordinates and cotangent, loaded at the mid of slice 0 (x_next_issue)
};

struct XCtx {
    const unsigned* stream;
    float* ring;
    const float* sm;
    int d, wave, lane, g;
    float w0, w, wsd, inv_s0;
    bool more;
    const char* ta;        // X_STORE: wave-uniform a_l tile base of (tile, wave), layer 0; layer l at + l * lbytes
    const char* td;        // X_STORE: the same for delta_l
    const char* cs;        // X_FWDS / X_REV: wave-uniform lane-major cos base of the wave tile (x_cos_off), + 16 lane
    const char* cs_next;   // X_REV: the same for the next tile (its first cos blocks are loaded at the mid of NS - 2)
    const float* xq;       // X_REV: this lane's x row and gy entry of the next tile (clamped to coordinate n - 1)
    const float* gq;
    int64_t lbytes;
    unsigned vl;           // 16 lane
    unsigned vt;           // X_STORE: this lane's byte offset in a tile block, 4 (4 g 16 + c)
    unsigned ring_vaddr;   // LDS byte address of this lane's 16 B in slot 0
    unsigned ring_vaddr2;  // ... in slot 2
};

// A pieces of block-sequence index BI (compile time) for this lane: three inline-asm ds_read_b128 into pa[BI % 3],
// retired by a counted wait that names exactly those registers (x_wait). The buffers are a static ring with no C++
// copies, so nothing reads a destination before its wait (tools/check_asm_waits.py checks the ISA); the loop-carried
// pieces of the next tile are read and waited in ONE statement (x_read_wait).
template <int OFF>
__device__ __forceinline__ u32x4 xread1(const XCtx& cx) {
    constexpr int HALFRING = 2 * X_SLICE * 4;  // ds offsets are 16-bit: slots 2, 3 use the second base
    if constexpr (OFF < HALFRING)
        return __builtin_bit_cast(u32x4, lds_read4<OFF>(cx.ring_vaddr));
    else
        return __builtin_bit_cast(u32x4, lds_read4<OFF - HALFRING>(cx.ring_vaddr2));
}
// ring byte offset of piece P of block-sequence index BI (slice BI / 8 of the tile in slot (BI / 8) % 4)
template <int BI, int P>
constexpr int xoff() {
    return ((BI / X_OBS) % X_NBUF) * X_SLICE * 4 + (3 * (BI % X_OBS) + P) * 1024;
}
template <int BI, int LH>
__device__ __forceinline__ void x_issue(XState<LH>& st, const XCtx& cx) {
    st.pa[BI % 3][0] = xread1<xoff<BI, 0>()>(cx);
    st.pa[BI % 3][1] = xread1<xoff<BI, 1>()>(cx);
    st.pa[BI % 3][2] = xread1<xoff<BI, 2>()>(cx);
}
template <int N>
__device__ __forceinline__ void x_wait(u32x4 (&a)[3]) {
    asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]) : "i"(N));
}
// blocks 0 and 1 of a tile (slot 0): six reads and their wait in one statement
__device__ __forceinline__ void x_read_wait01(u32x4 (&a)[3], u32x4 (&b)[3], unsigned vaddr) {
    asm volatile(
        "ds_read_b128 %0, %6\n\tds_read_b128 %1, %6 offset:1024\n\tds_read_b128 %2, %6 offset:2048\n\t"
        "ds_read_b128 %3, %6 offset:3072\n\tds_read_b128 %4, %6 offset:4096\n\tds_read_b128 %5, %6 offset:5120\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2])
        : "v"(vaddr));
}

// CPW 1 KiB global->LDS pieces of slice s for this wave (saddr form, as ring_issue4): 24 per slice over the waves
// (6 each at 4 waves per workgroup, 3 at 8)
template <int CPW>
__device__ __forceinline__ void xring_issue(const unsigned* __restrict__ stream, float* ring, int s, int wave,
                                            unsigned lane_off) {
    const char* src = (const char*)(stream + (int64_t)s * X_SLICE + wave * CPW * 256);
    const unsigned dst = lds_addr(ring + (s % X_NBUF) * X_SLICE + wave * CPW * 256);
#pragma unroll
    for (int q = 0; q < CPW; ++q) glds_x4(src + q * 1024, lane_off, dst + q * 1024);
}
// waves per workgroup: 4 (one per SIMD) for W1; 8 (two per SIMD, sharing the ring) for the forward-only W0, whose
// registers fit twice per SIMD without the parked cos
template <bool FWD>
constexpr int x_waves() { return FWD ? 8 : 4; }
// slices per coordinate tile: the forward-only modes and X_REV run L GEMMs, the others 2 L
template <int XM, int LH>
constexpr int x_ns() { return (x_fwd_like(XM) || XM == X_REV) ? LH * X_SPG : x_slices(LH); }
// the GEMM a tile starts at (X_REV: the reverse GEMMs G = LH .. 2 LH - 1)
template <int XM, int LH>
constexpr int x_g0() { return XM == X_REV ? LH : 0; }

template <int I, int N, typename F>
__device__ __forceinline__ void xstatic_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        xstatic_for<I + 1, N>(f);
    }
}
#ifndef X_REV_WAVES
#define X_REV_WAVES 4
#endif
// waves per workgroup of mode XM (X_REV: X_REV_WAVES)
template <int XM>
constexpr int x_nw() { return x_fwd_like(XM) ? 8 : XM == X_REV ? X_REV_WAVES : 4; }

__device__ __forceinline__ f32x4 x_to_agpr(f32x4 v) {
    f32x4 r;
    asm("; park in agpr" : "=a"(r) : "0"(v));
    return r;
}
__device__ __forceinline__ f32x4 x_from_agpr(f32x4 v) {
    f32x4 r;
    asm("; unpark" : "=v"(r) : "0"(v));
    return r;
}
__device__ __forceinline__ f32x4 x_pin(f32x4 v) {
    asm("; pin" : "+v"(v));
    return v;
}

// Epilogue of block B producing the B operand of GEMM E (see the table at the top; the previous GEMM's output is
// acc[(E + 1) & 1]).
// X_STORE: tile block B of layer l (the four 64 B pieces of the lane, as w1_kernel's memory modes); the layer stride
// is made opaque at each use so hipcc keeps no per-layer SGPR pairs live across the tile
__device__ __forceinline__ void x_tile_store(const char* base, const XCtx& cx, int l, int b, const f32x4& v) {
    int64_t lb = cx.lbytes;
    asm volatile("" : "+s"(lb));
    w3_store_tile(w3_at(base, l * lb + b * 1024), cx.vt, v);
}
// vector-memory stores an epilogue producing GEMM E's B operand issues per block: X_STORE a_E (4 dwords), at E = LH also
// delta_L, delta_{2 LH - E} beyond; X_FWDS a_E and (E >= 1) its cos block; X_REV delta
constexpr int x_epi_nst(int e, int lh, int xm) {
    return xm == X_STORE ? (e == lh ? 8 : 4) : xm == X_FWDS ? (e == 0 ? 4 : 5) : xm == X_REV ? 4 : 0;
}
constexpr int x_ns_rt(int xm, int lh) { return (x_fwd_like(xm) || xm == X_REV) ? lh * X_SPG : x_slices(lh); }
// stores of the in-slice epilogue of slice s (after its mid-slice wait: block 2 (KS + 1) + HALF of GEMM s / X_SPG's
// input when KS + 1 < X_KSTEPS), and of the two pre-GEMM blocks run before slice s when s starts a GEMM
constexpr int x_st_slice(int s, int lh, int xm) {
    return (s < 0 || s >= x_ns_rt(xm, lh) || ((s % X_SPG) >> 1) + 1 >= X_KSTEPS)
               ? 0
               : x_epi_nst((xm == X_REV ? lh : 0) + s / X_SPG, lh, xm);
}
constexpr int x_st_pre(int s, int lh, int xm) {
    return (s <= 0 || s >= x_ns_rt(xm, lh) || s % X_SPG != 0)
               ? 0
               : 2 * x_epi_nst((xm == X_REV ? lh : 0) + s / X_SPG, lh, xm);
}
// s_waitcnt vmcnt allowance of slice S's mid-slice wait (S + 2 < NS): ring slice S + 1 was issued at the mid of S - 2;
// after it come the epilogue stores of S - 2, the pre-GEMM blocks before S - 1, ring slice S + 2 (CPW pieces), the
// epilogue stores of S - 1 and the pre-GEMM blocks before S. The first two slices of a tile count CPW (the previous
// tile's serial tail sits between: CPW waits for more than needed, never less).
// X_REV reloads the cos block of each epilogue block X_COS_LEAD slices ahead (a split-bf16 slice is half a K-step,
// ~0.35 us: one slice of lead exposed the load latency, 0.36 of wave cycles waiting). A tile consumes its cos blocks in
// the order u = 16 r + b (block b of reverse GEMM r; b = 0, 1 before the GEMM's first slice, b >= 2 in slice 16 r + b
// - 2); the mid of slice m loads the in-slice block of slice m + X_COS_LEAD and, when slice m + X_COS_LEAD + 1 starts a
// GEMM, that GEMM's blocks 0, 1, into cq[u % 8] (the live blocks are a run of at most X_COS_LEAD + 3).
#ifndef X_COS_LEAD
#define X_COS_LEAD 4
#endif
static_assert(X_COS_LEAD >= 1 && X_COS_LEAD + 3 <= X_CQ, "cos reload slots");
constexpr int x_cos_n(int m, int lh) {  // cos loads issued at the mid of slice m
    const int ns = lh * X_SPG, t = m + X_COS_LEAD;
    return (t < ns && t % X_SPG <= X_SPG - 3 ? 1 : 0) + (t + 1 < ns && (t + 1) % X_SPG == 0 ? 2 : 0);
}
// X_REV: at the mid of slice S the blocks loaded at the mid of S - X_COS_LEAD must have landed (the in-slice block of S,
// and the next GEMM's pre-GEMM blocks when S ends a GEMM); after them: that mid's ring issue, the loads and ring issues
// of the mids in between, the epilogue stores of slices S - X_COS_LEAD .. S - 1 and the pre-GEMM stores before the GEMMs
// starting in (S - X_COS_LEAD, S]. Before slice X_COS_LEAD everything was loaded at the tile start (waited there).
constexpr int x_allow_rev(int S, int lh, int cpw) {
    int n = cpw;
    for (int m = S - X_COS_LEAD + 1; m < S; ++m) n += x_cos_n(m, lh) + cpw;
    for (int s = S - X_COS_LEAD; s < S; ++s) n += x_st_slice(s, lh, X_REV);
    for (int s = S - X_COS_LEAD + 1; s <= S; ++s) n += x_st_pre(s, lh, X_REV);
    return n;
}
// X_REV, ring constraint: ring slice S + 1 must have landed at the mid of S. It was issued at the mid of S - 2 (for
// S < 2 at the previous tile's mids NS - 2, NS - 1); after it come, in issue order, the epilogue stores of S - 2, the
// pre-GEMM stores before S - 1, the mid of S - 1 (its cos reloads, at NS - 2 the next tile's first X_COS_LEAD + 2 cos
// blocks (x_next_cos), its ring slice), the epilogue stores of S - 1 and the pre-GEMM stores before S. Across the tile
// boundary: the previous tile's 64 delta_0 tile stores, the seed's two pre-GEMM blocks, and at the mid of slice 0 the
// next tile's D + 1 input loads (x_next_issue) before its ring slice. The compiler's own conditional y / gx stores only
// add younger operations (waiting for more, never less); 63 is the counter's maximum.
constexpr int x_allow_ring_rev(int S, int lh, int cpw, int d) {
    const int ns = lh * X_SPG, pre0 = 2 * x_epi_nst(lh, lh, X_REV);
    int n = 0;
    if (S == 0)
        n = cpw + 64 + pre0;
    else if (S == 1)
        n = 64 + pre0 + x_cos_n(0, lh) + (d + 1) + cpw + x_st_slice(0, lh, X_REV);
    else
        n = x_st_slice(S - 2, lh, X_REV) + x_st_pre(S - 1, lh, X_REV) + x_cos_n(S - 1, lh) +
            (S - 1 == ns - 2 ? X_COS_LEAD + 2 : 0) + cpw + x_st_slice(S - 1, lh, X_REV) + x_st_pre(S, lh, X_REV);
    return n < 63 ? n : 63;
}
template <int S, int LH, int XM, int CPW, int D = 2>
constexpr int x_allow() {
    if constexpr (XM == X_REV) {
        // the cos blocks of slices < X_COS_LEAD were waited at the tile start; later ones at the mid of S - X_COS_LEAD
        constexpr int r = x_allow_ring_rev(S, LH, CPW, D);
        if constexpr (S < X_COS_LEAD) {
            return r;
        } else {
            constexpr int c = x_allow_rev(S, LH, CPW);
            return c < r ? c : r;
        }
    } else if constexpr ((XM != X_STORE && XM != X_FWDS) || S < 2) {
        return CPW;
    } else {
        constexpr int n = CPW + x_st_slice(S - 2, LH, XM) + x_st_pre(S - 1, LH, XM) + x_st_slice(S - 1, LH, XM) +
                          x_st_pre(S, LH, XM);
        static_assert(n < 64, "vmcnt is 6 bits");
        return n;
    }
}
// the layer whose cos an epilogue producing GEMM E's input reads in X_REV: L for the seed (E = LH), 2 LH - E beyond
constexpr int x_rev_layer(int e, int lh) { return e == lh ? lh : 2 * lh - e; }
// X_REV: cos block B of layer l into r (saddr form: wave-uniform base + 16 lane)
template <int L, int B>
__device__ __forceinline__ void x_cos_issue(f32x4& r, const XCtx& cx) {
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(r) : "v"(cx.vl), "s"(w3_at(cx.cs, (L * NB + B) * 1024)));
}
// X_REV, across the tile boundary: the next tile's first X_COS_LEAD + 2 cos blocks (the seed's pre-GEMM blocks 0, 1 and
// the in-slice blocks of its first X_COS_LEAD slices) into cq[0 ..], issued at the mid of slice NS - 2, when every
// block of this tile has been consumed, and waited (counted) at the next tile's start; and its D coordinates and gy
// entry, issued at the mid of slice 0 (before that mid's ring slice). Both are inline asm the compiler does not count:
// a compiler load consumed at the tile start made it drain the counter there (vmcnt(0) right after issuing the next
// tile's loads), a full memory latency per 64-coordinate tile. The inputs land in AGPRs and stay there until the
// tile start's wait names them (a VGPR destination was copied to an AGPR by the compiler while still in flight); so do
// the next tile's first cos blocks.
template <int LH, int U>
__device__ __forceinline__ void x_next_cos1(f32x4& r, const XCtx& cx) {
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=a"(r) : "v"(cx.vl), "s"(w3_at(cx.cs_next, (LH * NB + U) * 1024)));
}
template <int LH>
__device__ __forceinline__ void x_next_cos(XState<LH>& st, const XCtx& cx) {
    xstatic_for<0, X_COS_LEAD + 2>([&](auto U) { x_next_cos1<LH, decltype(U)::value>(st.cq[decltype(U)::value], cx); });
}
template <int D, int LH>
__device__ __forceinline__ void x_next_issue(XState<LH>& st, const XCtx& cx) {
#pragma unroll
    for (int k = 0; k < D; ++k) asm volatile("global_load_dword %0, %1, off" : "=a"(st.xn[k]) : "v"(cx.xq + k) : "memory");
    asm volatile("global_load_dword %0, %1, off" : "=a"(st.gn) : "v"(cx.gq) : "memory");
}
static_assert(X_EPI_AT >= 4, "the in-slice epilogue's stores are counted after the mid-slice wait");

template <int E, int B, int LH, int D, int XM>
__device__ __forceinline__ void x_epilogue(XState<LH>& st, const XCtx& cx) {
    constexpr bool FWD = x_fwd_like(XM), ST = XM == X_STORE, FWS = XM == X_FWDS, RV = XM == X_REV;
    constexpr int CQ = (XM == X_REV ? (16 * (E - LH) + B) % X_CQ : 0);  // X_REV: the reloaded cos block's slot
    constexpr int KS = B >> 1, HALF = B & 1;
    const int nb = 16 * B + 4 * cx.g;
    u32x4(&p)[3] = st.bx[KS & 1];
    if constexpr (E == 0) {
        f32x4 z = *(const f32x4*)(cx.sm + SM_BIAS + nb);
#pragma unroll
        for (int k = 0; k < D; ++k) z += st.xv[k] * *(const f32x4*)(cx.sm + SM_W0 + k * H + nb);
        f32x4 sn, cs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a_, c_;
            sincos_rev(z[r], a_, c_);
            sn[r] = a_;
            cs[r] = c_;
        }
        split_block<HALF>(sn, p);
        if constexpr (ST || FWS) x_tile_store(cx.ta, cx, 0, B, sn);
    } else if constexpr (E < LH) {
        const f32x4 z = st.acc[(E + 1) & 1][B] + *(const f32x4*)(cx.sm + SM_BIAS + E * H + nb);
        f32x4 sn, cs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a_, c_;
            sincos_rev(z[r], a_, c_);
            sn[r] = a_;
            cs[r] = c_;
        }
        if constexpr (!FWD) st.C[E][B] = x_to_agpr(cs);
        split_block<HALF>(sn, p);
        if constexpr (ST || FWS) x_tile_store(cx.ta, cx, E, B, sn);
        if constexpr (FWS) w3_store16(w3_at(cx.cs, (E * NB + B) * 1024), cx.vl, cs);
    } else if constexpr (E == LH && RV) {
        // delta_L = (gy Wout) . cos(w z_L) . w with cos from X_FWDS
        const f32x4 wo = *(const f32x4*)(cx.sm + SM_WO + nb);
        const f32x4 dl = ((opaque(st.gyv) * wo) * st.cq[CQ]) * cx.wsd;
        split_block<HALF>(dl, p);
        x_tile_store(cx.td, cx, LH, B, dl);
    } else if constexpr (E == LH) {
        const f32x4 z = st.acc[(E + 1) & 1][B] + *(const f32x4*)(cx.sm + SM_BIAS + LH * H + nb);
        f32x4 sn, cs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a_, c_;
            sincos_rev(z[r], a_, c_);
            sn[r] = a_;
            cs[r] = c_;
        }
        const f32x4 wo = *(const f32x4*)(cx.sm + SM_WO + nb);
        st.yp += wo[0] * sn[0] + wo[1] * sn[1] + wo[2] * sn[2] + wo[3] * sn[3];
        // delta_L = (gy Wout) . cos . w (W1: gy = ones, the seed row sum_j Wout_j)
        const f32x4 sd = ST ? opaque(st.gyv) * wo : *(const f32x4*)(cx.sm + SM_SEED + nb);
        const f32x4 dl = (sd * cs) * cx.wsd;
        split_block<HALF>(dl, p);
        if constexpr (ST) {
            x_tile_store(cx.ta, cx, LH, B, sn);
            x_tile_store(cx.td, cx, LH, B, dl);
        }
    } else {
        constexpr int L = 2 * LH - E;  // delta_L = u_L . cos(w z_L) . w, 1 <= L < LH
        const f32x4 dl = (st.acc[(E + 1) & 1][B] * (RV ? st.cq[CQ] : x_from_agpr(st.C[L][B]))) * cx.w;
        split_block<HALF>(dl, p);
        if constexpr (ST || RV) x_tile_store(cx.td, cx, L, B, dl);
    }
}

// Slice (G, KS, HALF): the output blocks ob = 8 HALF .. 8 HALF + 7 of K-step KS, six MFMAs each; the mid-slice ring
// barrier after block 3; the next block's (or the next slice's first block's) A pieces read one block ahead; then
// the epilogue block of K-step KS + 1 (block 2 (KS + 1) + HALF) of the previous GEMM's output.
template <int G, int KS, int HALF, int LH, int D, int XM>
__device__ __forceinline__ void x_slice(XState<LH>& st, const XCtx& cx) {
    constexpr bool FWD = x_fwd_like(XM);
    constexpr int NS = x_ns<XM, LH>();
    constexpr int CPW = 24 / x_nw<XM>();
    constexpr int S = (G - x_g0<XM, LH>()) * X_SPG + 2 * KS + HALF;
    constexpr int SLOT = (S % X_NBUF) * X_SLICE * 4;
    constexpr int NSLOT = ((S + 1) % X_NBUF) * X_SLICE * 4;
    f32x4(&acc)[NB] = st.acc[G & 1];
    const u32x4(&b)[3] = st.bx[KS & 1];
    xstatic_for<0, X_OBS>([&](auto OBL) {
        constexpr int obl = decltype(OBL)::value;
        constexpr int ob = X_OBS * HALF + obl;
        constexpr int BI = S * X_OBS + obl;  // block-sequence index in the tile (NS * 8 blocks, a multiple of 3)
        constexpr int NBI = NS * X_OBS;
        if constexpr (obl == 4) {
            if (S + 1 < NS || cx.more) {
                if constexpr (S + 2 < NS)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(x_allow<S, LH, XM, CPW, D>()) : "memory");
                else if (cx.more)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(XM == X_REV ? x_allow<S, LH, XM, CPW, D>() : CPW) : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if constexpr (XM == X_REV) {
                    // landed: this slice's in-slice cos block and, in a GEMM's last slice, the next GEMM's blocks 0, 1
                    if constexpr (S % X_SPG <= X_SPG - 3)
                        asm volatile("" : "+v"(st.cq[(S + 2) % X_CQ]));  // u = 16 (S / 16) + S % 16 + 2
                    if constexpr ((S + 1) % X_SPG == 0 && S + 1 < NS)
                        asm volatile("" : "+v"(st.cq[(S + 1) % X_CQ]), "+v"(st.cq[(S + 2) % X_CQ]));
                    // reload X_COS_LEAD slices ahead (x_cos_n)
                    constexpr int T = S + X_COS_LEAD;
                    if constexpr (T < NS && T % X_SPG <= X_SPG - 3)
                        x_cos_issue<x_rev_layer(LH + T / X_SPG, LH), T % X_SPG + 2>(st.cq[(T + 2) % X_CQ], cx);
                    if constexpr (T + 1 < NS && (T + 1) % X_SPG == 0) {
                        x_cos_issue<x_rev_layer(LH + (T + 1) / X_SPG, LH), 0>(st.cq[(T + 1) % X_CQ], cx);
                        x_cos_issue<x_rev_layer(LH + (T + 1) / X_SPG, LH), 1>(st.cq[(T + 2) % X_CQ], cx);
                    }
                    if constexpr (S == NS - 2) {
                        if (cx.more) x_next_cos<LH>(st, cx);
                    }
                }
                __builtin_amdgcn_s_barrier();
                if constexpr (XM == X_REV && S == 0) x_next_issue<D>(st, cx);
                if (S + 3 < NS || cx.more) {
                    const unsigned* sp = cx.stream;
                    asm volatile("" : "+s"(sp));
                    xring_issue<CPW>(sp, cx.ring, (S + 3) % NS, cx.wave, 16u * cx.lane);
                }
            }
        }
        // pieces of block BI + 2 (its slice is published: the next slice's, by this slice's mid barrier)
        if constexpr (BI + 2 < NBI) {
            x_issue<BI + 2, LH>(st, cx);
            x_wait<6>(st.pa[BI % 3]);
        } else if constexpr (BI + 1 < NBI) {
            x_wait<3>(st.pa[BI % 3]);
        } else {
            x_wait<0>(st.pa[BI % 3]);
        }
        const u32x4(&a)[3] = st.pa[BI % 3];
        // smallest products first
        acc[ob] = mfma_x(a[2], b[0], acc[ob]);
        acc[ob] = mfma_x(a[1], b[1], acc[ob]);
        acc[ob] = mfma_x(a[0], b[2], acc[ob]);
        acc[ob] = mfma_x(a[1], b[0], acc[ob]);
        acc[ob] = mfma_x(a[0], b[1], acc[ob]);
        acc[ob] = mfma_x(a[0], b[0], acc[ob]);
        // the next tile's blocks 0, 1 (slot 0, published by this slice's barrier), read and waited at once
        if constexpr (BI + 1 == NBI) {
            if (cx.more) x_read_wait01(st.pa[0], st.pa[1], cx.ring_vaddr);
        }
        // the epilogue block of K-step KS + 1, placed early in the slice so its VALU spreads over the remaining
        // blocks' MFMAs (after the last block it ran as a cluster with the matrix pipe idle)
        if constexpr (obl == X_EPI_AT && KS + 1 < X_KSTEPS) {
            if (X_EPI_FENCE) __builtin_amdgcn_sched_barrier(0);
            x_epilogue<G, 2 * (KS + 1) + HALF, LH, D, XM>(st, cx);
            if (X_EPI_FENCE) __builtin_amdgcn_sched_barrier(0);
        }
    });
}

template <int G, int LH, int D, int XM>
__device__ __forceinline__ void x_gemm(XState<LH>& st, const XCtx& cx) {
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) st.acc[G & 1][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    x_epilogue<G, 0, LH, D, XM>(st, cx);
    x_epilogue<G, 1, LH, D, XM>(st, cx);
    xstatic_for<0, X_KSTEPS>([&](auto KS) {
        x_slice<G, decltype(KS)::value, 0, LH, D, XM>(st, cx);
        x_slice<G, decltype(KS)::value, 1, LH, D, XM>(st, cx);
    });
}

template <int G, int LH, int D, int XM>
__device__ __forceinline__ void x_run(XState<LH>& st, const XCtx& cx) {
    if constexpr (G < (x_fwd_like(XM) ? LH : 2 * LH)) {
        x_gemm<G, LH, D, XM>(st, cx);
        x_run<G + 1, LH, D, XM>(st, cx);
    }
}

// ws: the split image of siren_pack_split (small block at ws_small, bf16 stream at stream); x (n, D); y (n) / gx
// (n, D) (y nullable; X_STORE: gx nullable). w0 / w as the fp32 kernel (phase-scaled pack). X_STORE: gy (n) the output
// cotangent, abuf / dbuf the a_l / delta_l tiles (L + 1 layers of n_pad H floats each, the wgrad layout).
template <int LH, int D, int XM>
__global__ __launch_bounds__(64 * x_nw<XM>(), 1) void w1x_kernel(
    const float* __restrict__ ws_small, const unsigned* __restrict__ stream, const float* __restrict__ x, int64_t n,
    float* __restrict__ y, float* __restrict__ gx, float w0, float w, const float* __restrict__ gy = nullptr,
    float* __restrict__ abuf = nullptr, float* __restrict__ dbuf = nullptr, int64_t n_pad = 0) {
    // X_FWDS: abuf = a_l tiles, dbuf = the lane-major cos buffer; X_REV: abuf = that cos buffer, dbuf = delta_l tiles
    constexpr bool FWD = x_fwd_like(XM), ST = XM == X_STORE, FWS = XM == X_FWDS, RV = XM == X_REV;
    constexpr int NS = x_ns<XM, LH>();
    constexpr int NW = x_nw<XM>(), NT = 64 * NW, TILEX = 16 * NW, CPW = 24 / NW;
    static_assert(NS % X_NBUF == 0, "the ring must wrap onto slot 0 at a tile boundary");
    // the small-parameter block FIRST: its epilogue reads are then one base register + immediate offsets (after the
    // 96 KiB ring they were out of ds offset range, and the compiler kept ~50 per-block addresses live and spilled them)
    constexpr int SMALL = (SM_BIAS + (LH + 1) * H + 255) / 256 * 256;
    __shared__ __attribute__((aligned(16))) float lds[SMALL + X_NBUF * X_SLICE];
    XCtx cx;
    XState<LH> st;
    cx.ring = lds + SMALL;
    float* sm = lds;
    cx.sm = sm;
    cx.stream = stream + (RV ? (int64_t)LH * X_SPG * X_SLICE : 0);  // X_REV: the reverse GEMMs' slices
    cx.lane = threadIdx.x & 63;
    cx.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    cx.g = cx.lane >> 4;
    cx.d = D;
    const int c = cx.lane & 15;
    {
        constexpr float two_pi = 6.28318530717958648f;
        const float s = w * 0.159154943091895336f;
        cx.w0 = w0 / s;
        cx.w = two_pi;
        cx.wsd = w;
        cx.inv_s0 = two_pi / w0;
    }
    cx.more = false;
    cx.ta = cx.td = cx.cs = nullptr;
    cx.lbytes = n_pad * H * 4;
    cx.vt = 4u * (4 * cx.g * 16 + c);
    cx.vl = 16u * cx.lane;
    cx.ring_vaddr = lds_addr(cx.ring) + cx.lane * 16;
    cx.ring_vaddr2 = cx.ring_vaddr + 2 * X_SLICE * 4;
    {
        const int nf4 = (SM_BIAS + (LH + 1) * H + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += NT) ((f32x4*)sm)[e] = ((const f32x4*)ws_small)[e];
    }
    // the stored split writes its tiles for every n_pad coordinate (the wgrad reads the padding too; n_pad a multiple of
    // 128, the forward's tile)
    const int64_t tiles = (FWS || RV) ? n_pad / TILEX : (n + TILEX - 1) / TILEX;
    float xn[4], gn = 0.f;
    auto load_inputs = [&](int64_t tile) {
        const int64_t cd = tile * TILEX + cx.wave * 16 + c;
        const bool ok = tile < tiles && cd < n;
#pragma unroll
        for (int k = 0; k < 4; ++k) xn[k] = (ok && k < D) ? x[cd * D + k] : 0.f;
        if constexpr (ST || RV) gn = ok ? gy[cd] : 0.f;
    };
    if constexpr (!RV) load_inputs(blockIdx.x);
    __syncthreads();
    xring_issue<CPW>(cx.stream, cx.ring, 0, cx.wave, 16u * cx.lane);
    xring_issue<CPW>(cx.stream, cx.ring, 1, cx.wave, 16u * cx.lane);
    xring_issue<CPW>(cx.stream, cx.ring, 2, cx.wave, 16u * cx.lane);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * CPW) : "memory");
    __builtin_amdgcn_s_barrier();
    x_read_wait01(st.pa[0], st.pa[1], cx.ring_vaddr);
    auto next_inputs = [&](int64_t tile) {  // X_REV: x_next_issue's addresses (clamped: the loads are unconditional)
        int64_t cd = tile * TILEX + cx.wave * 16 + c;
        cd = cd < n ? cd : n - 1;
        cx.xq = x + cd * D;
        cx.gq = gy + cd;
    };
    if constexpr (RV) {
#pragma unroll
        for (int k = 0; k < 4; ++k) st.xn[k] = 0.f;
        st.gn = 0.f;
        if (blockIdx.x < tiles) {
            // the first tile's blocks and inputs, issued and waited in one statement (separate statements let the
            // compiler copy the in-flight destinations before the wait)
            static_assert(X_COS_LEAD + 2 <= 6, "the first-tile load names six cos blocks");
            const char* cb = (const char*)(abuf + x_cos_off((int64_t)blockIdx.x * NW + cx.wave, LH));
            next_inputs(blockIdx.x);
            asm volatile(
                "global_load_dwordx4 %0, %10, %11\n\tglobal_load_dwordx4 %1, %10, %12\n\t"
                "global_load_dwordx4 %2, %10, %13\n\tglobal_load_dwordx4 %3, %10, %14\n\t"
                "global_load_dwordx4 %4, %10, %15\n\tglobal_load_dwordx4 %5, %10, %16\n\t"
                "global_load_dword %6, %17, off\n\tglobal_load_dword %7, %17, off offset:4\n\t"
                "global_load_dword %8, %17, off offset:%c19\n\tglobal_load_dword %9, %18, off\n\t"
                "s_waitcnt vmcnt(0)"
                : "=&a"(st.cq[0]), "=&a"(st.cq[1]), "=&a"(st.cq[2]), "=&a"(st.cq[3]), "=&a"(st.cq[4]), "=&a"(st.cq[5]),
                  "=&a"(st.xn[0]), "=&a"(st.xn[1]), "=&a"(st.xn[2]), "=&a"(st.gn)
                : "v"(cx.vl), "s"(w3_at(cb, (LH * NB + 0) * 1024)), "s"(w3_at(cb, (LH * NB + 1) * 1024)),
                  "s"(w3_at(cb, (LH * NB + 2) * 1024)), "s"(w3_at(cb, (LH * NB + 3) * 1024)),
                  "s"(w3_at(cb, (LH * NB + 4) * 1024)), "s"(w3_at(cb, (LH * NB + 5) * 1024)), "v"(cx.xq), "v"(cx.gq),
                  "i"(D == 3 ? 8 : 4)  // D = 2: the third load re-reads the row's second entry (xv zeroes k >= D)
                : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }

#pragma unroll 1
    for (int64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        cx.more = tile + gridDim.x < tiles;
        const int64_t coord = tile * TILEX + cx.wave * 16 + c;
        const bool valid = coord < n;
        if constexpr (!RV) {
#pragma unroll
            for (int k = 0; k < 4; ++k) st.xv[k] = xn[k];
            st.gyv = gn;
        }
        st.yp = 0.f;
        {
            const int64_t wt = tile * NW + cx.wave;  // the 16-coordinate wave tile (wave-uniform)
            const int64_t tbase = wt * (H * 16);
            if constexpr (ST) {
                cx.ta = (const char*)(abuf + tbase);
                cx.td = (const char*)(dbuf + tbase);
            }
            if constexpr (FWS) {
                cx.ta = (const char*)(abuf + tbase);
                cx.cs = (const char*)(dbuf + x_cos_off(wt, LH));
            }
            if constexpr (RV) {
                cx.td = (const char*)(dbuf + tbase);
                cx.cs = (const char*)(abuf + x_cos_off(wt, LH));
                cx.cs_next = (const char*)(abuf + x_cos_off(wt + (int64_t)gridDim.x * NW, LH));
                // landed: this tile's first cos blocks (x_next_cos at the previous tile's mid NS - 2, or the prologue)
                // and inputs (x_next_issue, older); after them only ring slices 1, 2 (2 CPW) and the 64 delta_0 stores
                // were issued (capped at the counter's 63: also waits for those ring slices, which mids 0, 1 need)
                static_assert(X_COS_LEAD + 2 <= 6, "the tile start's wait names six cos blocks");
                asm volatile("s_waitcnt vmcnt(%10)"
                             : "+a"(st.cq[0]), "+a"(st.cq[1]), "+a"(st.cq[2]), "+a"(st.cq[3]), "+a"(st.cq[4]),
                               "+a"(st.cq[5]), "+a"(st.xn[0]), "+a"(st.xn[1]), "+a"(st.xn[2]), "+a"(st.gn)
                             : "n"(2 * CPW + 64 < 63 ? 2 * CPW + 64 : 63)
                             : "memory");
#pragma unroll
                for (int k = 0; k < 4; ++k) st.xv[k] = (valid && k < D) ? st.xn[k] : 0.f;
                st.gyv = valid ? st.gn : 0.f;
                next_inputs(tile + gridDim.x);
            }
        }
        if constexpr (!RV) load_inputs(tile + gridDim.x);
        x_run<x_g0<XM, LH>(), LH, D, XM>(st, cx);
        if constexpr (FWD) {
            // last hidden layer: a_L = sin(w z_L) and y = a_L Wout^T + bout (serial over the 16 blocks)
            constexpr int GL = (LH - 1) & 1;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const int nb = 16 * rb + 4 * cx.g;
                const f32x4 z = st.acc[GL][rb] + *(const f32x4*)(sm + SM_BIAS + LH * H + nb);
                const f32x4 wo = *(const f32x4*)(sm + SM_WO + nb);
                f32x4 sn4, cs4;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float sn_, cs_;
                    sincos_rev(z[r], sn_, cs_);
                    st.yp += wo[r] * sn_;
                    sn4[r] = sn_;
                    cs4[r] = cs_;
                }
                if constexpr (FWS) {  // a_L tile and cos(w z_L) for the reverse's seed
                    x_tile_store(cx.ta, cx, LH, rb, sn4);
                    w3_store16(w3_at(cx.cs, (LH * NB + rb) * 1024), cx.vl, cs4);
                }
            }
            const float yv = sum_groups(st.yp) + sm[SM_BOUT];
            if (y != nullptr && valid && cx.g == 0) y[coord] = yv;
            continue;
        }
        {
            const float yv = sum_groups(st.yp) + sm[SM_BOUT];
            if (y != nullptr && valid && cx.g == 0) y[coord] = yv;
        }
        // delta_0 = u_0 . cos(w0 z_0) . w0 (cx.w0 = w0 / s undoes the pack scale); gx = delta_0 W0 (cx.inv_s0)
        constexpr int GL = (2 * LH - 1) & 1;
        float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            const int nb = 16 * rb + 4 * cx.g;
            f32x4 z = *(const f32x4*)(sm + SM_BIAS + nb);
#pragma unroll
            for (int k = 0; k < D; ++k) z += st.xv[k] * *(const f32x4*)(sm + SM_W0 + k * H + nb);
            f32x4 c0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float sn_, cs_;
                sincos_rev(z[r], sn_, cs_);
                c0[r] = cs_;
            }
            const f32x4 dl = (st.acc[GL][rb] * c0) * cx.w0;
            if constexpr (ST || RV) x_tile_store(cx.td, cx, 0, rb, dl);
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * cx.g);
                q[k] += wk[0] * dl[0] + wk[1] * dl[1] + wk[2] * dl[2] + wk[3] * dl[3];
            }
        }
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const float qk = sum_groups(q[k]) * cx.inv_s0;
            if (valid && cx.g == 0 && (!(ST || RV) || gx != nullptr)) gx[coord * D + k] = qk;
        }
    }
    if constexpr (RV) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last x_next_issue (clamped, unused)
}

// The split image's bf16 stream from the flat parameters (state-dict order): slice (G, s, half), output block
// ob = 8 half + obl, piece p: lane (g, m) holds 8 bf16 of A row 16 ob + m at K positions kn(s, g, j), where A is
// s_scale W_{G+1} for the forward GEMMs G < LH and s_scale W_{2LH-G}^T for the reverse ones (s_scale = w / 2 pi, the
// phase-scaled pack). One thread per (slice, chunk, lane) word quad.
__global__ void pack_split_kernel(const float* __restrict__ p, unsigned* __restrict__ stream, int d, int o, int lh,
                                  float s_scale) {
    const int64_t total = (int64_t)x_slices(lh) * 3 * X_OBS * 64;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= total) return;
    const int lane = (int)(q & 63), chunk = (int)((q >> 6) % (3 * X_OBS));
    const int64_t slice = (q >> 6) / (3 * X_OBS);
    const int G = (int)(slice / X_SPG), ks = (int)((slice % X_SPG) >> 1), half = (int)(slice & 1);
    const int obl = chunk / 3, piece = chunk % 3;
    const int g = lane >> 4, m = lane & 15;
    const int row = 16 * (X_OBS * half + obl) + m;
    // W_l offset in the flat buffer: W0 (H, d), b0, then (W_l, b_l) for l = 1..lh
    const int layer = G < lh ? G + 1 : 2 * lh - G;
    const int64_t wl = (int64_t)H * d + H + (int64_t)(layer - 1) * (H * H + H);
    unsigned out[4];
#pragma unroll
    for (int w2 = 0; w2 < 4; ++w2) {
        unsigned half16[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const int j = 2 * w2 + e;
            const int kn = 32 * ks + 16 * (j >> 2) + 4 * g + (j & 3);
            const float v = s_scale * (G < lh ? p[wl + (int64_t)row * H + kn] : p[wl + (int64_t)kn * H + row]);
            const unsigned bv = __float_as_uint(v);
            const float r = v - __uint_as_float(bv & 0xffff0000u);
            const unsigned br = __float_as_uint(r);
            const float r2 = r - __uint_as_float(br & 0xffff0000u);
            const unsigned pc = piece == 0 ? bv : (piece == 1 ? br : __float_as_uint(r2));
            half16[e] = pc >> 16;
        }
        out[w2] = half16[0] | (half16[1] << 16);
    }
    (void)o;
    *(u32x4*)(stream + ((slice * (3 * X_OBS) + chunk) * 64 + lane) * 4) = u32x4{out[0], out[1], out[2], out[3]};
}

}  // namespace siren

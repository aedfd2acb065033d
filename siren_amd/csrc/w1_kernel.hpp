// w1_kernel.hpp — the headline kernel: fused SIREN forward + coordinate vector-Jacobian product (W1) for
// gfx950, with every sin/cos epilogue interleaved into the NEXT layer's MFMA stream.
//
// Same math and tiling as fused_kernels.hpp: v_mfma_f32_16x16x4_f32, weights as A operands
// from an LDS ring of 16 KiB slices, activations as B operands kept in C/D layout. On top of it:
//   * The L forward and L reverse GEMMs are fully unrolled (G = 0 .. 2L-1): every slice index, ring slot and
//     register-array index is a compile-time constant, so the hot loop has no branches.
//   * Ping-pong accumulators acc[G & 1]: while GEMM G accumulates into acc[G&1] slice by slice, the epilogue
//     of GEMM G-1 (held in acc[(G+1)&1]) runs one 16-neuron block ahead: during slice kb the wave turns block
//     kb+1 of the previous pre-activation into the B operand of slice kb+1, so the ~25 VALU of each sin/cos
//     issue in the MFMA shadow (one wave per SIMD; the matrix pipe takes 32 cycles per MFMA).
//   * A operands are read by inline-asm ds_read_b128 one pair of output blocks ahead, and the consumer MFMAs
//     are tied to a counted s_waitcnt lgkmcnt(N) through "+v" operands (hipcc would otherwise read each pair
//     right before use and wait lgkmcnt(0)).
//   * 4-slot ring, ONE barrier per slice placed mid-slice: it publishes slice s+1 (landed two slices after its
//     global_load_lds) and frees slot s-1 for slice s+3, so the first operands of slice s+1 are read while the
//     second half of slice s still computes — no operand latency is exposed at slice boundaries.
//   * Epilogue per GEMM G (L = LH hidden layers):
//       G = 0         FIRST : z0 = x W0^T + b0 (VALU, K = d_in)  -> a_0 = sin(w0 z0), C[0] = cos(w0 z0)
//       1 <= G < L    SINCOS: z_G = acc + b_G                   -> a_G, C[G]
//       G = L         SEED  : z_L = acc + b_L -> y partials (a_L . Wout), delta_L = (gy Wout) . cos . w
//       L < G < 2L    DELTA : delta_{2L-G} = u . C[2L-G] . w
//     then after the last GEMM: delta_0 = u_0 . C[0] . w0 and gx = delta_0 W0.
//   * sincos_fast (siren_common.h) is branch-free: fma Cody-Waite with a full-precision pi/2, valid for
//     |w z| < 1e6 rad (|z| < 3.3e4 at w = 30), <= 1.1e-7 absolute error.
//   * STORE (W2 backward stage 1) additionally writes a_l and delta_l in 16-coordinate tiles.
//   * JET (W4, the fused Laplacian): forward sweep only, but the 16 MFMA columns of a wave are 4 coordinates x
//     4 jet streams s (column 4q + s): s = 0 the value z, s = 1, 2 the tangents dz/dx_s, s = 3 the second-order
//     sum sum_i d2z/dx_i2. Weights act on every stream (bias only on s = 0), and the epilogue maps the jet of z
//     to the jet of a = sin(w z) with the quad's stream-0/1/2 values broadcast by DPP quad_perm:
//       a = sin(w z), da_i = w cos(w z) dz_i, d2a = w cos(w z) d2z - w^2 sin(w z) sum_i dz_i^2.
//     The output layer turns the streams into y, grad y and the Laplacian (diff_operators.py:27-43).
// Requires outermost_linear (SingleBVPNet); the notebook Siren's final sine uses fused_kernel.
#pragma once
#include <type_traits>

#include "lds_ops.h"
#include "siren_common.h"
#include "tile_io.h"

namespace siren {

constexpr int W1_NBUF = 4;  // ring slots of this kernel (64 KiB)

// Where a slice runs its epilogue block (w1_slice). An f32 MFMA and the VALU share the wave's issue: a VALU placed
// singly between MFMAs costs ~14.5 cycles, in a cluster ~6-8.5 (tools/micro/mfma_valu_cluster.hip). The W1 mode (no
// loads or stores in its epilogue) runs the block as ONE cluster fenced by scheduling barriers after operand pair 1
// (A/B over pairs 0 / 1 / 2 / 5 / slice end: pair 1 -2.1 % kernel time, profiles/r03x_epilogue_placement.log); so
// does the forward-only W0; the modes with loads or stores in the epilogue (STORE / FWDS / REV: the REV cos prefetch
// lands at the mid-slice wait, and stores issued before it would be waited for by it) run it after pair 4.
#ifndef W1_EPI_PAIR
#define W1_EPI_PAIR 1
#endif
#ifndef W1_EPI_FWD
#define W1_EPI_FWD 1  // W0 3.29 -> 3.22 ms (profiles/r03x_epilogue_placement.log)
#endif
#ifndef W1_EPI_JET
#define W1_EPI_JET 8  // pair 1 measured neutral on the Poisson step
#endif
#ifndef W1_EPI_MEM
#define W1_EPI_MEM 6  // STORE / FWDS / REV (>= 4: after the mid-slice wait): pair 6 vs 4 -1 .. -1.5 % on the REV / FWDS
                      // kernels of the image-fit and hypernet steps (profiles/r04e_epilogue_mem.log)
#endif
template <int MODE>
constexpr int w1_epi_pair() {
    return (MODE & MODE_BASE) == MODE_W1    ? W1_EPI_PAIR
           : (MODE & MODE_BASE) == MODE_FWD ? W1_EPI_FWD
           : (MODE & MODE_BASE) == MODE_JET ? W1_EPI_JET
                                             : W1_EPI_MEM;
}
// MODE_REV reloads the cos block of epilogue E at the mid-slice of slice E - W1_COS_LEAD (before that mid's ring issue)
// into cq[E % W1_COS_SLOTS]. Lead 2 makes the mid-slice wait of slice E - 1 wait for it one slice after its issue; lead
// 3 lets it ride with ring slice E (two slices); lead 4 lands it one slice before the slice that runs its epilogue, which
// is what an epilogue placed ahead of the mid-slice wait (W1_EPI_MEM < 4) needs.
#ifndef W1_COS_LEAD
#define W1_COS_LEAD 3
#endif
constexpr int W1_COS_SLOTS = W1_COS_LEAD <= 3 ? 3 : 4;
static_assert(W1_COS_LEAD >= 2 && W1_COS_LEAD <= 4, "cos reload lead of 2..4 slices");
static_assert(W1_EPI_MEM >= 4 || W1_COS_LEAD >= 4, "an epilogue ahead of the mid-slice wait needs the cos lead of 4");

enum { EPI_FIRST = 0, EPI_SINCOS = 1, EPI_SEED = 2, EPI_DELTA = 3 };


template <int G, int LH>
constexpr int epi_kind() {
    return G == 0 ? EPI_FIRST : (G < LH ? EPI_SINCOS : (G == LH ? EPI_SEED : EPI_DELTA));
}
// LDS parameter reads an epilogue block needs: FIRST W0T[0..3] + b0; SINCOS b_G; SEED b_L + WoutT[0..3] + seed
template <int KIND>
constexpr int epi_nparams() {
    return KIND == EPI_FIRST ? 5 : (KIND == EPI_SINCOS ? 1 : (KIND == EPI_SEED ? 6 : 0));
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// cos(w z_l) of layers l >= 1 is parked in AGPRs (the accumulator half of the unified register file): it is
// only read back once, by the reverse epilogue. The empty asm statements pin the register class.
__device__ __forceinline__ f32x4 to_agpr(f32x4 v) {
    f32x4 r;
    asm("; park in agpr" : "=a"(r) : "0"(v));
    return r;
}
__device__ __forceinline__ f32x4 from_agpr(f32x4 v) {
    f32x4 r;
    asm("; unpark" : "=v"(r) : "0"(v));
    return r;
}
// Opaque identity: materialises v here (LLVM would otherwise sink the cos bit-select to its use in the
// reverse sweep and keep ~5 intermediates per element alive across the whole forward pass).
__device__ __forceinline__ f32x4 pin(f32x4 v) {
    asm("; pin" : "+v"(v));
    return v;
}

template <int MODE>
constexpr int npasses() { return forward_only(MODE & MODE_BASE) || (MODE & MODE_BASE) == MODE_REV ? 1 : 2; }
// first GEMM of a tile: MODE_REV runs only the reverse GEMMs G = LH .. 2 LH - 1 (its stream pointer starts at the
// transposed slices, so slice indices are counted from G0)
template <int MODE, int LH>
constexpr int gemm0() { return (MODE & MODE_BASE) == MODE_REV ? LH : 0; }
template <int MODE>
constexpr bool is_rev() { return (MODE & MODE_BASE) == MODE_REV; }
template <int MODE>
constexpr bool is_jet() { return (MODE & MODE_BASE) == MODE_JET || (MODE & MODE_BASE) == MODE_JETS; }

// ---- the memory modes' epilogue stores (STORE / FWDS / REV) ----------------------------------------------------------
// Epilogue E of a tile (E = (G - G0) NB + b builds block b of GEMM G's B operand; E % NB == 0 runs before the GEMM, the
// others inside slice E - 1) writes its tile blocks (a_l: FIRST / SINCOS / STORE's SEED; delta_l: SEED / DELTA), and
// FWDS its lane-major cos block. Every store is ONE inline-asm instruction, so the mid-slice wait of slice S counts the
// ops issued after the ring slice it publishes exactly (w1_allow) instead of waiting for every store of the last two
// epilogues. Tile blocks leave as the four 64 B dword pieces from the epilogue itself; W1_STAGE=1 instead transposes
// them through LDS into one coalesced 1 KiB store flushed at the start of slice E (STORE / REV only: FWDS runs two
// workgroups per CU and has no LDS left for the scratch), measured 1.5 % slower on the REV kernel of the image-fit
// step (profiles/r05_w1_mem_ab.log).
#ifndef W1_STAGE
#define W1_STAGE 0
#endif
template <int MODE>
constexpr bool w1_mem() {
    return (MODE & MODE_BASE) == MODE_STORE || (MODE & MODE_BASE) == MODE_FWDS || (MODE & MODE_BASE) == MODE_REV ||
           (MODE & MODE_BASE) == MODE_JETS;
}
// the forward halves (two workgroups per CU: no LDS for the transpose scratch) store their tiles directly
constexpr bool w1_fwd_half(int mode) {
    return (mode & MODE_BASE) == MODE_FWDS || (mode & MODE_BASE) == MODE_JETS;
}
template <int MODE>
constexpr bool w1_staged() { return W1_STAGE != 0 && w1_mem<MODE>() && !w1_fwd_half(MODE); }
template <int MODE>
constexpr bool w1_tiles() { return w1_mem<MODE>() && (MODE & MODE_NOTILE) == 0; }
// the next tile's inputs as inline-asm loads retired by the tile's counted waits: the memory modes at one wave per SIMD
// (STORE, REV). The forward-only modes run two workgroups per CU (the other one covers a drain) in 256 registers, where
// hipcc reallocated an in-flight asm destination (tools/check_asm_waits.py), so they keep compiler loads. So does the W1
// mode: its headline body is spill-free only with cos(w0 z_0) parked in LDS, and that body, with these loads, measured
// 0.1-0.8 % slower than the spilling one on four same-box A/Bs — the spill reloads' drains hit a
// ring slice that has mostly landed.
template <int MODE>
constexpr bool w1_asm_inputs() {
    return ((MODE & MODE_BASE) == MODE_STORE || (MODE & MODE_BASE) == MODE_REV) && (MODE & MODE_PROF) == 0;
}
constexpr bool w1_mem_rt(int mode) {
    return (mode & MODE_BASE) == MODE_STORE || (mode & MODE_BASE) == MODE_FWDS || (mode & MODE_BASE) == MODE_REV ||
           (mode & MODE_BASE) == MODE_JETS;
}
constexpr int w1_nslices(int lh, int mode) {
    return (mode & MODE_BASE) == MODE_STORE || (mode & MODE_BASE) == MODE_W1 ? 2 * lh * NB : lh * NB;
}
// tile blocks epilogue E writes (STORE's SEED: a_L and delta_L)
constexpr int w1_ntile(int e, int lh, int mode) {
    if (!w1_mem_rt(mode) || (mode & MODE_NOTILE) != 0 || e < 0 || e >= w1_nslices(lh, mode)) return 0;
    const int g = ((mode & MODE_BASE) == MODE_REV ? lh : 0) + e / NB;
    return (mode & MODE_BASE) == MODE_STORE && g == lh ? 2 : 1;
}
// Vector-memory instructions of epilogue E by position in the slice sequence, in half slices (half 2 s: slice s before
// its mid-slice wait, 2 s + 1: after it). The epilogue's own stores run at pair W1_EPI_MEM of slice E - 1 (E % NB == 0:
// after slice E - 1, before the GEMM); its staged tile blocks leave at the start of slice E (half 2 E).
constexpr int w1_direct(int e, int lh, int mode) {
    if (e < 0 || e >= w1_nslices(lh, mode)) return 0;
    return (W1_STAGE != 0 && !w1_fwd_half(mode) ? 0 : 4 * w1_ntile(e, lh, mode)) + (w1_fwd_half(mode) ? 1 : 0);
}
constexpr int w1_direct_half(int e) { return e % NB != 0 && W1_EPI_MEM < 4 ? 2 * (e - 1) : 2 * (e - 1) + 1; }
constexpr int w1_ops_in_half(int h, int lh, int mode) {
    int n = 0;
    for (int e = h / 2; e <= h / 2 + 1; ++e)
        if (w1_direct_half(e) == h) n += w1_direct(e, lh, mode);
    if (h % 2 == 0 && W1_STAGE != 0 && !w1_fwd_half(mode)) n += w1_ntile(h / 2, lh, mode);
    return n;
}
// s_waitcnt vmcnt allowance of slice S's mid-slice wait (S + 2 < NS): ring slice S + 1 (issued at the mid of S - 2) and,
// in REV, the cos reload of the epilogue that runs before the next mid-slice wait (S + 1; S + 2 when the epilogue sits
// ahead of the wait) must have landed; everything issued after the later of the two may stay in flight. The mid of m
// issues the cos reload of epilogue m + W1_COS_LEAD, then ring slice m + 3. The first two slices of a tile count 4 (the
// previous tile's serial tail or the prologue sits between: 4 waits for more than needed, never less).
constexpr int w1_allow_rt(int S, int lh, int mode) {
    if (!w1_mem_rt(mode) || S < 2) return 4;
    const bool rev = (mode & MODE_BASE) == MODE_REV;
    const int ns = w1_nslices(lh, mode);
    const int need = S + 1 + (W1_EPI_MEM < 4 ? 1 : 0);  // REV: the cos reload that must have landed
    const int mc = need - W1_COS_LEAD;                 // ... issued at this mid
    int m0 = S - 2, n = 0;
    if (rev && mc > S - 2) {
        m0 = mc;
        n += 4;  // that mid's ring issue, behind the cos reload
    }
    for (int h = 2 * m0 + 1; h <= 2 * S; ++h) n += w1_ops_in_half(h, lh, mode);
    for (int m = m0 + 1; m < S; ++m) n += (rev && m + W1_COS_LEAD < ns ? 1 : 0) + 4;
    return n;
}
template <int S, int LH, int MODE>
constexpr int w1_allow() {
    constexpr int n = w1_allow_rt(S, LH, MODE);
    static_assert(n >= 0 && n < 64, "vmcnt is 6 bits");
    return n;
}

template <int LH, int MODE>
struct W1State {
    f32x4 act[NB];     // B operand of the current GEMM (filled one block ahead)
    f32x4 acc[2][NB];  // ping-pong accumulators
    f32x4 C[forward_only(MODE & MODE_BASE) || (MODE & MODE_BASE) == MODE_REV ? 1 : LH][NB];  // cos(w z_l), l < LH
                                                                     // (unused in forward-only modes and REV)
    f32x4 pa0, pa1;    // prefetched first operand pair of the next slice
    float xv[MAXD];    // this lane's coordinate
    float gyv[MAXO];   // this lane's output cotangent
    float yp[MAXO];    // partial y over this lane's neurons
    f32x4 cq[W1_COS_SLOTS];  // MODE_REV: cos blocks of the next epilogues (slot e % W1_COS_SLOTS, W1_COS_LEAD)
    f32x4 c0q[(MODE & MODE_BASE) == MODE_REV ? NB : 1];  // MODE_REV: cos(w0 z_0) of the delta_0 tail (loaded at mid NS - 3)
    f32x4 tq[2];       // W1_STAGE: the last epilogue's tile blocks, transposed (stored at the start of the next slice)
};

struct W1Ctx {
    const float* stream;
    float* ring;
    const float* sm;
    int d, o, wave, lane, g;
    // phase-scaled pack (weights carry w / 2 pi, pack_kernel): w = 2 pi multiplies the reverse GEMM output s W^T delta
    // into W^T delta . w cos, w0 = w0_true / s does the same for layer 0, wsd = w_true seeds delta_L, inv_s0 = 1 / s0
    // undoes the first layer's scale in gx
    float w0, w, wsd, inv_s0;
    bool seed_ones;
    float* abuf;  // STORE / FWDS: lane-adjusted tile base of layer 0; layer l at + l * lstride (the serial tails)
    float* dbuf;  // STORE / REV: delta tiles, same layout
    const char* ta;     // STORE / FWDS: wave-uniform a_l tile base of (tile, wave), layer 0; layer l at + l * lbytes
    const char* td;     // STORE / REV: the same for the delta tiles
    const char* cs;     // FWDS: wave-uniform lane-major cos base of (tile, wave) (cos_off(tile, wave, LH, 0, 0, 0))
    const char* cbase;  // REV: wave-uniform cos base of (tile, wave) (SGPRs), + 16 * lane per lane
    const char* cnext;  // REV: the same for the next tile of this workgroup (its first cos blocks load at mid NS - 1)
    unsigned vl, vt;    // this lane's byte offset: 16 lane (coalesced blocks), 4 (4 g 16 + c) (the 64 B pieces)
    unsigned tw, tr;    // W1_STAGE: LDS transpose scratch of the wave, this lane's write / read address
    int64_t lbytes;
    bool more;    // persistent grid: this workgroup runs another coordinate tile after the current one, so the
                  // ring keeps streaming (slices 0..2 of the next tile are issued during the last 3 slices)
    int64_t lstride;
    unsigned ring_vaddr;  // LDS byte address of this lane's 16 B in slot 0 of the ring
    unsigned sm_vaddr;    // LDS byte address of the small-parameter block + this lane's 4*g neuron offset
    unsigned long long* prof;  // MODE_PROF: this wave's stamp row of the current tile (nullptr: not recorded)
    unsigned long long stamp[PROF_EVENTS];  // MODE_PROF: stamps of the current tile (uniform: SGPRs), stored at its end
    // JET: per-lane stream coefficients (stream s = lane & 3)
    float jcf[MAXD];      // first layer: z = sum_k jcf[k] W0[:, k] + jcb b0  (value: x_k; tangent s: e_{s-1})
    float jcb;            // 1 on the value stream (bias), else 0
    float ja, jb0, jg0, jb, jg;  // a = ja sin + jb cos dz - jg sin |dz|^2  (jb0/jg0 with w0, jb/jg with w)
    float jdA0, jdB0, jdC0, jdA, jdB, jdC;  // JETS: the reverse's z-jet combinations (jet_sin_d_rev), layer 0 / >= 1
};

// Four 1 KiB global->LDS pieces of slice s for this wave, as saddr-form global_load_lds_dwordx4: SGPR slice base
// (+ q KiB by s_add), the per-lane 16 B as a 32-bit VGPR offset, the LDS destination in M0 — no 64-bit VALU address
// arithmetic per piece (hipcc's builtin lowering builds a 64-bit VGPR address each time; VALU issue is what an
// f32-MFMA kernel pays for, siren_common.h sincos_fast). wave must be wave-uniform. The loads are counted in vmcnt
// exactly like the builtin's (the ring's counted waits are unchanged).
__device__ __forceinline__ void ring_issue4(const float* __restrict__ stream, float* ring, int s, int wave,
                                            unsigned lane_off) {
    const char* src = (const char*)(stream + (int64_t)s * SLICE + wave * 1024);
    const unsigned dst = lds_addr(ring + (s % W1_NBUF) * SLICE + wave * 1024);
#pragma unroll
    for (int q = 0; q < 4; ++q) glds_x4(src + q * 1024, lane_off, dst + q * 1024);
}

// MODE_REV: cos block of epilogue index E (E = (G - LH) NB + b handles block b of reverse GEMM G's epilogue: layer
// LH for the SEED epilogue G = LH, layer 2 LH - G for DELTA) as a saddr-form global_load_dwordx4 into
// cq[E % W1_COS_SLOTS].
// Issued before a ring issue, so the ring's counted s_waitcnt vmcnt(4) one slice later also covers it.
template <int E, int LH, int MODE>
__device__ __forceinline__ void cos_issue(W1State<LH, MODE>& st, const W1Ctx& cx, const char* base) {
    constexpr int GE = LH + E / NB, BE = E % NB;
    constexpr int LC = GE == LH ? LH : 2 * LH - GE;
    asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(st.cq[E % W1_COS_SLOTS]) : "v"(16u * cx.lane),
                 "s"(base + (LC * NB + BE) * 1024));
}
template <int E, int LH, int MODE>
__device__ __forceinline__ void cos_issue(W1State<LH, MODE>& st, const W1Ctx& cx) {
    cos_issue<E, LH, MODE>(st, cx, cx.cbase);
}
// MODE_REV: the delta_0 tail's 16 cos(w0 z_0) blocks (layer 0 of this tile's cos buffer), issued at the mid of slice
// NS - 3 behind its wait and ahead of its ring issue; the mid of slice NS - 2 waits vmcnt(0) anyway (its epilogue's cos
// block), and that one wait statement names them (one shape on every path: no copies of in-flight registers)
template <int LH, int MODE>
__device__ __forceinline__ void c0_issue(W1State<LH, MODE>& st, const W1Ctx& cx) {
#pragma unroll
    for (int b = 0; b < NB; ++b)
        asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(st.c0q[b]) : "v"(16u * cx.lane), "s"(cx.cbase + b * 1024));
}
// the wait that retires them, naming every destination (hipcc must not copy one before it)
template <int N, int LH, int MODE>
__device__ __forceinline__ void c0_wait(W1State<LH, MODE>& st) {
    asm volatile("s_waitcnt vmcnt(%16)"
                 : "+v"(st.c0q[0]), "+v"(st.c0q[1]), "+v"(st.c0q[2]), "+v"(st.c0q[3]), "+v"(st.c0q[4]), "+v"(st.c0q[5]),
                   "+v"(st.c0q[6]), "+v"(st.c0q[7]), "+v"(st.c0q[8]), "+v"(st.c0q[9]), "+v"(st.c0q[10]), "+v"(st.c0q[11]),
                   "+v"(st.c0q[12]), "+v"(st.c0q[13]), "+v"(st.c0q[14]), "+v"(st.c0q[15])
                 : "n"(N)
                 : "memory");
}

// ---- epilogue parameters (LDS) -------------------------------------------------------------------------
template <int KIND, int G, int LH>
struct EpiParams {
    f32x4 v[epi_nparams<KIND>() > 0 ? epi_nparams<KIND>() : 1];
};

// Byte offset (inside the small block, relative to this lane's neuron offset 4*g) of parameter i, block b.
template <int KIND, int G, int LH>
constexpr int epi_param_off(int i, int b) {
    return 4 * (16 * b) + 4 * (KIND == EPI_FIRST ? (i < 4 ? SM_W0 + i * H : SM_BIAS)
                                : KIND == EPI_SINCOS ? SM_BIAS + G * H
                                : (i == 0 ? SM_BIAS + LH * H : (i < 5 ? SM_WO + (i - 1) * H : SM_SEED)));
}

// asm reads (counted by the caller's lgkmcnt) of block B's parameters
template <int KIND, int G, int LH, int B>
__device__ __forceinline__ void epi_issue(EpiParams<KIND, G, LH>& ep, unsigned sm_vaddr) {
    static_for<0, epi_nparams<KIND>()>([&](auto I) {
        ep.v[decltype(I)::value] = lds_read4<epi_param_off<KIND, G, LH>(decltype(I)::value, B)>(sm_vaddr);
    });
}

// plain loads (block 0, outside the pipelined slice loop)
template <int KIND, int G, int LH>
__device__ __forceinline__ void epi_load(EpiParams<KIND, G, LH>& ep, const W1Ctx& cx, int b) {
#pragma unroll
    for (int i = 0; i < epi_nparams<KIND>(); ++i)
        ep.v[i] = *(const f32x4*)((const char*)cx.sm + epi_param_off<KIND, G, LH>(i, b) + 16 * cx.g);
}

// Tile block b of an epilogue (layer base wave-uniform): staged into tq[K] for the flush at the start of the next slice,
// or (FWDS) stored at once as the four 64 B pieces.
// Byte offset of (layer l, block b) in a tile buffer. The layer stride is made opaque at each use: hipcc would otherwise
// keep the products l * lbytes of every layer live in SGPRs across the tile (spilled to VGPR lanes).
__device__ __forceinline__ int64_t w1_tile_off(const W1Ctx& cx, int l, int b) {
    int64_t lb = cx.lbytes;
    asm volatile("" : "+s"(lb));
    return l * lb + b * 1024;
}
template <int MODE, int K, int LH>
__device__ __forceinline__ void w1_tile_put(W1State<LH, MODE>& st, const W1Ctx& cx, const char* base, int l, int b,
                                            const f32x4& v) {
    if constexpr (w1_staged<MODE>())
        w3_stage(st.tq[K], v, cx.tw, cx.tr);
    else
        w3_store_tile(w3_at(base, w1_tile_off(cx, l, b)), cx.vt, v);
}

// The staged tile blocks of epilogue E, stored at the start of slice E (after the lgkmcnt wait that retired them).
template <int E, int LH, int MODE>
__device__ __forceinline__ void w1_flush(W1State<LH, MODE>& st, const W1Ctx& cx) {
    if constexpr (w1_staged<MODE>() && w1_ntile(E, LH, MODE) > 0) {
        constexpr int GE = gemm0<MODE, LH>() + E / NB, BE = E % NB, K = epi_kind<GE, LH>();
        constexpr int L = K == EPI_DELTA ? 2 * LH - GE : (K == EPI_SEED ? LH : GE);
        if constexpr (w1_ntile(E, LH, MODE) == 2) {  // STORE's SEED: a_L, delta_L
            asm volatile("" : "+v"(st.tq[0]), "+v"(st.tq[1]));
            w3_store16(w3_at(cx.ta, w1_tile_off(cx, L, BE)), cx.vl, st.tq[0]);
            w3_store16(w3_at(cx.td, w1_tile_off(cx, L, BE)), cx.vl, st.tq[1]);
        } else {
            asm volatile("" : "+v"(st.tq[0]));
            const char* base = (K == EPI_FIRST || K == EPI_SINCOS) ? cx.ta : cx.td;
            w3_store16(w3_at(base, w1_tile_off(cx, L, BE)), cx.vl, st.tq[0]);
        }
    }
}

// Epilogue for one 16-neuron block b of GEMM G (see the table at the top).
template <int G, int LH, int MODE>
__device__ __forceinline__ void w1_epilogue(W1State<LH, MODE>& st, const W1Ctx& cx, int b,
                                            const EpiParams<epi_kind<G, LH>(), G, LH>& ep) {
    constexpr int KIND = epi_kind<G, LH>();
    constexpr bool STORE = (MODE & MODE_BASE) == MODE_STORE;
    constexpr bool FWD = forward_only(MODE & MODE_BASE);
    constexpr bool FWDS = (MODE & MODE_BASE) == MODE_FWDS;
    constexpr bool REV = is_rev<MODE>();
    if constexpr ((MODE & MODE_BASE) == MODE_JET && KIND == EPI_FIRST) {
        f32x4 z = cx.jcf[0] * ep.v[0];
#pragma unroll
        for (int k = 1; k < MAXD; ++k)
            if (k < cx.d) z += cx.jcf[k] * ep.v[k];
        z += cx.jcb * ep.v[4];
        st.act[b] = jet_sin_rev(z, cx.ja, cx.jb0, cx.jg0);
    } else if constexpr ((MODE & MODE_BASE) == MODE_JET && KIND == EPI_SINCOS) {
        const f32x4 z = st.acc[(G + 1) & 1][b] + cx.jcb * ep.v[0];
        st.act[b] = jet_sin_rev(z, cx.ja, cx.jb, cx.jg);
    } else if constexpr ((MODE & MODE_BASE) == MODE_JETS) {
        f32x4 z, dz;
        if constexpr (KIND == EPI_FIRST) {
            z = cx.jcf[0] * ep.v[0];
#pragma unroll
            for (int k = 1; k < MAXD; ++k)
                if (k < cx.d) z += cx.jcf[k] * ep.v[k];
            z += cx.jcb * ep.v[4];
            st.act[b] = jet_sin_d_rev(z, cx.ja, cx.jb0, cx.jg0, cx.jdA0, cx.jdB0, cx.jdC0, dz);
        } else {
            z = st.acc[(G + 1) & 1][b] + cx.jcb * ep.v[0];
            st.act[b] = jet_sin_d_rev(z, cx.ja, cx.jb, cx.jg, cx.jdA, cx.jdB, cx.jdC, dz);
        }
        w1_tile_put<MODE, 0>(st, cx, cx.ta, G, b, st.act[b]);
        w3_store16(w3_at(cx.cs, w1_tile_off(cx, G, b)), cx.vl, dz);
    } else if constexpr (KIND == EPI_FIRST) {
        f32x4 z = st.xv[0] * ep.v[0];  // phase u_0 = w0 (x W0^T + b0) / 2 pi: the pack carries the scale
#pragma unroll
        for (int k = 1; k < MAXD; ++k)
            if (k < cx.d) z += st.xv[k] * ep.v[k];
        z += ep.v[4];
        f32x4 cs4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sn, cs;
            sincos_rev(z[r], sn, cs);
            st.act[b][r] = sn;
            cs4[r] = cs;
        }
        if constexpr (!FWD) st.C[0][b] = pin(cs4);
        if constexpr (w1_tiles<MODE>()) w1_tile_put<MODE, 0>(st, cx, cx.ta, 0, b, st.act[b]);
        if constexpr (FWDS) w3_store16(w3_at(cx.cs, b * 1024), cx.vl, cs4);
    } else if constexpr (KIND == EPI_SINCOS) {
        const f32x4 z = st.acc[(G + 1) & 1][b] + ep.v[0];
        f32x4 cs4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sn, cs;
            sincos_rev(z[r], sn, cs);
            st.act[b][r] = sn;
            cs4[r] = cs;
        }
        if constexpr (!FWD) st.C[G][b] = to_agpr(cs4);
        if constexpr (w1_tiles<MODE>()) w1_tile_put<MODE, 0>(st, cx, cx.ta, G, b, st.act[b]);
        if constexpr (FWDS) w3_store16(w3_at(cx.cs, (G * NB + b) * 1024), cx.vl, cs4);
    } else if constexpr (KIND == EPI_SEED && REV) {
        // delta_L = (gy Wout) . cos(w z_L) . w with cos from the forward's store
        const f32x4 cs = st.cq[((G - LH) * NB + b) % W1_COS_SLOTS];
        f32x4 ga = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < MAXO; ++j)
            if (j < cx.o && !cx.seed_ones) ga += st.gyv[j] * ep.v[1 + j];
        if (cx.seed_ones) ga = ep.v[5];
        st.act[b] = (ga * cs) * opaque(cx.wsd);
        if constexpr (w1_tiles<MODE>()) w1_tile_put<MODE, 0>(st, cx, cx.td, LH, b, st.act[b]);
    } else if constexpr (KIND == EPI_SEED) {
        const f32x4 z = st.acc[(G + 1) & 1][b] + ep.v[0];
        f32x4 sn, cs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a, c;
            sincos_rev(z[r], a, c);
            sn[r] = a;
            cs[r] = c;
        }
        if constexpr (STORE) w1_tile_put<MODE, 0>(st, cx, cx.ta, LH, b, sn);
        f32x4 ga = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            if (j < cx.o) {
                const f32x4 wj = ep.v[1 + j];
                st.yp[j] += wj[0] * sn[0] + wj[1] * sn[1] + wj[2] * sn[2] + wj[3] * sn[3];
                if (!cx.seed_ones) ga += st.gyv[j] * wj;
            }
        }
        if (cx.seed_ones) ga = ep.v[5];
        st.act[b] = (ga * cs) * opaque(cx.wsd);
        if constexpr (STORE) w1_tile_put<MODE, 1>(st, cx, cx.td, LH, b, st.act[b]);
    } else {
        constexpr int L = 2 * LH - G;  // delta_L = u_L . cos(w z_L) . w,  1 <= L < LH
        if constexpr (REV)
            st.act[b] = (st.acc[(G + 1) & 1][b] * st.cq[((G - LH) * NB + b) % W1_COS_SLOTS]) * cx.w;
        else
            st.act[b] = (st.acc[(G + 1) & 1][b] * from_agpr(st.C[L][b])) * cx.w;
        if constexpr (w1_tiles<MODE>()) w1_tile_put<MODE, 0>(st, cx, cx.td, L, b, st.act[b]);
    }
}

// One slice s = 16 G + KB: 8 operand pairs x 8 MFMAs, the mid-slice ring barrier after pair 3, the next
// slice's first pair prefetched during pair 7, and epilogue block KB+1 of GEMM G-1 in the MFMA shadow.
template <int G, int KB, int LH, int MODE>
__device__ __forceinline__ void w1_slice(W1State<LH, MODE>& st, const W1Ctx& cx) {
    constexpr int NS = npasses<MODE>() * LH * NB;
    constexpr int S = (G - gemm0<MODE, LH>()) * NB + KB;
    constexpr int SLOT = (S % W1_NBUF) * SLICE * 4;
    constexpr int NSLOT = ((S + 1) % W1_NBUF) * SLICE * 4;
    constexpr int KIND = epi_kind<G, LH>();
    constexpr bool EPI = KB + 1 < NB;
    constexpr int EPI_AT = w1_epi_pair<MODE>();
    f32x4 (&acc)[NB] = st.acc[G & 1];
    const f32x4 bop = st.act[KB];
    EpiParams<KIND, G, LH> ep;
    if constexpr (EPI && epi_nparams<KIND>() > 0) epi_issue<KIND, G, LH, KB + 1>(ep, cx.sm_vaddr);
    f32x4 a0 = st.pa0, a1 = st.pa1;
    static_for<0, NB / 2>([&](auto P) {
        constexpr int p = decltype(P)::value;
        if constexpr (p == 4) {
            // publish slice S+1 (own part landed: at most slice S+2's 4 loads still outstanding) and free the
            // slot of slice S-1 (every wave is past its last read of it) for slice S+3. Slices past the end of the
            // tile are the next tile's slices 0..2 (NS is a multiple of the ring size, so the slots line up).
            if (S + 1 < NS || cx.more) {
                if constexpr (S + 2 < NS) {
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(w1_allow<S, LH, MODE>()) : "memory");
                } else if constexpr (is_rev<MODE>() && S + 2 == NS) {
                    // the last epilogue's cos block (issued W1_COS_LEAD slices earlier) is retired whether or not the next
                    // tile's ring slices were issued behind it: one wait shape on every path (a `more`-dependent
                    // vmcnt(4) / vmcnt(0) pair compiles into branches the static ISA check cannot correlate); then the
                    // delta_0 tail's cos blocks
                    static_assert(NB == 16, "c0_wait names 16 blocks");
                    c0_wait<0>(st);  // ... and the delta_0 tail's cos blocks (issued at the previous mid)
                } else if (cx.more) {
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if constexpr (is_rev<MODE>()) {
                    // the cos block of the epilogue before the next mid-slice wait has landed; reload epilogue S + W1_COS_LEAD's
                    constexpr int NEED = S + 1 + (W1_EPI_MEM < 4 ? 1 : 0);
                    if constexpr (NEED < NS) asm volatile("" : "+v"(st.cq[NEED % W1_COS_SLOTS]));
                    if constexpr (S + W1_COS_LEAD < NS) cos_issue<S + W1_COS_LEAD, LH, MODE>(st, cx);
                    if constexpr (S + 3 == NS) c0_issue<LH, MODE>(st, cx);  // retired by the next mid's vmcnt(0)
                    // the next tile's first W1_COS_LEAD cos blocks (every epilogue of this tile has run: the last one ran
                    // in slice NS - 2), behind this mid's wait and ahead of its ring issue: the tile start waits for the
                    // first of them with a counted vmcnt (no drain of the ring slices in flight)
                    if constexpr (S + 1 == NS) {
                        if (cx.more)
                            static_for<0, W1_COS_LEAD>(
                                [&](auto E) { cos_issue<decltype(E)::value, LH, MODE>(st, cx, cx.cnext); });
                    }
                }
                __builtin_amdgcn_s_barrier();
                if (S + 3 < NS || cx.more) {
                    const float* sp = cx.stream;
                    asm volatile("" : "+s"(sp));  // keep slice addresses from being hoisted into SGPRs
                    ring_issue4(sp, cx.ring, (S + 3) % NS, cx.wave, 16u * cx.lane);
                }
            }
        }
        f32x4 n0, n1;
        constexpr bool NEXT_IN_SLICE = p + 1 < NB / 2;
        constexpr bool NEXT_SLICE = !NEXT_IN_SLICE && S + 1 < NS;
        constexpr bool NEXT_TILE = !NEXT_IN_SLICE && S + 1 == NS;  // first pair of the next tile's slice 0
        static_assert(NS % W1_NBUF == 0, "the ring must wrap onto slot 0 at a tile boundary");
        bool next = NEXT_IN_SLICE || NEXT_SLICE;
        if constexpr (NEXT_IN_SLICE) {
            n0 = lds_read4<SLOT + (2 * p + 2) * 1024>(cx.ring_vaddr);
            n1 = lds_read4<SLOT + (2 * p + 3) * 1024>(cx.ring_vaddr);
        } else if constexpr (NEXT_SLICE) {
            n0 = lds_read4<NSLOT>(cx.ring_vaddr);
            n1 = lds_read4<NSLOT + 1024>(cx.ring_vaddr);
        }
        if constexpr (NEXT_IN_SLICE || NEXT_SLICE) {
            lgkm_wait<2>(a0, a1);
        } else if constexpr (NEXT_TILE) {
            // the next tile's first pair is read after this pair's MFMAs, read and wait in one statement (below)
            lgkm_wait<0>(a0, a1);
        } else {
            lgkm_wait<0>(a0, a1);
        }
        if constexpr (p == 0 && EPI) {
            // the epilogue parameters were issued before pair 1's reads: the wait above covered them
#pragma unroll
            for (int i = 0; i < epi_nparams<KIND>(); ++i) asm volatile("" : "+v"(ep.v[i]));
        }
        if constexpr (p == 0) w1_flush<S, LH, MODE>(st, cx);  // the wait above retired the transpose
        if constexpr (p == EPI_AT && EPI) {
            __builtin_amdgcn_sched_barrier(0);
            w1_epilogue<G, LH, MODE>(st, cx, KB + 1, ep);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            acc[2 * p] = mfma4(a0[r], bop[r], acc[2 * p]);
            acc[2 * p + 1] = mfma4(a1[r], bop[r], acc[2 * p + 1]);
        }
        if constexpr (NEXT_TILE) {
            if (cx.more) lds_read4x2_wait<NSLOT>(cx.ring_vaddr, a0, a1);
        } else if (next) {
            a0 = n0;
            a1 = n1;
        }
    });
    st.pa0 = a0;
    st.pa1 = a1;
    if constexpr (EPI && EPI_AT >= NB / 2) w1_epilogue<G, LH, MODE>(st, cx, KB + 1, ep);
}

template <int G, int LH, int MODE>
__device__ __forceinline__ void w1_gemm(W1State<LH, MODE>& st, const W1Ctx& cx) {
    constexpr int KIND = epi_kind<G, LH>();
    f32x4 (&acc)[NB] = st.acc[G & 1];
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) acc[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
        EpiParams<KIND, G, LH> ep;
        epi_load<KIND, G, LH>(ep, cx, 0);
        w1_epilogue<G, LH, MODE>(st, cx, 0, ep);
    }
    static_for<0, NB>([&](auto KB) { w1_slice<G, decltype(KB)::value, LH, MODE>(st, cx); });
}

__device__ __forceinline__ void prof_mark(const W1Ctx& cx, int ev) {
    const_cast<W1Ctx&>(cx).stamp[ev] = __builtin_amdgcn_s_memtime();
}

template <int G, int LH, int MODE>
__device__ __forceinline__ void w1_run(W1State<LH, MODE>& st, const W1Ctx& cx) {
    if constexpr (G < gemm0<MODE, LH>() + npasses<MODE>() * LH) {
        w1_gemm<G, LH, MODE>(st, cx);
        if constexpr ((MODE & MODE_PROF) != 0) prof_mark(cx, G + 1);
        w1_run<G + 1, LH, MODE>(st, cx);
    }
}

constexpr int small_floats_ct(int lh) { return SM_BIAS + (lh + 1) * H; }

// JET mode: 16 coordinates per workgroup (4 per wave); lap (n) receives sum_j Laplacian(y_j), gx (n, d) sum_j
// grad y_j (the quantities diff_operators.laplace / gradient return); abuf is reused as the lap pointer. JETS: the same
// outputs (lap in the last argument), abuf = a-jet tiles, dbuf = the reverse's z-jet scratch (jet_kernel.hpp layout).
template <int LH, int MODE>
__global__ __launch_bounds__(THREADS, forward_only(MODE & MODE_BASE) ? 2 : 1) void w1_kernel(const float* __restrict__ ws, const float* __restrict__ x,
                                                        int64_t n, const float* __restrict__ gy, float* __restrict__ y,
                                                        float* __restrict__ gx, int d, int o, float w0, float w,
                                                        float* __restrict__ abuf, float* __restrict__ dbuf,
                                                        int64_t n_pad, int64_t ws_bstride,
                                                        float* __restrict__ lap = nullptr) {
    constexpr bool STORE = (MODE & MODE_BASE) == MODE_STORE;
    constexpr bool JET = is_jet<MODE>();
    constexpr bool JETS = (MODE & MODE_BASE) == MODE_JETS;
    if constexpr (!JETS) lap = abuf;
    constexpr bool FWDS = (MODE & MODE_BASE) == MODE_FWDS;  // abuf = a_l tiles, dbuf = lane-major cos buffer
    constexpr bool REV = is_rev<MODE>();                     // abuf = lane-major cos buffer, dbuf = delta tiles
    constexpr int NS = npasses<MODE>() * LH * NB;
    constexpr int SMALL4 = (small_floats_ct(LH) + 3) / 4 * 4;
    __shared__ __attribute__((aligned(16))) float lds[W1_NBUF * SLICE + SMALL4 + (w1_staged<MODE>() ? WAVES * STB_SCRATCH : 0)];
    W1Ctx cx;
    W1State<LH, MODE> st;
    cx.ring = lds;
    float* sm = lds + W1_NBUF * SLICE;
    cx.sm = sm;
    cx.lane = threadIdx.x & 63;
    cx.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR address math
    cx.g = cx.lane >> 4;
    const int c = cx.lane & 15;
    if constexpr (mode_din(MODE) != 0) d = mode_din(MODE);
    if constexpr ((MODE & MODE_O1S) != 0) {
        o = 1;
        gy = nullptr;
    }
    cx.d = d;
    cx.o = o;
    // grouped launch over batched (hypernetwork) weights: block (x, element), renumbered XCD-major (xcd_remap) so each
    // XCD's 4 MiB L2 streams one or two elements' weights at a time instead of a slice of every element's
    int64_t bx = blockIdx.x;
    if (ws_bstride != 0) {
        unsigned rx, ry;
        xcd_remap(rx, ry);
        bx = rx;
        const int64_t b = ry;
        ws += b * ws_bstride;
        x += b * n * d;
        if (y != nullptr) y += b * n * o;
        if (gx != nullptr) gx += b * n * d;
        if (gy != nullptr) gy += b * n * o;
        if constexpr (STORE || FWDS || REV) {  // grouped W2: per-element a / delta tiles and lane-major cos
            abuf += b * (LH + 1) * n_pad * H;    // (each (LH + 1) n_pad H floats)
            dbuf += b * (LH + 1) * n_pad * H;
        }
    }
    {
        constexpr float two_pi = 6.28318530717958648f;
        const float s = w * 0.159154943091895336f;  // hidden-layer scale of the phase-scaled pack
        cx.w0 = w0 / s;
        cx.w = two_pi;
        cx.wsd = w;
        cx.inv_s0 = two_pi / w0;
    }
    cx.seed_ones = gy == nullptr;
    cx.abuf = cx.dbuf = nullptr;
    cx.ta = cx.td = cx.cs = nullptr;
    cx.more = false;
    cx.prof = nullptr;
    cx.stream = ws + small_pad(LH) + (REV ? (int64_t)LH * NB * SLICE : 0);
    cx.lstride = (JETS ? 4 : 1) * n_pad * H;  // jet tiles: 4 streams per coordinate
    const unsigned lds_base = (unsigned)(uintptr_t)((__attribute__((address_space(3))) float*)lds);
    cx.ring_vaddr = lds_base + cx.lane * 16;
    cx.sm_vaddr = lds_base + W1_NBUF * SLICE * 4 + 16 * cx.g;
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
    const int js = c & 3;  // JET stream of this lane
    // (JETS writes its tiles for all n_pad coordinates: the wgrad and the reverse read every column, padding included)
    const int64_t tiles = JETS ? n_pad / 16 : JET ? (n + 15) / 16 : (n + TILE - 1) / TILE;
    auto coord_of = [&](int64_t tile) -> int64_t {
        return JET ? tile * 16 + cx.wave * 4 + (c >> 2) : tile * TILE + cx.wave * 16 + c;
    };
    // this lane's inputs for a tile (prefetched one tile ahead so the loads never stall the MFMA stream)
    float xn[MAXD], gn[MAXO];
    auto load_inputs = [&](int64_t tile) {
        const int64_t cd = coord_of(tile);
        const bool ok = tile < tiles && cd < n;
        if constexpr (w1_asm_inputs<MODE>()) {
            // the next tile's inputs as asm loads into AGPRs ("+a": the zero of an idle lane and the loaded value
            // share one register, and hipcc has no reason to move an AGPR while it flies; into VGPRs it parked them in
            // AGPRs right after the issue, tools/check_asm_waits.py). A compiler load would be consumed at the next tile
            // start behind a compiler vmcnt(0) that drains the ring slices 0..2 already in flight; these are retired by
            // the tile's counted mid-slice waits long before (any vmcnt(4) two ring issues later)
#pragma unroll
            for (int k = 0; k < MAXD; ++k) xn[k] = 0.f;
#pragma unroll
            for (int j = 0; j < MAXO; ++j) gn[j] = 0.f;
            if (ok) {
                const float* xp = x + cd * d;
#pragma unroll
                for (int k = 0; k < MAXD; ++k)
                    if (k < d && !REV) asm volatile("global_load_dword %0, %1, off offset:%2" : "+a"(xn[k]) : "v"(xp), "i"(4 * k));
                if (gy != nullptr) {
                    const float* gp = gy + cd * o;
#pragma unroll
                    for (int j = 0; j < MAXO; ++j)
                        if (j < o) asm volatile("global_load_dword %0, %1, off offset:%2" : "+a"(gn[j]) : "v"(gp), "i"(4 * j));
                }
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < MAXD; ++k) xn[k] = (ok && k < d) ? x[cd * d + k] : 0.f;
#pragma unroll
        for (int j = 0; j < MAXO; ++j) gn[j] = (gy != nullptr && ok && j < o) ? gy[cd * o + j] : 0.f;
    };
    load_inputs(bx);
    if constexpr (w1_asm_inputs<MODE>()) {
        static_assert(MAXD == 4 && MAXO == 4, "one wait statement names every input register");
        asm volatile("s_waitcnt vmcnt(0)"
                     : "+a"(xn[0]), "+a"(xn[1]), "+a"(xn[2]), "+a"(xn[3]), "+a"(gn[0]), "+a"(gn[1]), "+a"(gn[2]), "+a"(gn[3])
                     :
                     : "memory");
    }
    if constexpr (JET) {
        // jet coefficients on phase-scaled jets: w / s = 2 pi for every layer (jet_sin_rev)
        const float val = js == 0 ? 1.f : 0.f;
        cx.jcb = val;
        cx.ja = val;
        cx.jb0 = cx.jb = js == 0 ? 0.f : 6.28318530717958648f;
        cx.jg0 = cx.jg = js == 3 ? 39.4784176043574344f : 0.f;
        // JETS scratch coefficients (jet_kernel.hpp PH): (w_l / s) (1, 2 pi, 4 pi^2) on streams (0, != 0, 3)
        constexpr float two_pi = 6.28318530717958648f, four_pi2 = 39.4784176043574344f;
        const float rw0 = w0 / (w * 0.159154943091895336f);
        cx.jdA0 = js == 0 ? rw0 : 0.f;
        cx.jdB0 = js == 0 ? 0.f : two_pi * rw0;
        cx.jdC0 = js == 3 ? four_pi2 * rw0 : 0.f;
        cx.jdA = js == 0 ? two_pi : 0.f;
        cx.jdB = js == 0 ? 0.f : four_pi2;
        cx.jdC = js == 3 ? two_pi * four_pi2 : 0.f;
    }
    __syncthreads();
    // ring prologue: slices 0..2 in flight; slice 0 published; its first operand pair read
    static_assert(NS >= 3, "ring prologue issues three slices");
    ring_issue4(cx.stream, cx.ring, 0, cx.wave, 16u * cx.lane);
    ring_issue4(cx.stream, cx.ring, 1, cx.wave, 16u * cx.lane);
    if constexpr (REV) {
        // the first tile's first cos blocks, in the position the next tiles' take (between ring slices 1 and 2): the
        // tile start then waits for them with one counted shape on every tile
        cx.cnext = (const char*)(abuf + cos_off(bx, cx.wave, LH, 0, 0, 0));
        if (bx < tiles) static_for<0, W1_COS_LEAD>([&](auto E) { cos_issue<decltype(E)::value, LH, MODE>(st, cx, cx.cnext); });
    }
    ring_issue4(cx.stream, cx.ring, 2, cx.wave, 16u * cx.lane);
    if constexpr (REV)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 + W1_COS_LEAD) : "memory");
    else
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    st.pa0 = lds_read4<0>(cx.ring_vaddr);
    st.pa1 = lds_read4<1024>(cx.ring_vaddr);

    // ---- coordinate tiles: a persistent grid walks tile = blockIdx.x, + gridDim.x, ... (a one-tile-per-
    // workgroup grid runs the loop once); the weight ring streams on across tile boundaries ----------------------
#pragma unroll 1
    for (int64_t tile = bx; tile < tiles; tile += gridDim.x) {
        if constexpr (REV) {
            // cos blocks of the first epilogues (SEED blocks 0 .. W1_COS_LEAD - 1), issued at the previous tile's last
            // mid-slice (the prologue for the first tile) ahead of ring slice 2: block 0 is needed now, blocks 1, 2 at
            // the next two mid-slice waits
            static_assert(W1_COS_LEAD == 3, "the tile-start count");
            asm volatile("s_waitcnt vmcnt(6)" : "+v"(st.cq[0]) : : "memory");
            cx.cbase = cx.cnext;
            cx.cnext = (const char*)(abuf + cos_off(tile + gridDim.x, cx.wave, LH, 0, 0, 0));
        }
        cx.more = tile + gridDim.x < tiles;
        const int64_t coord = coord_of(tile);
        const bool valid = coord < n;
#pragma unroll
        for (int k = 0; k < MAXD; ++k) st.xv[k] = xn[k];
#pragma unroll
        for (int j = 0; j < MAXO; ++j) {
            st.gyv[j] = gn[j];
            st.yp[j] = 0.f;
        }
        load_inputs(tile + gridDim.x);
        if constexpr (JET) {
#pragma unroll
            for (int k = 0; k < MAXD; ++k) cx.jcf[k] = cx.ja * st.xv[k] + (js == k + 1 ? 1.f : 0.f);
        }
        if constexpr (w1_tiles<MODE>()) {
            const int64_t tbase = (tile * WAVES + cx.wave) * (H * 16);  // wave-uniform
            const int64_t toff = tbase + 4 * cx.g * 16 + c;
            if constexpr (!REV) {
                cx.abuf = abuf + toff;
                cx.ta = (const char*)(abuf + tbase);
            }
            if constexpr (!FWDS && !JETS) {
                cx.dbuf = dbuf + toff;
                cx.td = (const char*)(dbuf + tbase);
            }
            if constexpr (JETS) cx.cs = (const char*)(dbuf + tbase);  // lane-major, + 16 lane
        }
        if constexpr (FWDS) cx.cs = (const char*)(dbuf + cos_off(tile, cx.wave, LH, 0, 0, 0));

        if constexpr ((MODE & MODE_PROF) != 0) {
            const int64_t it = (tile - bx) / gridDim.x;
            cx.prof = (blockIdx.x < PROF_BLOCKS && it < PROF_TILES)
                          ? (unsigned long long*)abuf + ((blockIdx.x * PROF_TILES + it) * WAVES + cx.wave) * PROF_EVENTS
                          : nullptr;
            prof_mark(cx, 0);
        }
        w1_run<gemm0<MODE, LH>(), LH, MODE>(st, cx);

        if constexpr (JET) {
            // last hidden layer's jet, output layer per stream, then y / grad / Laplacian from the quad's lanes
            constexpr int GL = (LH - 1) & 1;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const int nb = 16 * rb + 4 * cx.g;
                const f32x4 z = st.acc[GL][rb] + cx.jcb * *(const f32x4*)(sm + SM_BIAS + LH * H + nb);
                f32x4 a;
                if constexpr (JETS) {
                    f32x4 dz;
                    a = jet_sin_d_rev(z, cx.ja, cx.jb, cx.jg, cx.jdA, cx.jdB, cx.jdC, dz);
                    w3_store_tile(w3_at(cx.ta, w1_tile_off(cx, LH, rb)), cx.vt, a);
                    w3_store16(w3_at(cx.cs, w1_tile_off(cx, LH, rb)), cx.vl, dz);
                } else {
                    a = jet_sin_rev(z, cx.ja, cx.jb, cx.jg);
                }
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    if (j < o) {
                        const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + nb);
                        st.yp[j] += wj[0] * a[0] + wj[1] * a[1] + wj[2] * a[2] + wj[3] * a[3];
                    }
                }
            }
            float tot = 0.f;
#pragma unroll
            for (int j = 0; j < MAXO; ++j) {
                if (j < o) {
                    const float vj = sum_groups(st.yp[j]) + cx.jcb * sm[SM_BOUT + j];
                    if (y != nullptr && valid && cx.g == 0 && js == 0) y[coord * o + j] = vj;
                    tot += vj;
                }
            }
            if (valid && cx.g == 0) {
                if (js == 3) {
                    if (lap != nullptr) lap[coord] = tot;
                }
                else if (js >= 1 && js <= d && gx != nullptr) gx[coord * d + js - 1] = tot;
            }
        } else if constexpr ((MODE & MODE_BASE) == MODE_FWD || FWDS) {
            // last hidden layer: z_L = acc + b_L, a_L = sin(w z_L), y = a_L Wout^T + bout (serial epilogue)
            constexpr int GL = (LH - 1) & 1;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const int nb = 16 * rb + 4 * cx.g;
                const f32x4 z = st.acc[GL][rb] + *(const f32x4*)(sm + SM_BIAS + LH * H + nb);
                f32x4 sn, cs4;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float a, cc;
                    sincos_rev(z[r], a, cc);
                    sn[r] = a;
                    cs4[r] = cc;
                }
                if constexpr (FWDS) {
                    if constexpr (w1_tiles<MODE>()) store_block(cx.abuf + LH * cx.lstride, rb, sn);
                    w3_store16(w3_at(cx.cs, (LH * NB + rb) * 1024), cx.vl, cs4);
                }
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    if (j < o) {
                        const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + nb);
                        st.yp[j] += wj[0] * sn[0] + wj[1] * sn[1] + wj[2] * sn[2] + wj[3] * sn[3];
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < MAXO; ++j) {
                if (j < o) {
                    const float yj = sum_groups(st.yp[j]) + sm[SM_BOUT + j];
                    if (y != nullptr && valid && cx.g == 0) y[coord * o + j] = yj;
                }
            }
        } else {
            // y (reduced over the 4 lane groups)
#pragma unroll
            for (int j = 0; j < MAXO; ++j) {
                if (j < o) {
                    const float yj = sum_groups(st.yp[j]) + sm[SM_BOUT + j];
                    if (y != nullptr && valid && cx.g == 0) y[coord * o + j] = yj;
                }
            }
            // delta_0 = u_0 . cos(w0 z_0) . w0 (u_0 = s W_1^T delta_1 from the scaled pack: cx.w0 = w0 / s);
            // gx = delta_0 W0 (the LDS W0^T carries s0: cx.inv_s0)
            constexpr int GL = (2 * LH - 1) & 1;
            if constexpr (REV) {
#pragma unroll
                for (int rb = 0; rb < NB; ++rb) st.act[rb] = (st.acc[GL][rb] * st.c0q[rb]) * cx.w0;
            } else {
#pragma unroll
                for (int rb = 0; rb < NB; ++rb) st.act[rb] = (st.acc[GL][rb] * st.C[0][rb]) * cx.w0;
            }
            if constexpr (w1_tiles<MODE>()) store_tile(cx.dbuf, st.act);
#pragma unroll
            for (int k = 0; k < MAXD; ++k) {
                if (k < d) {
                    float q = 0.f;
#pragma unroll
                    for (int rb = 0; rb < NB; ++rb) {
                        const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * cx.g);
                        q += wk[0] * st.act[rb][0] + wk[1] * st.act[rb][1] + wk[2] * st.act[rb][2] +
                             wk[3] * st.act[rb][3];
                    }
                    q = sum_groups(q) * cx.inv_s0;
                    if (valid && cx.g == 0) gx[coord * d + k] = q;
                }
            }
        }
        if constexpr ((MODE & MODE_PROF) != 0) {
            prof_mark(cx, PROF_EVENTS - 1);
            if (cx.prof != nullptr && cx.lane == 0) {
#pragma unroll
                for (int e = 0; e < PROF_EVENTS; ++e) cx.prof[e] = cx.stamp[e];
            }
        }
    }
}

}  // namespace siren

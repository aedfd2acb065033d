// siren_common.h — shared constants and device helpers of the MI355X SIREN engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace siren {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------------------------------------
// Geometry of the fused H=256 kernels.
//   * MFMA v_mfma_f32_16x16x4_f32: A = weights (16 out-neurons x 4 in-neurons), B = activations
//     (4 in-neurons x 16 coordinates), C/D = 16 out-neurons x 16 coordinates.
//   * One wave owns 16 coordinates; its activation tile (256 neurons x 16 coords) is 16 blocks x f32x4 in
//     C/D layout: lane l = 16*g + c holds neuron 16*blk + 4*g + r of coordinate c in element r.
//     That C/D tile IS the B operand of the next layer's K-step (blk, r) — no data movement between layers.
//   * Weights stream through LDS in 16 KiB "slices": 16 K-neurons x 256 out-neurons, pre-packed by
//     siren_pack so that lane l's A operands for 4 consecutive K-steps are one ds_read_b128 at l*16 B.
// ---------------------------------------------------------------------------------------------------------
constexpr int H = 256;            // hidden width of the fused kernels
constexpr int NB = H / 16;        // neuron blocks per activation tile
constexpr int SLICE = 16 * H;     // floats per weight slice (16 KiB)
constexpr int NBUF = 3;           // LDS ring slots
constexpr int WAVES = 4;          // waves per workgroup (one per SIMD)
constexpr int THREADS = 64 * WAVES;
constexpr int TILE = 16 * WAVES;  // coordinates per workgroup
constexpr int MAXD = 4;           // max in_features of the fused kernels
constexpr int MAXO = 4;           // max out_features of the fused kernels
constexpr int MAX_LH_FWD = 8;     // max hidden layers of the forward-only kernel
constexpr int MAX_LH_GRAD = 3;    // max hidden layers of the forward+grad kernel (cos kept in VGPRs)
constexpr int MAX_LH_DEEP = 5;    // hidden 256, 4..5 hidden layers: derivatives through the stored split (cos to HBM)

// w1_kernel modes: W1 (forward + vjp_x), STORE (W2 backward stage 1: also writes a_l, delta_l), FWD (W0: forward
// only, sin epilogues without cos, output layer folded into a final serial epilogue).
// MODE_JET (W4): forward-mode Taylor jet for the Laplacian — 4 coordinates x 4 jet streams (value, d/dx_1,
// d/dx_2, sum_i d2/dx_i2) in the 16 MFMA columns, y / grad / Laplacian in one forward sweep.
// MODE_FWDS (W2 split, forward half): MODE_FWD + a_l tiles (wgrad layout) and cos(w z_l) (lane-major) to HBM, so
// the backward needs no forward recompute. MODE_REV (W2 split, backward half): the L reverse GEMMs only, cos read
// back from HBM, delta_l tiles stored like MODE_STORE.
// MODE_JETS (W4s split, forward half): MODE_JET + the a-jet tiles (wgrad layout, 4 n_pad H floats per layer) and the
// reverse's combinations of the z jet (jet_sin_d_rev, lane-major) for jet_store_kernel<JET_REV, PH>.
enum { MODE_W1 = 0, MODE_STORE = 1, MODE_FWD = 2, MODE_JET = 3, MODE_FWDS = 4, MODE_REV = 5, MODE_JETS = 6 };
// w1_kernel modifier bits (MODE & MODE_BASE is the mode proper): MODE_PROF records per-GEMM s_memtime stamps;
// MODE_O1S specialises d_out == 1 with the all-ones output cotangent (gy == NULL); MODE_D(k) fixes d_in = k at
// compile time. Both only remove runtime-uniform branches and selects from the epilogues (whose VALU count is the
// kernel's overhead, see sincos_fast).
// MODE_NOTILE: MODE_FWDS without the a_l tiles (lane-major cos only) / MODE_REV without the delta tiles (gx only), so
// the slice loops count the epilogues' vector-memory ops at compile time.
enum { MODE_BASE = 15, MODE_NOTILE = 32, MODE_PROF = 64, MODE_O1S = 128 };
constexpr int MODE_D(int k) { return k << 8; }
constexpr int mode_din(int mode) { return (mode >> 8) & 7; }
// MODE_PROF (diagnostics, siren_w1_phase_profile): s_memtime stamps at tile start, after each GEMM and at tile end
constexpr int PROF_TILES = 4, PROF_EVENTS = 8, PROF_BLOCKS = 256;
__host__ __device__ constexpr bool forward_only(int mode) {
    return mode == MODE_FWD || mode == MODE_JET || mode == MODE_FWDS || mode == MODE_JETS;
}
// lane-major cos(w z_l) buffer of MODE_FWDS / MODE_REV: per (tile, wave) (LH + 1) layers x NB blocks x 64 lanes x f32x4
// (one coalesced dwordx4 per lane per block): float offset of (tile, wave, layer, block, lane)
__host__ __device__ constexpr int64_t cos_off(int64_t tile, int wave, int lh, int l, int b, int lane) {
    return (((tile * WAVES + wave) * (lh + 1) + l) * NB + b) * 256 + lane * 4;
}

// Small-parameter block (head of the workspace, copied to LDS by every workgroup):
//   [SM_W0,  +4H)  W0T[k][n] = W_0[n][k]  (k < d_in, zero padded to 4 rows)
//   [SM_WO,  +4H)  WoT[j][n] = W_out[j][n] (j < d_out, zero padded)
//   [SM_SEED, +H)  seed[n]   = sum_j W_out[j][n]  (vjp seed for gy == ones)
//   [SM_BOUT, +4)  b_out
//   [SM_BIAS, +(LH+1)H) bias[l][n], l = 0 (first layer) .. LH (last hidden layer)
constexpr int SM_W0 = 0;
constexpr int SM_WO = 4 * H;
constexpr int SM_SEED = 8 * H;
constexpr int SM_BOUT = 9 * H;
constexpr int SM_BIAS = 9 * H + 4;
constexpr int SMALL_MAX = SM_BIAS + (MAX_LH_FWD + 1) * H;

__host__ __device__ inline int small_floats(int lh) { return SM_BIAS + (lh + 1) * H; }
__host__ __device__ inline int64_t small_pad(int lh) { return ((int64_t)small_floats(lh) + 1023) / 1024 * 1024; }

// The same block for a hidden width hw (the H = 512 kernels of wide_kernel.hpp): offsets scale with hw.
struct SmallLayout {
    int w0, wo, seed, bout, bias, h;
    __host__ __device__ explicit SmallLayout(int hw) : w0(0), wo(4 * hw), seed(8 * hw), bout(9 * hw),
                                                       bias(9 * hw + 4), h(hw) {}
    __host__ __device__ int floats(int lh) const { return bias + (lh + 1) * h; }
    __host__ __device__ int64_t pad(int lh) const { return ((int64_t)floats(lh) + 1023) / 1024 * 1024; }
};

// sin/cos of a fp32 phase t = w*z, to ~1 ulp of the true values (what torch.sin/torch.cos return on the
// reference's CPU path). Cody-Waite reduction by pi/2 with a 3-part constant (exact products for
// |quadrant| < 2^16), then minimax polynomials on [-pi/4, pi/4]. Phases beyond 1e5 rad (never produced
// by SIREN weights in practice) take the precise OCML path.
__device__ __forceinline__ void sincos_phase(float t, float& sn, float& cs) {
    if (__builtin_expect(__builtin_fabsf(t) > 1.0e5f, 0)) {
        sn = sinf(t);
        cs = cosf(t);
        return;
    }
    const float q = __builtin_rintf(t * 0.636619772367581343f);
    float r = __builtin_fmaf(-q, 1.5703125f, t);
    r = __builtin_fmaf(-q, 4.837512969970703125e-4f, r);
    r = __builtin_fmaf(-q, 7.54978995489188216e-8f, r);
    const float r2 = r * r;
    const float ps = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f), r2, -1.6666654611e-1f);
    const float sr = __builtin_fmaf(ps * r2, r, r);
    const float pc = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f), r2,
                                    4.166664568298827e-2f);
    const float cr = __builtin_fmaf(pc * r2, r2, __builtin_fmaf(-0.5f, r2, 1.0f));
    const int qi = (int)q;
    const float sv = (qi & 1) ? cr : sr;
    const float cv = (qi & 1) ? sr : cr;
    sn = (qi & 2) ? -sv : sv;
    cs = ((qi + 1) & 2) ? -cv : cv;
}

// One 1 KiB global->LDS piece (16 B per lane) in the saddr form: wave-uniform source base (SGPR pair) + the lane's
// 32-bit byte offset (VGPR) -> LDS at m0 (wave-uniform byte address). hipcc lowers __builtin_amdgcn_global_load_lds
// to a 64-bit VGPR address built with VALU for every piece; VALU issue is what the f32-MFMA kernels pay for (see
// sincos_fast below). Counted in vmcnt like any load; the kernels' ring protocols wait on it explicitly.
__device__ __forceinline__ void glds_x4(const void* sbase, unsigned lane_off, unsigned m0) {
    asm volatile("global_load_lds_dwordx4 %0, %1" ::"v"(lane_off), "s"(sbase), "{m0}"(m0) : "memory");
}
__device__ __forceinline__ unsigned lds_addr(const void* p) {
    return (unsigned)(uintptr_t)((__attribute__((address_space(3))) const void*)p);
}

// sin/cos for the MFMA kernels' epilogues, via the transcendental unit: Cody-Waite reduction of t by 2 pi
// (C1 = fp32(2 pi), C2 = 2 pi - C1; q*C1 is exact inside the fma, so r is accurate while q is exact), then
// v_sin_f32 / v_cos_f32 on revolutions in [-1/2, 1/2]. Branch-free, 5 VALU + 2 transcendental. Max abs error
// 3.7e-7 on |t| <= 100 (profiles/r01_vsin_accuracy.log; the earlier minimax-polynomial version: 1.1e-7 at ~30 VALU).
// Why the instruction count matters: an f32 MFMA (v_mfma_f32_16x16x4_f32) shares the SIMD's vector issue with
// VALU — a filler VALU is never hidden behind it (tools/micro/mfma_valu_overlap: the first costs ~14 cycles, each
// further ~4.5) — so every epilogue instruction is paid in full: W1 70.1% -> 76.4% of the fp32 MFMA peak.
// (Round 6 A/B: the reduction in revolutions, u = t / 2 pi rounded once and r = u - rint(u), is 3 VALU but 4.0e-6
// instead of 3.7e-7 on |t| <= 100 — the fp32 phase loses the bits its integer part takes — and at the first layer's
// w0 = 3000 (golden G2) it broke the 1e-4 third-order bar; tools/micro/sincos_accuracy.hip.)
__device__ __forceinline__ void sincos_fast(float t, float& sn, float& cs) {
    const float q = __builtin_rintf(t * 0.159154943091895336f);
    float r = __builtin_fmaf(-q, 6.28318548202514648f, t);
    r = __builtin_fmaf(-q, -1.74845553146951e-7f, r);
    const float u = r * 0.159154943091895336f;
    sn = __builtin_amdgcn_sinf(u);
    cs = __builtin_amdgcn_cosf(u);
}

// sin/cos of 2 pi u for a phase already in revolutions (w1_kernel's phase-scaled pack: weights and biases carry
// w / 2 pi, so the MFMA accumulators hold u = w z / 2 pi directly). r = u - rint(u) is exact, so the reduction costs
// 2 VALU instead of sincos_fast's 5; the argument's own rounding is one fp32 rounding of w z, like the reference's
// fl(30 z) (modules.py:34).
__device__ __forceinline__ void sincos_rev(float u, float& sn, float& cs) {
#ifndef SIREN_FRACT
#define SIREN_FRACT 0
#endif
#if SIREN_FRACT
    const float r = __builtin_amdgcn_fractf(u);  // one VALU; [0, 1) instead of [-1/2, 1/2]
#else
    const float r = u - __builtin_rintf(u);
#endif
    sn = __builtin_amdgcn_sinf(r);
    cs = __builtin_amdgcn_cosf(r);
}

// ---- forward-mode Taylor jets (MODE_JET, jet_kernel.hpp) ---------------------------------------------------
// A wave's 16 MFMA columns are 4 coordinates x 4 jet streams (column 4q + s): s = 0 value, s = 1, 2 the tangents
// d/dx_1, d/dx_2, s = 3 the second-order sum sum_i d2/dx_i2. A coordinate's streams sit in one DPP quad.
template <int SEL>
__device__ __forceinline__ float quad_bcast(float v) {  // value of quad lane SEL
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), SEL * 0x55, 0xf, 0xf, false));
}

// the jet of z (this lane's stream) -> the jet of sin(w z):
//   a = sin(w z0), a_i = w cos(w z0) z_i, a_3 = w cos(w z0) z_3 - w^2 sin(w z0) (z_1^2 + z_2^2)
// with per-lane coefficients ka = [s == 0], kb = w [s != 0], kg = w^2 [s == 3].
// MIX: the mixed second-order jet of two independent tangents (stream 1 along v, stream 2 along g, stream 3 the
// mixed second derivative D2[v, g]; the third-order adjoint of jet_kernel.hpp): a_3 = w cos z_3 - w^2 sin z_1 z_2.
template <bool MIX = false>
__device__ __forceinline__ f32x4 jet_sin(const f32x4& z, float w, float ka, float kb, float kg) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float z0 = quad_bcast<0>(z[r]), t1 = quad_bcast<1>(z[r]), t2 = quad_bcast<2>(z[r]);
        float sn, cs;
        sincos_fast(w * z0, sn, cs);
        const float q2 = MIX ? t1 * t2 : __builtin_fmaf(t1, t1, t2 * t2);
        out[r] = __builtin_fmaf(ka, sn, __builtin_fmaf(kb * cs, z[r], -(kg * sn) * q2));
    }
    return out;
}

// jet_sin on a phase-scaled jet (w1_kernel's revolution-domain pack: z is already w z / 2 pi on every stream, so
// kb = 2 pi [s != 0], kg = 4 pi^2 [s == 3] give the same a_i = w cos z_i and a_3 = w cos z_3 - w^2 sin |z_12|^2)
__device__ __forceinline__ f32x4 jet_sin_rev(const f32x4& z, float ka, float kb, float kg) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float z0 = quad_bcast<0>(z[r]), t1 = quad_bcast<1>(z[r]), t2 = quad_bcast<2>(z[r]);
        float sn, cs;
        sincos_rev(z0, sn, cs);
        const float q2 = __builtin_fmaf(t1, t1, t2 * t2);
        out[r] = __builtin_fmaf(ka, sn, __builtin_fmaf(kb * cs, z[r], -(kg * sn) * q2));
    }
    return out;
}

// Adjoint of jet_sin: given this lane's stream of the cotangent u of the output jet and of the input jet z,
// the cotangent of z (m0 = [s == 0], m12 = [s == 1 or 2]):
//   zb_3 = w c u_3
//   zb_i = w c u_i - 2 w^2 s z_i u_3
//   zb_0 = w c u_0 - w^2 s (u_1 z_1 + u_2 z_2) - u_3 (w^2 s z_3 + w^3 c (z_1^2 + z_2^2))
// MIX (a_3 = w c z_3 - w^2 s z_1 z_2): zb_1 = w c u_1 - w^2 s z_2 u_3, zb_2 = w c u_2 - w^2 s z_1 u_3 (s1 = [s == 1]
// picks the other tangent), zb_0's last term u_3 (w^2 s z_3 + w^3 c z_1 z_2).
template <bool MIX = false>
__device__ __forceinline__ f32x4 jet_sin_adjoint(const f32x4& u, const f32x4& z, float w, float m0, float m12,
                                                 bool s1 = false) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float z0 = quad_bcast<0>(z[r]), z1 = quad_bcast<1>(z[r]), z2 = quad_bcast<2>(z[r]);
        const float z3 = quad_bcast<3>(z[r]);
        const float u1 = quad_bcast<1>(u[r]), u2 = quad_bcast<2>(u[r]), u3 = quad_bcast<3>(u[r]);
        float sn, cs;
        sincos_fast(w * z0, sn, cs);
        const float wc = w * cs, w2s = w * w * sn;
        const float t12 = MIX ? w2s * ((s1 ? z2 : z1) * u3) : (2.f * w2s) * (z[r] * u3);
        const float q2 = MIX ? z1 * z2 : __builtin_fmaf(z1, z1, z2 * z2);
        const float t0 = __builtin_fmaf(w2s, __builtin_fmaf(u1, z1, u2 * z2),
                                        u3 * __builtin_fmaf(w2s, z3, (w * w * wc) * q2));
        out[r] = __builtin_fmaf(wc, u[r], -__builtin_fmaf(m12, t12, m0 * t0));
    }
    return out;
}

// The reverse needs each coordinate's jet of z only through four combinations, one per stream lane:
//   P = w c (lane 0),  R_i = w^2 s z_i (lanes 1, 2),  T = w^2 s z_3 + w^3 c (z_1^2 + z_2^2) (lane 3)
// so the forward stores those (jet_sin_d) in the z-jet scratch in place of z, and the reverse (jet_sin_adjoint_d) is
// linear in them: no sine, cosine or range reduction (the adjoint epilogue was 3.3 VALU per MFMA).
// Per-lane coefficients dA = w [s == 0], dB = w^2 [s != 0], dC = w^3 [s == 3]: D = dA c + dB s z + dC c (z_1^2 + z_2^2).
__device__ __forceinline__ f32x4 jet_sin_d(const f32x4& z, float w, float ka, float kb, float kg, float dA, float dB,
                                           float dC, f32x4& D) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float z0 = quad_bcast<0>(z[r]), t1 = quad_bcast<1>(z[r]), t2 = quad_bcast<2>(z[r]);
        float sn, cs;
        sincos_fast(w * z0, sn, cs);
        const float q2 = __builtin_fmaf(t1, t1, t2 * t2);
        out[r] = __builtin_fmaf(ka, sn, __builtin_fmaf(kb * cs, z[r], -(kg * sn) * q2));
        D[r] = __builtin_fmaf(dA, cs, __builtin_fmaf(dB * sn, z[r], (dC * cs) * q2));
    }
    return out;
}
// jet_sin_d on a phase-scaled jet (w1_kernel's revolution-domain pack, jet_sin_rev): sincos_rev of the value stream
// (2 reduction VALU instead of sincos_fast's 5 and the scale multiply), kb = 2 pi, kg = 4 pi^2 on every layer and the
// scratch combinations divided by the reverse GEMMs' scale s (jet_store_kernel PH)
__device__ __forceinline__ f32x4 jet_sin_d_rev(const f32x4& z, float ka, float kb, float kg, float dA, float dB,
                                               float dC, f32x4& D) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float z0 = quad_bcast<0>(z[r]), t1 = quad_bcast<1>(z[r]), t2 = quad_bcast<2>(z[r]);
        float sn, cs;
        sincos_rev(z0, sn, cs);
        const float q2 = __builtin_fmaf(t1, t1, t2 * t2);
        out[r] = __builtin_fmaf(ka, sn, __builtin_fmaf(kb * cs, z[r], -(kg * sn) * q2));
        D[r] = __builtin_fmaf(dA, cs, __builtin_fmaf(dB * sn, z[r], (dC * cs) * q2));
    }
    return out;
}
//   zb_3 = P u_3,  zb_i = P u_i - 2 R_i u_3,  zb_0 = P u_0 - (R_1 u_1 + R_2 u_2 + T u_3)      (m0 = [s == 0],
// m12 = [s == 1 or 2]; the same cotangent as jet_sin_adjoint<false>)
__device__ __forceinline__ f32x4 jet_sin_adjoint_d(const f32x4& u, const f32x4& D, float m0, float m12) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float P = quad_bcast<0>(D[r]), u3 = quad_bcast<3>(u[r]);
        const float e = D[r] * u[r];
        const float rest = quad_bcast<1>(e) + quad_bcast<2>(e) + quad_bcast<3>(e);
        out[r] = __builtin_fmaf(P, u[r], -__builtin_fmaf(m12, (2.f * D[r]) * u3, m0 * rest));
    }
    return out;
}

// QUAD (the backward of a Hessian node, Hm = sum_j u_j H_j (n, d, d), d <= 2): streams (value, d/dx_1, d/dx_2, second)
// with the second-order stream along the per-coordinate symmetric quadratic form Q = sym(cotangent of Hm). Lanes of
// streams 1 and 2 hold their row of 2 Q as (c1, c2): lin = c1 z1 + c2 z2 = (2 Q z)_i there, and the form comes from
// those two lanes, z^T Q z = (z1 lin_1 + z2 lin_2) / 2.
// forward (stream 3): a_3 = w c z_3 - w^2 s z^T Q z. The reverse needs z_3 and z^T Q z only in the combination
// K = w^2 s z_3 + w^3 c z^T Q z (zb_0's last term), so the stream-3 lane stores K in the z-jet scratch instead of z_3
// (kz): the reverse epilogue then computes no quadratic form (it sits at the 2-waves-per-SIMD register budget).
__device__ __forceinline__ f32x4 jet_sin_q(const f32x4& z, float w, float ka, float kb, float kg, float c1, float c2,
                                           bool s3, f32x4& kz) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float z0 = quad_bcast<0>(z[r]), t1 = quad_bcast<1>(z[r]), t2 = quad_bcast<2>(z[r]);
        const float lin = __builtin_fmaf(c1, t1, c2 * t2);
        const float q2 = 0.5f * __builtin_fmaf(t1, quad_bcast<1>(lin), t2 * quad_bcast<2>(lin));
        float sn, cs;
        sincos_fast(w * z0, sn, cs);
        out[r] = __builtin_fmaf(ka, sn, __builtin_fmaf(kb * cs, z[r], -(kg * sn) * q2));
        kz[r] = s3 ? __builtin_fmaf(kg * sn, z[r], (kg * w * cs) * q2) : z[r];
    }
    return out;
}
// its adjoint (z = the stored jet, stream 3 holding K): zb_3 = w c u_3, zb_i = w c u_i - w^2 s (2 Q z)_i u_3,
// zb_0 = w c u_0 - w^2 s (u_1 z_1 + u_2 z_2) - u_3 K
__device__ __forceinline__ f32x4 jet_sin_adjoint_q(const f32x4& u, const f32x4& z, float w, float m0, float m12,
                                                   float c1, float c2) {
    f32x4 out;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float z0 = quad_bcast<0>(z[r]), z1 = quad_bcast<1>(z[r]), z2 = quad_bcast<2>(z[r]);
        const float K = quad_bcast<3>(z[r]);
        const float u1 = quad_bcast<1>(u[r]), u2 = quad_bcast<2>(u[r]), u3 = quad_bcast<3>(u[r]);
        float sn, cs;
        sincos_fast(w * z0, sn, cs);
        const float wc = w * cs, w2s = w * w * sn;
        const float t12 = w2s * (__builtin_fmaf(c1, z1, c2 * z2) * u3);
        const float t0 = __builtin_fmaf(w2s, __builtin_fmaf(u1, z1, u2 * z2), u3 * K);
        out[r] = __builtin_fmaf(wc, u[r], -__builtin_fmaf(m12, t12, m0 * t0));
    }
    return out;
}

__device__ __forceinline__ float sin_phase(float t) {
    float s, c;
    sincos_phase(t, s, c);
    return s;
}

// Grouped launches over batched weights (grid.y = element): the hardware deals blocks round-robin over the 8 XCDs
// (blocks b and b + 8 share one; MI355X_MICROARCH.md, workgroup dispatch — observed placement, used for speed only),
// so the linear block id is renumbered XCD-major: the blocks of one XCD take consecutive (element, x) slots, an XCD
// works through its elements one or two at a time, and its 4 MiB L2 holds those elements' weight streams instead of
// a slice of every element's.
// XCD-major slot of linear block L in a grid of `total` blocks: XCD x holds blocks x, x + 8, ... (k + 1 of them for
// x < r, k otherwise, total = 8 k + r), and they take the consecutive slots prefix(x) + L / 8 — a bijection for any
// total (a group of consecutive slots straddles two XCDs only at the 8 XCD boundaries).
__device__ __forceinline__ unsigned xcd_slot(unsigned L, unsigned total) {
    const unsigned x = L % 8u, k = total / 8u, r = total % 8u;
    return x * k + (x < r ? x : r) + L / 8u;
}
__device__ __forceinline__ void xcd_remap(unsigned& bx, unsigned& by) {
    const unsigned gx = gridDim.x, total = gridDim.x * gridDim.y;
    const unsigned q = xcd_slot(blockIdx.x + blockIdx.y * gx, total);
    by = q / gx;
    bx = q % gx;
}

// Sum over the 4 lane groups g (lanes c, c+16, c+32, c+48 hold partial sums of one coordinate).
__device__ __forceinline__ float sum_groups(float v) {
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

// s * v + z with one rounding per element (an explicit fma chain: hipcc's contraction of a*b + c*d may fuse either
// product, which made two kernels with the same arithmetic differ in the last bit)
__device__ __forceinline__ f32x4 fma4(float s, const f32x4& v, const f32x4& z) {
    return f32x4{__builtin_fmaf(s, v[0], z[0]), __builtin_fmaf(s, v[1], z[1]), __builtin_fmaf(s, v[2], z[2]),
                 __builtin_fmaf(s, v[3], z[3])};
}

// q + w . v over the four elements as one explicit fma chain (the same rounding in every kernel that reduces a block
// this way: hipcc's contraction of the plain sum differs by context)
__device__ __forceinline__ float dot4_acc(const f32x4& w, const f32x4& v, float q) {
    return __builtin_fmaf(w[3], v[3], __builtin_fmaf(w[2], v[2], __builtin_fmaf(w[1], v[1], __builtin_fmaf(w[0], v[0], q))));
}

// A scalar operand as an opaque value. A context-struct field splat into an f32x4 product is otherwise widened by
// instcombine into a 16-byte load across the neighbouring fields; SROA then cannot split the struct, it stays in
// scratch, and its fields are reloaded from scratch (with a vmcnt wait) inside the MFMA loops (round 4: the W1
// seed epilogue, every w3i epilogue). Census: no private alloca in any kernel (`= alloca` in the device IR).
__device__ __forceinline__ float opaque(float v) {
    asm("" : "+v"(v));
    return v;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Global-memory views of generic pointers. A pointer stepped through an opaque register (asm "+v", to keep hipcc from
// hoisting one 64-bit address per block) loses its address space, and hipcc then emits FLAT loads / stores — which
// count in lgkmcnt as well as vmcnt, so every counted LDS-operand wait of the next MFMA slice also waited for the
// epilogue's stores to reach memory (and a counted lgkmcnt with FLAT ops outstanding is not a valid LDS wait).
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) f32x4 gf32x4_t;
__device__ __forceinline__ gfloat* gmem(float* p) { return (gfloat*)p; }
__device__ __forceinline__ const gf32x4_t* gmem4(const float* p) { return (const gf32x4_t*)p; }
__device__ __forceinline__ gf32x4_t* gmem4(float* p) { return (gf32x4_t*)p; }

// STORE-mode writers: element (neuron 16*rb + 4*g + r, coord c) of a 16-coordinate tile lives at
// neuron*16 + c, so lane (g, c) writes 4 floats 64 B apart per block; p already points at 4*g*16 + c (global memory).
// Stores of the tiles / kept jets / cos buffers a LATER kernel reads back carry the nontemporal hint (global_store ...
// nt): gigabytes per launch that no workgroup of the writing kernel re-reads, streamed past L2 instead of allocated in
// it, where the weight ring every CU re-reads lives. A/B (round 6, profile_paths kernel totals): qfi_rev_kernel<3>
// 4.96 -> 4.39 ms, w3i_kernel<3,1,1> 5.91 -> 5.51 ms, jets / split forward and reverse -1 %, the consumers (wgrad,
// edge) unchanged within 1 %; the wgrad's own operand loads with nt measured neutral-to-worse (+1 % video) and stay
// plain. SIREN_STORE_NT=0 restores plain stores (the A/B baseline).
#ifndef SIREN_STORE_NT
#define SIREN_STORE_NT 1
#endif
template <typename T, typename P>
__device__ __forceinline__ void st_tile(P* p, const T& v) {
    if constexpr (SIREN_STORE_NT != 0)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
__device__ __forceinline__ void store_block(float* p, int rb, const f32x4& v) {
    gfloat* q = gmem(p) + 16 * rb * 16;
    st_tile(q, v[0]);
    st_tile(q + 16, v[1]);
    st_tile(q + 32, v[2]);
    st_tile(q + 48, v[3]);
}
// The same block as ONE coalesced global_store_dwordx4 per lane (1 KiB per instruction instead of four scattered
// dword stores: epilogue store tails are store-ISSUE-bound, MI355X_MICROARCH.md), transposed through a per-wave LDS
// scratch of STB_SCRATCH floats (rows padded to 20 floats: conflict-free b32 writes, 16 B-aligned b128 reads). LDS
// operations of one wave execute in order, so back-to-back blocks may reuse the scratch. tile points at the
// wave's tile (no lane offset).
constexpr int STB_ROW = 20;
constexpr int STB_SCRATCH = 16 * STB_ROW;
__device__ __forceinline__ void store_block4(float* tile, int rb, const f32x4& v, float* scr, int lane) {
    const int g = lane >> 4, c = lane & 15;
#pragma unroll
    for (int r = 0; r < 4; ++r) scr[(4 * g + r) * STB_ROW + c] = v[r];
    const int n = lane >> 2, q = lane & 3;
    const f32x4 w = *(const f32x4*)(scr + n * STB_ROW + 4 * q);
    st_tile((f32x4*)(tile + rb * 256 + n * 16 + 4 * q), w);
}
__device__ __forceinline__ void store_tile(float* p, const f32x4 (&v)[NB]) {
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) store_block(p, rb, v[rb]);
}

}  // namespace siren

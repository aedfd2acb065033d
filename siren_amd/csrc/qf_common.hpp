#pragma once
// qf_common.hpp — the Hessian node's kept backward on the node's own layout (the reverse-only quadratic-form jet,
// laid out like the node's forward, hess_kernel.hpp, instead of the W4 jet's 4 coordinates x 4 streams per
// 16-column tile): the per-element arithmetic shared by qf_rev_kernel (qf_kernel.hpp) and qfi_rev_kernel
// (qfi_kernel.hpp, the interleaved schedule).
//
// Math (jet_kernel.hpp QG): with Q = sym(G) per coordinate and the kept pre-activation streams z, z_1, z_2, z_11, z_12,
// z_22 of layer l, the forward jet it differentiates is
//     a_0 = s,  a_i = w c z_i,  a_3 = w c z_3 - w^2 s z^T Q z,     z_3 = sum_ij Q_ij z_ij     (s, c = sin, cos(w z))
// and, for the cotangent u of the a-jet, the cotangent of the z-jet is
//     zb_3 = w c u_3,  zb_i = w c u_i - w^2 s (2 Q z)_i u_3,  zb_0 = w c u_0 - w^2 s (u_1 z_1 + u_2 z_2) - u_3 K,
//     K = w^2 s z_3 + w^3 c z^T Q z.
// The reverse GEMMs carry the 4 zb streams back through W_l^T; the a-jets of every layer and the zb-jets go to the
// MFMA wgrad (4 n columns) and the edge kernel (EDGE_Q8) for the parameter gradient.
//
// Layout ("Q8"): one wave owns 8 coordinates in TWO 16-column MFMA tiles that share every A operand (8 MFMAs per
// ds_read_b128): column c of tile 0 holds stream 0 (value) of coordinate c & 7 for c < 8 ("lo" lanes) and stream 1
// (d/dx_1) for c >= 8 ("hi"); tile 1 holds stream 2 (lo) and stream 3 (the Q stream, hi). The kept scratch has the
// same 8-coordinate lo / hi split (lo: z, z_2, z_12; hi: z_1, z_11, z_22), so one DPP row_ror:8 hands a lane its
// partner's value of a stream: per element 5 DPP moves (z, z_1 / z_2, the z_3 partial sum, two cotangents) produce
// two output streams, where the W4 jet layout spends 9 quad broadcasts per output stream (4.6 VALU per
// MFMA, 0.47 MFMA busy). Tiles in HBM: [layer][tile pair 2 grp, 2 grp + 1][neuron][16 columns] (4 n_pad columns
// per layer, n_pad a multiple of 32); the wgrad's bias takes the value columns (jet_bias 3: even tiles, columns < 8).
#include "hess_kernel.hpp"
#include "siren_common.h"

namespace siren {

// this lane's three kept streams of block rb (tiles 0..2 of hess_kept_off), one 16 B global load each
struct QfKept {
    f32x4 k[3];
};
__device__ __forceinline__ QfKept qf_load(const float* p) {
    typedef const __attribute__((address_space(1))) f32x4 gf32x4;
    QfKept r;
    r.k[0] = *(gf32x4*)p;
    r.k[1] = *(gf32x4*)(p + 256);
    r.k[2] = *(gf32x4*)(p + 512);
    return r;
}

__device__ __forceinline__ void qf_store_block(float* p, const f32x4& v) { store_block(p, 0, v); }

// layer 0's jet of block rb, rebuilt from the coordinate exactly as hess_kernel computes it (it is not kept):
// lo lanes (z, z_2, z_12) = (W0 x + b0, W0[:, 1], 0), hi lanes (z_1, z_11, z_22) = (W0[:, 0], 0, 0)
__device__ __forceinline__ QfKept qf_layer0(const float* sm, int rb, int g, bool hi, float x0, float x1) {
    const int nb = 16 * rb + 4 * g;
    const f32x4 wa = *(const f32x4*)(sm + SM_W0 + nb);
    const f32x4 wb = *(const f32x4*)(sm + SM_W0 + H + nb);  // zero padded row when d == 1
    const f32x4 zv = layer0_z(*(const f32x4*)(sm + SM_BIAS + nb), wa, wb, x0, x1);
    const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    QfKept r;
    r.k[0] = hi ? wa : zv;
    r.k[1] = hi ? zero : wb;
    r.k[2] = zero;
    return r;
}

// per-coordinate coefficients of the quadratic form (lane constants): q11 = G_11, q12 = G_12 + G_21, q22 = G_22
struct QfCoef {
    float q11, q12, q22;
    float e1, e2;  // own z_3 partial: lo e2 z_12 (e1 = 0), hi e1 z_11 + e2 z_22
    float ca, cb;  // own (2 Q z) row: lo (2 Q z)_2 = q12 z_1 + 2 q22 z_2, hi (2 Q z)_1 = 2 q11 z_1 + q12 z_2
    float mlo;     // 1 on lo lanes, 0 on hi lanes (zb's t3 term as an fma addend instead of a select)
};

// sin / cos of w z for the kept reverse's hidden layers: the phase u = z (w / 2 pi) in revolutions, then sincos_rev
// (3 VALU + 2 transcendental against sincos_fast's 6 + 2 with the w z product; qf_elem runs ~50 VALU per element at
// one wave per SIMD, where the VALU shares the issue with the f32 MFMAs). The phase is one fp32 rounding of w z / 2 pi,
// the accuracy class of the phase-scaled W1 family; layer 0 (qf_elem0) keeps sincos_fast: its w0 is arbitrary (3000 in
// golden G2), and an fp32 phase of thousands of revolutions keeps too few fraction bits. A/B (r06g): qfi_rev_kernel<3>
// 5.05 -> 4.96 ms per Poisson-recipe step (static VALU 12970 -> 12028 with the select-free zb below).
__device__ __forceinline__ void qf_sincos(float z, float wl, float& sn, float& cs) {
    sincos_rev(z * (wl * 0.159154943091895336f), sn, cs);
}

// one layer's epilogue for one element (row r of block rb): kept streams k0..k2, cotangents ua (tile 0), ub (tile 1)
// -> a-jet (aa, ab) and z-jet cotangent (za, zb) of this lane's two streams
// (phase: the hidden layers' qf_sincos; false for layer 0, whose w0 is arbitrary — the serial kernel runs layer 0
// through here, the interleaved one through qf_elem0, and both must round alike)
__device__ __forceinline__ void qf_elem(float k0, float k1, float k2, float ua, float ub, float wl, float wl2,
                                        const QfCoef& q, bool hi, float& aa, float& ab, float& za, float& zb,
                                        bool phase = true) {
    const float p0 = row_ror8(k0), p1 = row_ror8(k1);
    const float zp = __builtin_fmaf(q.e1, k1, q.e2 * k2);
    const float z3 = zp + row_ror8(zp);
    const float pa = row_ror8(ua), pb = row_ror8(ub);
    const float z = hi ? p0 : k0;
    const float z1 = hi ? k0 : p0;
    const float z2 = hi ? p1 : k1;
    float sn, cs;
    if (phase)
        qf_sincos(z, wl, sn, cs);
    else
        sincos_fast(wl * z, sn, cs);
    const float wc = wl * cs, w2s = wl2 * sn;
    const float qz = __builtin_fmaf(z1, __builtin_fmaf(q.q11, z1, q.q12 * z2), (q.q22 * z2) * z2);  // z^T Q z
    const float lin = __builtin_fmaf(q.ca, z1, q.cb * z2);                                       // (2 Q z)_own
    const float u3 = hi ? ub : pb;
    aa = hi ? wc * z1 : sn;                                       // a_1 | a_0
    ab = hi ? __builtin_fmaf(wc, z3, -w2s * qz) : wc * z2;        // a_3 | a_2
    const float t3 = w2s * (lin * u3);                            // w^2 s (2 Q z)_i u_3
    zb = __builtin_fmaf(wc, ub, -(t3 * q.mlo));                   // zb_3 | zb_2 (hi: fma with -0 = the product)
    const float K = __builtin_fmaf(w2s, z3, (wl2 * wc) * qz);     // w^2 s z_3 + w^3 c z^T Q z
    const float t0 = __builtin_fmaf(w2s, __builtin_fmaf(pa, z1, ub * z2), u3 * K);
    za = __builtin_fmaf(wc, ua, -(hi ? t3 : t0));                 // zb_1 | zb_0
}

// qf_elem for layer 0, whose jet every lane can form itself (qf_layer0's values, no partner exchange): z = W0 x + b0,
// z_i = W0[:, i], z_ij = 0 — so z_3 = 0 and K = w^3 c z^T Q z. Same arithmetic as qf_elem on those values (every
// product with the zero streams dropped), hence bitwise the same results.
__device__ __forceinline__ void qf_elem0(float z, float z1, float z2, float ua, float ub, float wl, float wl2,
                                         const QfCoef& q, bool hi, float& aa, float& ab, float& za, float& zb) {
    const float pa = row_ror8(ua), pb = row_ror8(ub);
    float sn, cs;
    sincos_fast(wl * z, sn, cs);
    const float wc = wl * cs, w2s = wl2 * sn;
    const float qz = __builtin_fmaf(z1, __builtin_fmaf(q.q11, z1, q.q12 * z2), (q.q22 * z2) * z2);  // z^T Q z
    const float lin = __builtin_fmaf(q.ca, z1, q.cb * z2);                                       // (2 Q z)_own
    const float u3 = hi ? ub : pb;
    aa = hi ? wc * z1 : sn;                                       // a_1 | a_0
    ab = hi ? __builtin_fmaf(wc, 0.f, -w2s * qz) : wc * z2;       // a_3 | a_2   (z_3 = 0)
    const float t3 = w2s * (lin * u3);
    zb = __builtin_fmaf(wc, ub, -(t3 * q.mlo));                   // zb_3 | zb_2
    const float K = __builtin_fmaf(w2s, 0.f, (wl2 * wc) * qz);
    const float t0 = __builtin_fmaf(w2s, __builtin_fmaf(pa, z1, ub * z2), u3 * K);
    za = __builtin_fmaf(wc, ua, -(hi ? t3 : t0));                 // zb_1 | zb_0
}

}  // namespace siren

#pragma once
// hess_kernel.hpp — the forward of the Hessian node (SirenHessian, autograd.py): Hm = sum_j u_j H_j(x) (n, d, d),
// d <= 2, in ONE forward-mode sweep (no reverse pass).
//
// Every divergence() / hessian() column the reference takes of one gradient node (diff_operators.py:5-36; the
// Poisson recipe laplace = divergence(gradient(y, x), x), loss_functions.py:104-109) differentiates the same
// J = dy/dx, so the node returns the whole per-coordinate Hessian. It is the second-order Taylor jet of the network
// along the coordinate axes: per layer the pre-activation streams
//     z,  dz/dx_1,  dz/dx_2,  d2z/dx_1^2,  d2z/dx_1 dx_2,  d2z/dx_2^2                       (6 streams)
// all pass through W_l (bias on z only), and the sine maps them elementwise (a = sin(w z), c = cos, s = sin):
//     a_i = w c z_i,    a_ij = w c z_ij - w^2 s z_i z_j
// Hm_ij = sum_j' u_j' Wout_j' . a_ij of the last hidden layer.
// Against the previous forward (one W3 reverse-over-forward launch per axis: 2 forward + 2 reverse streams each, i.e.
// 8 column-GEMMs per coordinate and layer for d = 2) this is 6, with no reverse sweep and no spill traffic.
//
// MFMA layout: one wave owns 8 coordinates in THREE 16-column tiles (48 columns = 8 coordinates x 6 streams) that
// share every A operand (12 MFMAs per ds_read, lds_ops.h slice_mma3_mid). Column c of a tile holds coordinate c & 7;
// lanes c < 8 ("lo") carry (z, dz/dx_2, d2z/dx_1dx_2) in tiles (0, 1, 2), lanes c >= 8 ("hi") carry (dz/dx_1,
// d2z/dx_1^2, d2z/dx_2^2). Partner columns c ^ 8 sit in the same 16-lane row, so one DPP row_ror:8 per tile hands
// each lane the other three streams of its coordinate (hess_sin).
//
// KEEP: the pre-activation jets of every layer (bias included) go to a lane-major scratch, kept by the node for its
// backward: the quadratic-form jet (jet_kernel.hpp QG, KEPT) then reads its forward from it instead of recomputing
// the forward GEMMs (its second-order stream along Q is the linear combination sum_ij Q_ij d2z/dx_i dx_j).
// Layout (hess_kept_off): [layer l - 1][8-coordinate group][block rb][tile t][lane] f32x4 for layers l = 1 .. L —
// each wave's stores are 1 KiB contiguous. Layer 0's jet (z = W0 x + b0, z_i = W0[:, i], z_ij = 0) is not kept: the
// backward rebuilds it from x (qf_layer0), which saves a quarter of the kept traffic at L = 3 (round 4).
#include "lds_ops.h"
#include "ring.hpp"
#include "siren_common.h"

namespace siren {

// 8-coordinate groups of a Hessian sweep over n coordinates (workgroups of 32)
__host__ __device__ constexpr int64_t hess_groups(int64_t n) { return (n + 31) / 32 * 4; }
// float offset of (layer l >= 1, group grp, block rb, tile t, lane) in the kept scratch, and the stride between layers
// (a group-major order, each workgroup's jets of all layers contiguous, measured the same: 5.32 vs 5.31 ms forward)
__host__ __device__ constexpr int64_t hess_kept_off(int64_t ngroups, int lh, int l, int64_t grp, int rb, int t,
                                                    int lane) {
    return ((((int64_t)(l - 1) * ngroups + grp) * NB + rb) * 3 + t) * 256 + lane * 4;
}
__host__ __device__ constexpr int64_t hess_kept_lstride(int64_t ngroups) { return ngroups * NB * 3 * 256; }

// this lane's index, recomputed at each use (exec must be full there): an asm without inputs is neither hoisted nor
// merged, so the lane-derived LDS / global addresses of the epilogues (bias and Wout rows, kept pointer, coordinate)
// are rebuilt in two VALU ops instead of living across the layer loop — at 512 registers they were the spills, each
// reload a vmcnt(0) that also drained the weight ring's in-flight slices
__device__ __forceinline__ int lane_here() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// layer 0's pre-activation z = b0 + x_0 W0[:, 0] + x_1 W0[:, 1] as one explicit fma chain: the Hessian node's forward
// and every backward that rebuilds layer 0 from x (qf_common.hpp) must round it identically (hipcc's contraction of
// the plain expression differs by context)
__device__ __forceinline__ f32x4 layer0_z(const f32x4& b, const f32x4& wa, const f32x4& wb, float x0, float x1) {
    return fma4(x1, wb, fma4(x0, wa, b));
}

__device__ __forceinline__ float row_ror8(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xf, 0xf, false));
}

// the three streams of this lane (t0, t1, t2 in tiles 0, 1, 2) of the pre-activation jet -> those of a = sin(w z)
__device__ __forceinline__ void hess_sin(const f32x4& t0, const f32x4& t1, const f32x4& t2, float w, bool hi,
                                         f32x4& o0, f32x4& o1, f32x4& o2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float p0 = row_ror8(t0[r]), p1 = row_ror8(t1[r]);
        const float z = hi ? p0 : t0[r];
        const float z1 = hi ? t0[r] : p0;
        const float z2 = hi ? p1 : t1[r];
        float sn, cs;
        sincos_fast(w * z, sn, cs);
        const float wc = w * cs, w2s = w * w * sn;
        o0[r] = hi ? wc * t0[r] : sn;                                         // a | a_1
        o1[r] = __builtin_fmaf(wc, t1[r], hi ? -(w2s * z1) * z1 : 0.f);       // a_2 | a_11
        o2[r] = __builtin_fmaf(wc, t2[r], -(w2s * z2) * (hi ? z2 : z1));      // a_12 | a_22
    }
}

template <bool KEEP>
__global__ __launch_bounds__(THREADS, 1) void hess_kernel(const float* __restrict__ ws, const float* __restrict__ x,
                                                          int64_t n, const float* __restrict__ u, int d, int o,
                                                          int lh, float w0, float w, float* __restrict__ hm,
                                                          float* __restrict__ kept, float* __restrict__ yo,
                                                          float* __restrict__ gxo) {
    __shared__ __attribute__((aligned(16))) float lds[NBUF * SLICE + SMALL_MAX];
    float* ring = lds;
    float* sm = lds + NBUF * SLICE;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR): never a spilled VGPR
    const int g = lane >> 4, c = lane & 15;
    const bool hi = c >= 8;
    const int nslices = lh * NB;
    const float* stream = ws + small_pad(lh);
    {
        const int nf4 = (small_floats(lh) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t ngroups = hess_groups(n);
    const int64_t grp = (int64_t)blockIdx.x * WAVES + wave;
    const int64_t coord = grp * 8 + (c & 7);
    const bool valid = coord < n;
    const float x0 = valid ? x[coord * d] : 0.f;
    const float x1 = (valid && d > 1) ? x[coord * d + 1] : 0.f;
    __syncthreads();
    int s = 0;
    ring_issue(stream, ring, 0, nslices, wave, lane);
    ring_issue(stream, ring, 1, nslices, wave, lane);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // slice 0 landed: publish it (later ones: mid-slice barriers)
    __builtin_amdgcn_s_barrier();

    f32x4 act[3][NB], acc[3][NB];
    // ---- layer 0 (VALU, K = d_in): z = W0 x + b0, z_i = W0[:, i], second order 0 -------------------------------
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        const int nb = 16 * rb + 4 * g;
        const f32x4 wa = *(const f32x4*)(sm + SM_W0 + nb);
        const f32x4 wb = *(const f32x4*)(sm + SM_W0 + H + nb);  // zero padded row when d == 1
        const f32x4 zv = layer0_z(*(const f32x4*)(sm + SM_BIAS + nb), wa, wb, x0, x1);
        const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
        const f32x4 t0 = hi ? wa : zv, t1 = hi ? zero : wb;  // (not kept: qf_layer0 rebuilds it)
        hess_sin(t0, t1, zero, w0, hi, act[0][rb], act[1][rb], act[2][rb]);
    }

#pragma unroll 1
    for (int l = 1; l <= lh; ++l) {
#pragma unroll
        for (int ob = 0; ob < NB; ++ob) acc[0][ob] = acc[1][ob] = acc[2][ob] = f32x4{0.f, 0.f, 0.f, 0.f};
        {
            const unsigned rbase = lds_addr(ring) + 16u * lane;
            f32x4 a = lds_read4<0>(rbase + (s % NBUF) * SLICE * 4);
#pragma unroll
            for (int kb = 0; kb < NB; ++kb) {
                const unsigned va = rbase + (s % NBUF) * SLICE * 4, vn = rbase + ((s + 1) % NBUF) * SLICE * 4;
                auto mid = [&]() { ring_mid(stream, ring, s, nslices, wave, lane); };
                if (kb + 1 < NB)
                    slice_mma3_mid<NB, NB / 2, true>(va, vn, act[0][kb], act[1][kb], act[2][kb], acc, a, a, mid);
                else
                    slice_mma3_mid<NB, NB / 2, false>(va, vn, act[0][kb], act[1][kb], act[2][kb], acc, a, a, mid);
                ++s;
            }
        }
        const int le = lane_here();
        const float* bl = sm + SM_BIAS + l * H + 4 * (le >> 4);
#pragma unroll
        for (int rb = 0; rb < NB; ++rb) {
            const f32x4 t0 = hi ? acc[0][rb] : acc[0][rb] + *(const f32x4*)(bl + 16 * rb);
            if constexpr (KEEP) {
                float* kpl = kept + hess_kept_off(ngroups, lh, l, grp, 0, 0, le);
                st_tile((f32x4*)(kpl + rb * 768), t0);
                st_tile((f32x4*)(kpl + rb * 768 + 256), acc[1][rb]);
                st_tile((f32x4*)(kpl + rb * 768 + 512), acc[2][rb]);
            }
            hess_sin(t0, acc[1][rb], acc[2][rb], w, hi, act[0][rb], act[1][rb], act[2][rb]);
        }
    }

    // ---- Hm = Wout-weighted last jet: seed sum_j u_j Wout_j (u == NULL: sum_j Wout_j) ---------------------------
    // (yo / gxo nullable: y_j = Wout_j . a_L + bout_j and the seed-weighted gradient sum_j u_j dPhi_j/dx from the
    // same last jet — the value / first-order streams — so a caller that needs (y, dPhi/dx, Hm) runs ONE sweep)
    const int lf = lane_here();
    const int gf = lf >> 4;
    const int64_t cf = grp * 8 + (lf & 7);
    const bool vf = cf < n;
    float uw[MAXO];
#pragma unroll
    for (int j = 0; j < MAXO; ++j) uw[j] = (u != nullptr && j < o && vf) ? u[cf * o + j] : 0.f;
    float p0 = 0.f, p1 = 0.f, p2 = 0.f;
    float yv[MAXO] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        f32x4 sd;
        if (u != nullptr) {  // WoT rows j >= o are zero padded
            const float* wo = sm + SM_WO + 16 * rb + 4 * gf;
            sd = uw[0] * *(const f32x4*)wo + uw[1] * *(const f32x4*)(wo + H) + uw[2] * *(const f32x4*)(wo + 2 * H) +
                 uw[3] * *(const f32x4*)(wo + 3 * H);
        } else {
            sd = *(const f32x4*)(sm + SM_SEED + 16 * rb + 4 * gf);
        }
        p1 += sd[0] * act[1][rb][0] + sd[1] * act[1][rb][1] + sd[2] * act[1][rb][2] + sd[3] * act[1][rb][3];
        p2 += sd[0] * act[2][rb][0] + sd[1] * act[2][rb][1] + sd[2] * act[2][rb][2] + sd[3] * act[2][rb][3];
        if (gxo != nullptr)
            p0 += sd[0] * act[0][rb][0] + sd[1] * act[0][rb][1] + sd[2] * act[0][rb][2] + sd[3] * act[0][rb][3];
        if (yo != nullptr) {
#pragma unroll
            for (int j = 0; j < MAXO; ++j) {
                if (j < o) {  // wave-uniform
                    const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + 16 * rb + 4 * gf);
                    yv[j] += wj[0] * act[0][rb][0] + wj[1] * act[0][rb][1] + wj[2] * act[0][rb][2] +
                             wj[3] * act[0][rb][3];
                }
            }
        }
    }
    p1 = sum_groups(p1);  // lo: u . dy/dx_2 | hi: H_11
    p2 = sum_groups(p2);  // lo: H_12 | hi: H_22
    if (gxo != nullptr) p0 = sum_groups(p0);  // lo: (u . (y - bout), unused) | hi: u . dy/dx_1
    if (yo != nullptr) {
#pragma unroll
        for (int j = 0; j < MAXO; ++j)
            if (j < o) yv[j] = sum_groups(yv[j]);  // lo: Wout_j . a_L
    }
    if (vf && gf == 0) {
        if (gxo != nullptr) {
            if (hi)
                gxo[cf * d] = p0;
            else if (d > 1)
                gxo[cf * d + 1] = p1;
        }
        if (yo != nullptr && !hi) {
#pragma unroll
            for (int j = 0; j < MAXO; ++j)
                if (j < o) yo[cf * o + j] = yv[j] + sm[SM_BOUT + j];
        }
        if (d == 1) {
            if (hi) hm[cf] = p1;
        } else if (hi) {
            hm[cf * 4] = p1;
            hm[cf * 4 + 3] = p2;
        } else {
            hm[cf * 4 + 1] = p2;
            hm[cf * 4 + 2] = p2;
        }
    }
}

}  // namespace siren

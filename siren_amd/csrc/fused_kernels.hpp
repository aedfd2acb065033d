#pragma once
// fused_kernels.hpp — fused SIREN forward (W0) and forward + coordinate-gradient (W1) kernels for gfx950.
//
// Replaces the reference's per-layer ATen chain (modules.py:23 matmul, :24 bias add_, :34 mul+sin) and the
// autograd reverse sweep that diff_operators.gradient (diff_operators.py:39-43) records, with one launch:
//   forward : a_0 = sin(w0 (x W0^T + b0))          first layer on VALU (K = d_in <= 4)
//             a_l = sin(w (a_{l-1} W_l^T + b_l))   hidden layers on v_mfma_f32_16x16x4_f32 (exact fp32)
//             y   = a_L Wout^T + bout              VALU dot + cross-lane reduction
//   reverse : delta_L = (gy Wout) . cos(w z_L) . w,  delta_{l-1} = (delta_l W_l) . cos(w z_{l-1}) . w,
//             gx = delta_0 W0                       (same MFMA tiles with W^T slices)
// Activations, cos(w z_l) of every layer and the reverse-sweep deltas never leave VGPRs: the only HBM
// traffic per coordinate is x (d*4 B), y (o*4 B) and gx (d*4 B); weights stream from L2 through a 3-slot
// LDS ring filled by global_load_lds_dwordx4.
#include "siren_common.h"
#include "siren_params.h"
#include "ring.hpp"

namespace siren {

// ------------------------------------------------------------------------------------------------------
// Pack kernel: flat params -> [small block | forward slices | transposed slices].
//   forward slice (layer l, K-block kb), element ((ob*4 + g)*16 + i)*4 + r = W_l[16ob + i][16kb + 4g + r]
//   reverse slice (layer l, K-block kb), element ((ib*4 + g)*16 + i)*4 + r = W_l[16kb + 4g + r][16ib + i]
// Forward slices are stored for l = 1..LH, reverse slices for l = LH..1: exactly the order the fused
// kernel consumes them, so its ring loader walks the workspace linearly.
// ------------------------------------------------------------------------------------------------------
// With base > 0 (hidden 256) a second, phase-scaled copy follows at ws + base for w1_kernel: W0^T and b0 times
// s0 = w0 / 2 pi, hidden-layer slices and biases times s = w / 2 pi (W_out, b_out and the seed unscaled), so that
// kernel's accumulators are phases in revolutions (sincos_rev) and its reverse GEMMs return s W^T delta.
__global__ void pack_kernel(const float* __restrict__ p, float* __restrict__ ws, int d, int o, int lh,
                            int64_t spad, int64_t total, int h, int64_t base, float s0, float s,
                            int64_t p_bstride, int64_t begin) {
    // grouped over batched weights (grid.y = batch element): params rows of p_bstride, workspaces of total floats;
    // elements [begin, total) of each workspace are written (the batched pack skips the unscaled copy)
    p += (int64_t)blockIdx.y * p_bstride;
    ws += (int64_t)blockIdx.y * total;
    // h = hidden width (256: the H kernels, 512: wide_kernel.hpp); a slice is 16 K-rows x h out-neurons. All
    // per-element index math is 32-bit shifts and masks (h is a power of two; one workspace < 2^31 floats): the
    // 64-bit divisions of the first version made the batched pack instruction-bound (98 us for 32 x 3.2 MB)
    const ParamOffsets off(d, o, lh, h);
    const SmallLayout sl(h);
    const int nb = h / 16;
    const int lsf = 4 + __builtin_ctz((unsigned)h);  // log2(slice floats)
    const unsigned sfm = (1u << lsf) - 1u;
    const unsigned hm = (unsigned)h - 1u, lh2 = (unsigned)__builtin_ctz((unsigned)h);
    // one thread per 4 consecutive workspace floats (one 16 B store; region boundaries of the small block are multiples
    // of 4): a slice quad is 4 consecutive floats of one W row (forward) or one float of 4 rows (transposed), so the
    // index math runs once per quad (the per-float version was instruction-bound: 49 us for 32 x 1.6 MB)
    const int64_t qend = total >> 2;
    for (int64_t qi = (begin >> 2) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; qi < qend;
         qi += (int64_t)gridDim.x * blockDim.x) {
        const int64_t gidx = qi << 2;
        const bool scaled = base > 0 && gidx >= base;
        const unsigned idx = (unsigned)(scaled ? gidx - base : gidx);
        f32x4 v4 = {0.f, 0.f, 0.f, 0.f};
        float sc = 1.f;
        if (idx < (unsigned)spad) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int e = (int)idx + q;
                float v = 0.f;
                if (e < sl.wo) {
                    const int k = e >> lh2, n = e & hm;
                    v = k < d ? p[off.w0 + (int64_t)n * d + k] : 0.f;
                    sc = s0;
                } else if (e < sl.seed) {
                    const int j = (e - sl.wo) >> lh2, n = (e - sl.wo) & hm;
                    v = j < o ? p[off.wout + (int64_t)j * h + n] : 0.f;
                } else if (e < sl.bout) {
                    const int n = e - sl.seed;
                    float acc = 0.f;
                    for (int j = 0; j < o; ++j) acc += p[off.wout + (int64_t)j * h + n];
                    v = acc;
                } else if (e < sl.bias) {
                    const int j = e - sl.bout;
                    v = j < o ? p[off.bout + j] : 0.f;
                } else if (e < sl.floats(lh)) {
                    const int l = (e - sl.bias) >> lh2, n = (e - sl.bias) & hm;
                    v = p[off.b(l) + n];
                    sc = l == 0 ? s0 : s;
                }
                v4[q] = v;
            }
        } else {
            const unsigned e = idx - (unsigned)spad;
            const unsigned slice = e >> lsf;
            const unsigned w = e & sfm;
            const int i = (w >> 2) & 15, g = (w >> 6) & 3, blk = w >> 8;
            if (slice < (unsigned)(lh * nb)) {
                const int l = (int)(slice / nb) + 1, kb = (int)(slice % nb);
                const float* src = p + off.w(l) + (int64_t)(16 * blk + i) * h + 16 * kb + 4 * g;
                v4 = f32x4{src[0], src[1], src[2], src[3]};
            } else {
                const int s2 = (int)slice - lh * nb;
                const int l = lh - s2 / nb, kb = s2 % nb;
                const float* src = p + off.w(l) + (int64_t)(16 * kb + 4 * g) * h + 16 * blk + i;
                v4 = f32x4{src[0], src[h], src[2 * h], src[3 * h]};
            }
            sc = s;
        }
        *(f32x4*)(ws + gidx) = scaled ? v4 * sc : v4;
    }
}

// One 16 KiB slice: acc[ob] += W-slice(ob) x B(kb), 64 MFMAs per wave. Output blocks are processed in
// pairs so consecutive MFMAs never hit the same accumulator (16x16x4 f32: 32-cycle issue, 40-cycle
// dependent latency) and the next pair's A operands are read from LDS while the current pair computes.
__device__ __forceinline__ void slice_mma(const float* sl, const f32x4& bop, f32x4 (&acc)[NB]) {
    f32x4 a0 = *(const f32x4*)(sl);
    f32x4 a1 = *(const f32x4*)(sl + 256);
#pragma unroll
    for (int ob = 0; ob < NB; ob += 2) {
        f32x4 n0, n1;
        if (ob + 2 < NB) {
            n0 = *(const f32x4*)(sl + (ob + 2) * 256);
            n1 = *(const f32x4*)(sl + (ob + 3) * 256);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            acc[ob] = mfma4(a0[r], bop[r], acc[ob]);
            acc[ob + 1] = mfma4(a1[r], bop[r], acc[ob + 1]);
        }
        if (ob + 2 < NB) {
            a0 = n0;
            a1 = n1;
        }
    }
}

// One layer GEMM over 16 slices (K = 256); the slice counter s runs across layers.
__device__ __forceinline__ void layer_mma(const float* __restrict__ stream, float* ring, int& s, int nslices,
                                          int wave, int lane, const f32x4 (&act)[NB], f32x4 (&acc)[NB]) {
#pragma unroll
    for (int ob = 0; ob < NB; ++ob) acc[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < NB; ++kb) {
        ring_wait(s, nslices);
        ring_issue(stream, ring, s + 2, nslices, wave, lane);
        slice_mma(ring + (s % NBUF) * SLICE + lane * 4, act[kb], acc);
        ++s;
    }
}

// Hidden-layer epilogue: z = acc + b; t = w z; act = sin(t); cs = cos(t)  (modules.py:24, :34).
__device__ __forceinline__ void epilogue_sincos(const f32x4 (&acc)[NB], const float* bl, float w, f32x4 (&act)[NB],
                                                f32x4 (&cs)[NB]) {
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        const f32x4 z = acc[rb] + *(const f32x4*)(bl + 16 * rb);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sn, cn;
            sincos_phase(w * z[r], sn, cn);
            act[rb][r] = sn;
            cs[rb][r] = cn;
        }
    }
}

// ------------------------------------------------------------------------------------------------------
// The fused kernel. GRAD = false: forward only (W0), any number of hidden layers (runtime lh).
//                   GRAD = true : forward + vjp_x (W1), LH (template) hidden layers.
// ------------------------------------------------------------------------------------------------------
// STORE = true (with GRAD): the W2 backward's first stage. Additionally writes the sin activations a_l
// (l = 0..LH) to abuf and the reverse-sweep deltas delta_l (l = 0..LH) to dbuf, both in the coordinate-tile
// layout [l][tile of 16 coords][neuron][16] that the weight-gradient kernel stages into LDS (siren_train.hip).
template <int LH_T, bool GRAD, bool STORE = false>
__global__ __launch_bounds__(THREADS, GRAD ? 1 : 2) void fused_kernel(
    const float* __restrict__ ws, const float* __restrict__ x, int64_t n, const float* __restrict__ gy,
    float* __restrict__ y, float* __restrict__ gx, int d, int o, int lh_rt, float w0, float w, int final_sine,
    float* __restrict__ abuf = nullptr, float* __restrict__ dbuf = nullptr, int64_t n_pad = 0) {
    __shared__ __attribute__((aligned(16))) float lds[NBUF * SLICE + SMALL_MAX];
    const int LH = GRAD ? LH_T : lh_rt;
    float* ring = lds;
    float* sm = lds + NBUF * SLICE;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15;
    const int nslices = (GRAD ? 2 : 1) * LH * NB;
    const float* stream = ws + small_pad(LH);

    // ---- small parameters -> LDS; coordinates -> VGPRs --------------------------------------------------
    {
        const int nf4 = (small_floats(LH) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t coord = (int64_t)blockIdx.x * TILE + wave * 16 + c;
    const bool valid = coord < n;
    const int64_t lstride = n_pad * H;                                            // STORE: floats per layer
    const int64_t toff = ((int64_t)blockIdx.x * WAVES + wave) * (H * 16) + 4 * g * 16 + c;  // tile + lane
    float xv[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) xv[k] = (valid && k < d) ? x[coord * d + k] : 0.f;
    __syncthreads();
    ring_issue(stream, ring, 0, nslices, wave, lane);
    ring_issue(stream, ring, 1, nslices, wave, lane);

    // ---- first layer (K = d_in) on VALU ----------------------------------------------------------------
    f32x4 act[NB];
    f32x4 C0[NB], C1[NB], C2[NB];  // cos(w z_l) of layers 0, 1, 2 for the reverse sweep (GRAD only)
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        const int nb = 16 * rb + 4 * g;
        const f32x4 b4 = *(const f32x4*)(sm + SM_BIAS + nb);
        f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < MAXD; ++k) {
            if (k < d) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + nb);
                z = k == 0 ? xv[0] * wk : z + xv[k] * wk;
            }
        }
        z += b4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float sn, cs;
            sincos_phase(w0 * z[r], sn, cs);
            act[rb][r] = sn;
            if (GRAD) C0[rb][r] = cs;
        }
    }
    if (STORE) store_tile(abuf + toff, act);

    // ---- hidden layers on MFMA ---------------------------------------------------------------------------
    // cos(w z_l) of layer l is kept in C{l} (C0 from the first layer). The layer loop is a runtime loop so
    // the 1024-MFMA layer body exists once in the code object; only the epilogue is specialised per layer.
    // The last hidden layer's epilogue folds the output layer in (y partial sums) and leaves cos(w z_L)
    // in `act`, where the reverse sweep's seed is formed.
    int s = 0;
    f32x4 acc[NB];
    float yp[MAXO] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int l = 1; l <= LH; ++l) {
        layer_mma(stream, ring, s, nslices, wave, lane, act, acc);
        const float* bl = sm + SM_BIAS + l * H + 4 * g;
        if (l == LH) {
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 z = acc[rb] + *(const f32x4*)(bl + 16 * rb);
                f32x4 sn;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (GRAD) {
                        float a, cn;
                        sincos_phase(w * z[r], a, cn);
                        sn[r] = a;
                        act[rb][r] = cn;
                    } else {
                        sn[r] = sin_phase(w * z[r]);
                    }
                }
                if (STORE) store_block(abuf + (int64_t)LH * lstride + toff, rb, sn);
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    if (j < o) {
                        const f32x4 wj = *(const f32x4*)(sm + SM_WO + j * H + 16 * rb + 4 * g);
                        yp[j] += wj[0] * sn[0] + wj[1] * sn[1] + wj[2] * sn[2] + wj[3] * sn[3];
                    }
                }
            }
        } else if (!GRAD) {
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 z = acc[rb] + *(const f32x4*)(bl + 16 * rb);
#pragma unroll
                for (int r = 0; r < 4; ++r) act[rb][r] = sin_phase(w * z[r]);
            }
        } else if (l == 1) {
            epilogue_sincos(acc, bl, w, act, C1);
            if (STORE) store_tile(abuf + lstride + toff, act);
        } else {
            epilogue_sincos(acc, bl, w, act, C2);
            if (STORE) store_tile(abuf + 2 * lstride + toff, act);
        }
    }

    // ---- output layer: y = a_L Wout^T + bout (partials above + cross-group reduction) -------------------
    float gyv[MAXO];
#pragma unroll
    for (int j = 0; j < MAXO; ++j) {
        gyv[j] = 0.f;
        if (j < o) {
            float yj = sum_groups(yp[j]) + sm[SM_BOUT + j];
            float fs = 1.f;
            if (final_sine) {
                float sn, cs;
                sincos_phase(w * yj, sn, cs);
                yj = sn;
                fs = cs;
            }
            if (y != nullptr && valid && g == 0) y[coord * o + j] = yj;
            if (GRAD) {
                float gj = 1.f;
                if (gy != nullptr) gj = valid ? gy[coord * o + j] : 0.f;
                gyv[j] = final_sine ? (gj * fs) * w : gj;
            }
        }
    }
    if (!GRAD) return;

    // ---- reverse sweep ----------------------------------------------------------------------------------
    // delta_L[n] = (sum_j gy_j Wout[j][n]) * cos(w z_L[n]) * w
    const bool seed_ones = (gy == nullptr) && !final_sine;
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
        const int nb = 16 * rb + 4 * g;
        f32x4 ga;
        if (seed_ones) {
            ga = *(const f32x4*)(sm + SM_SEED + nb);
        } else {
            ga = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < MAXO; ++j)
                if (j < o) ga += gyv[j] * *(const f32x4*)(sm + SM_WO + j * H + nb);
        }
        act[rb] = (ga * act[rb]) * w;
    }
    if (STORE) store_tile(dbuf + (int64_t)LH * lstride + toff, act);
#pragma unroll 1
    for (int l = LH; l >= 1; --l) {
        layer_mma(stream, ring, s, nslices, wave, lane, act, acc);
        if (l == 1) {
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) act[rb] = (acc[rb] * C0[rb]) * w0;
        } else if (l == 2) {
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) act[rb] = (acc[rb] * C1[rb]) * w;
        } else {
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) act[rb] = (acc[rb] * C2[rb]) * w;
        }
        if (STORE) store_tile(dbuf + (int64_t)(l - 1) * lstride + toff, act);
    }

    // ---- gx = delta_0 W0 ----------------------------------------------------------------------------------
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (k < d) {
            float p = 0.f;
#pragma unroll
            for (int rb = 0; rb < NB; ++rb) {
                const f32x4 wk = *(const f32x4*)(sm + SM_W0 + k * H + 16 * rb + 4 * g);
                p += wk[0] * act[rb][0] + wk[1] * act[rb][1] + wk[2] * act[rb][2] + wk[3] * act[rb][3];
            }
            p = sum_groups(p);
            if (valid && g == 0) gx[coord * d + k] = p;
        }
    }
}

}  // namespace siren


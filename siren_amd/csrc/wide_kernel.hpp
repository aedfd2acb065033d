#pragma once
// wide_kernel.hpp — fused SIREN kernels for hidden width 512 (BASELINE config 4: SingleBVPNet(hidden_features=512),
// the 5x512 image / video fits; reference modules.py:37-160 with hidden_features=512).
//
// Same MFMA tiling as the H = 256 kernels (siren_common.h): one wave owns 16 coordinates, the activation tile
// is 32 neuron blocks x f32x4 in C/D layout, and it IS the next layer's B operand. At H = 512 the activation
// and accumulator tiles alone take 256 VGPRs per lane, so nothing else of the forward pass can stay in
// registers: cos(w z_l) of layers 0..L-1 — needed by the reverse sweep — is spilled to an HBM scratch in a
// lane-major layout (one coalesced dwordx4 per lane per block, 16 KiB per wave per layer) and read back by
// the reverse epilogues. Per coordinate that is 2 x L x 2 KiB of scratch traffic against ~3.2 MFLOP of MFMA
// work (W1, L = 3): 0.004 B/FLOP, i.e. ~0.6 TB/s at the fp32 MFMA peak — far below the HBM roofline.
//
// Weights stream through a 3-slot ring of 32 KiB slices (16 K-neurons x 512 out-neurons, the layout
// pack_kernel writes for h = 512). The forward and the reverse layer GEMMs run through ONE copy of the
// 4096-MFMA layer body (a single pass loop over 2 L passes) to keep the code object inside the I-cache.
//
// Modes (siren_common.h): MODE_FWD (W0: y only), MODE_W1 (y and vjp_x), MODE_STORE (W2 backward stage 1:
// additionally a_l and delta_l of every layer to abuf / dbuf in the [l][tile][neuron][16] layout that
// wgrad_kernel / small_kernel read with h = 512). Stored-forward W2 split: MODE_FWDS = the forward passes with
// a_l tiles to abuf and cos(w z_l) of layers 0..L (L + 1 scratch layers) to the scratch; MODE_REV = the seed from
// the stored cos(w z_L) and the L reverse passes only, delta_l tiles to dbuf.
#include "lds_ops.h"
#include "siren_common.h"
#include "siren_params.h"

namespace siren {

constexpr int WH = 512;
constexpr int WNB = WH / 16;       // 32 neuron blocks per activation tile
constexpr int WSLICE = 16 * WH;    // floats per weight slice (32 KiB)
constexpr int WNBUF = 3;
constexpr int WSMALL_MAX = 9 * WH + 4 + (MAX_LH_FWD + 1) * WH;

// wave w copies 8 KiB (8 x 1 KiB global_load_lds_dwordx4) of every 32 KiB slice
__device__ __forceinline__ void wring_issue(const float* __restrict__ stream, float* ring, int s, int nslices,
                                            int wave, int lane) {
    if (s < nslices) {
        const int wu = __builtin_amdgcn_readfirstlane(wave);
        const char* src = (const char*)(stream + (int64_t)s * WSLICE + wu * 2048);
        const unsigned dst = lds_addr(ring + (s % WNBUF) * WSLICE + wu * 2048);
#pragma unroll
        for (int q = 0; q < 8; ++q) glds_x4(src + q * 1024, 16u * lane, dst + q * 1024);
    }
}

// slice s landed for this wave (s+1 may stay in flight; the count also covers scratch stores issued since),
// then a barrier: every wave's part landed and the slot refilled next has been read by everyone
__device__ __forceinline__ void wring_wait(int s, int nslices) {
    if (s + 1 < nslices)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// STORE-mode tile writer; the pointer is stepped through an opaque register so the compiler cannot hoist 32
// precomputed 64-bit block addresses (they would not fit next to the 256 VGPRs of act + acc)
__device__ __forceinline__ void wstore_tile(float* p, const f32x4 (&v)[WNB]) {
#pragma unroll
    for (int rb = 0; rb < WNB; ++rb) {
        store_block(p, 0, v[rb]);
        p += 256;
        asm volatile("" : "+v"(p));
    }
}

template <int MODE>
__global__ __launch_bounds__(THREADS, 1) void wide_kernel(
    const float* __restrict__ ws, const float* __restrict__ x, int64_t n, const float* __restrict__ gy,
    float* __restrict__ y, float* __restrict__ gx, int d, int o, int lh, float w0, float w, int final_sine,
    float* __restrict__ spill, float* __restrict__ abuf, float* __restrict__ dbuf, int64_t n_pad) {
    constexpr bool FWDS = MODE == MODE_FWDS, REV = MODE == MODE_REV;
    constexpr bool GRAD = MODE == MODE_W1 || MODE == MODE_STORE || REV;  // runs the reverse passes
    constexpr bool SPILLC = GRAD || FWDS;                                // forward writes cos to the scratch
    constexpr bool STORE = MODE == MODE_STORE || FWDS;                   // a_l tiles (STORE, FWDS)
    constexpr bool DSTORE = MODE == MODE_STORE || REV;                   // delta_l tiles (STORE, REV)
    __shared__ __attribute__((aligned(16))) float lds[WNBUF * WSLICE + WSMALL_MAX];
    const SmallLayout L(WH);
    float* ring = lds;
    float* sm = lds + WNBUF * WSLICE;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, c = lane & 15;
    const int npass = (GRAD ? 2 : 1) * lh;
    const int nslices = npass * WNB;
    const int p0 = REV ? lh : 0;  // REV: reverse passes only (slices from lh * WNB on)
    const float* stream = ws + L.pad(lh);

    {
        const int nf4 = (L.floats(lh) + 3) / 4;
        for (int e = threadIdx.x; e < nf4; e += THREADS) ((f32x4*)sm)[e] = ((const f32x4*)ws)[e];
    }
    const int64_t coord = (int64_t)blockIdx.x * TILE + wave * 16 + c;
    const bool valid = coord < n;
    const int64_t wt = (int64_t)blockIdx.x * WAVES + wave;             // this wave's 16-coordinate tile
    const int64_t lstride = n_pad * WH;                                 // floats per layer (abuf/dbuf/spill)
    const int64_t toff = wt * (WH * 16) + 4 * g * 16 + c;               // STORE: tile + lane
    float* sp = spill + wt * (WH * 16) + lane * 4;                      // scratch: lane-major blocks
    float xv[MAXD];
#pragma unroll
    for (int k = 0; k < MAXD; ++k) xv[k] = (valid && k < d) ? x[coord * d + k] : 0.f;
    __syncthreads();
    int s = p0 * WNB;
    wring_issue(stream, ring, s, nslices, wave, lane);
    wring_issue(stream, ring, s + 1, nslices, wave, lane);

    // ---- first layer (K = d_in) on VALU ----------------------------------------------------------------
    f32x4 act[WNB], acc[WNB];
    if constexpr (REV) {
        // seed delta_L = (gy Wout) . cos(w z_L) . w from the forward's stored cos
        float gyv[MAXO];
#pragma unroll
        for (int j = 0; j < MAXO; ++j) gyv[j] = (j < o) ? (gy == nullptr ? 1.f : (valid ? gy[coord * o + j] : 0.f)) : 0.f;
        const float* cp = sp + (int64_t)lh * lstride;
#pragma unroll
        for (int rb = 0; rb < WNB; ++rb) {
            f32x4 ga = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < MAXO; ++j)
                if (j < o) ga += gyv[j] * *(const f32x4*)(sm + L.wo + j * WH + 16 * rb + 4 * g);
            act[rb] = (ga * *(const f32x4*)(cp + rb * 256)) * w;
        }
        wstore_tile(dbuf + (int64_t)lh * lstride + toff, act);
    }
#pragma unroll
    for (int rb = 0; rb < (REV ? 0 : WNB); ++rb) {
        const int nb = 16 * rb + 4 * g;
        f32x4 z = *(const f32x4*)(sm + L.bias + nb);
#pragma unroll
        for (int k = 0; k < MAXD; ++k)
            if (k < d) z += xv[k] * *(const f32x4*)(sm + L.w0 + k * WH + nb);
        f32x4 sn, cs;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float a, cn;
            sincos_fast(w0 * z[r], a, cn);
            sn[r] = a;
            cs[r] = cn;
        }
        act[rb] = sn;
        if (SPILLC) *(f32x4*)(sp + rb * 256) = cs;
    }
    if (STORE && !REV) wstore_tile(abuf + toff, act);

    // ---- 2 L layer passes through one layer body: forward l = 1..L, then reverse l = L..1 ----------------
    float yp[MAXO] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int p = p0; p < npass; ++p) {
#pragma unroll
        for (int ob = 0; ob < WNB; ++ob) acc[ob] = f32x4{0.f, 0.f, 0.f, 0.f};
        // reverse passes: cos(w z_lm) block kb of the epilogue is loaded into act[kb] as soon as slice kb has
        // consumed it (the B operand is dead after its slice), so the epilogue's 32 scratch loads are in flight
        // under the remaining slices instead of exposed after the GEMM. The ring's vmcnt(8) stays correct (it
        // only waits for more).
        const bool rev_pass = GRAD && p >= lh;
        const float* cpre = rev_pass ? sp + (int64_t)(2 * lh - p - 1) * lstride : sp;
#pragma unroll
        for (int kb = 0; kb < WNB; ++kb) {
            wring_wait(s, nslices);
            wring_issue(stream, ring, s + 2, nslices, wave, lane);
            slice_mma<WNB>(lds_addr(ring + (s % WNBUF) * WSLICE) + 16u * lane, act[kb], acc);  // lds_ops.h
            if (rev_pass) act[kb] = *(const f32x4*)(cpre + kb * 256);
            ++s;
        }
        if (p < lh - 1) {
            // hidden layer l = p + 1: a_l = sin(w z_l), cos(w z_l) -> scratch
            const int l = p + 1;
            const float* bl = sm + L.bias + l * WH + 4 * g;
#pragma unroll
            for (int rb = 0; rb < WNB; ++rb) {
                const f32x4 z = acc[rb] + *(const f32x4*)(bl + 16 * rb);
                f32x4 sn, cs;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float a, cn;
                    sincos_fast(w * z[r], a, cn);
                    sn[r] = a;
                    cs[r] = cn;
                }
                act[rb] = sn;
                if (SPILLC) *(f32x4*)(sp + (int64_t)l * lstride + rb * 256) = cs;
            }
            if (STORE) wstore_tile(abuf + (int64_t)l * lstride + toff, act);
        } else if (p == lh - 1) {
            // last hidden layer: a_L folded into y; cos(w z_L) stays in act for the seed
            const float* bl = sm + L.bias + lh * WH + 4 * g;
            float* ap = STORE ? abuf + (int64_t)lh * lstride + toff : nullptr;
#pragma unroll
            for (int rb = 0; rb < WNB; ++rb) {
                const f32x4 z = acc[rb] + *(const f32x4*)(bl + 16 * rb);
                f32x4 sn;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float a, cn;
                    sincos_fast(w * z[r], a, cn);
                    sn[r] = a;
                    act[rb][r] = cn;
                }
                if (FWDS) *(f32x4*)(sp + (int64_t)lh * lstride + rb * 256) = act[rb];
                if (STORE) {
                    store_block(ap, 0, sn);
                    ap += 256;
                    asm volatile("" : "+v"(ap));
                }
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    if (j < o) {
                        const f32x4 wj = *(const f32x4*)(sm + L.wo + j * WH + 16 * rb + 4 * g);
                        yp[j] += wj[0] * sn[0] + wj[1] * sn[1] + wj[2] * sn[2] + wj[3] * sn[3];
                    }
                }
            }
            // output layer and the reverse-sweep seed delta_L = (gy Wout) . cos(w z_L) . w
            float gyv[MAXO];
#pragma unroll
            for (int j = 0; j < MAXO; ++j) {
                gyv[j] = 0.f;
                if (j < o) {
                    float yj = sum_groups(yp[j]) + sm[L.bout + j];
                    float fs = 1.f;
                    if (final_sine) {
                        float sn, cs;
                        sincos_fast(w * yj, sn, cs);
                        yj = sn;
                        fs = cs;
                    }
                    if (y != nullptr && valid && g == 0) y[coord * o + j] = yj;
                    float gj = 1.f;
                    if (gy != nullptr) gj = valid ? gy[coord * o + j] : 0.f;
                    gyv[j] = final_sine ? (gj * fs) * w : gj;
                }
            }
            if (!GRAD) return;
#pragma unroll
            for (int rb = 0; rb < WNB; ++rb) {
                f32x4 ga = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < MAXO; ++j)
                    if (j < o) ga += gyv[j] * *(const f32x4*)(sm + L.wo + j * WH + 16 * rb + 4 * g);
                act[rb] = (ga * act[rb]) * w;
            }
            if (DSTORE) wstore_tile(dbuf + (int64_t)lh * lstride + toff, act);
        } else {
            // reverse pass through W_l (l = 2L - p): delta_{l-1} = (delta_l W_l) . cos(w z_{l-1}) . w_{l-1}
            const int lm = 2 * lh - p - 1;
            const float wl = lm == 0 ? w0 : w;
#pragma unroll
            for (int rb = 0; rb < WNB; ++rb) act[rb] = (acc[rb] * act[rb]) * wl;  // act = the prefetched cos
            if (DSTORE) wstore_tile(dbuf + (int64_t)lm * lstride + toff, act);
        }
    }

    // ---- gx = delta_0 W0 ----------------------------------------------------------------------------------
#pragma unroll
    for (int k = 0; k < MAXD; ++k) {
        if (k < d) {
            float q = 0.f;
#pragma unroll
            for (int rb = 0; rb < WNB; ++rb) {
                const f32x4 wk = *(const f32x4*)(sm + L.w0 + k * WH + 16 * rb + 4 * g);
                q = dot4_acc(wk, act[rb], q);
            }
            q = sum_groups(q);
            if (valid && g == 0) gx[coord * d + k] = q;
        }
    }
}

}  // namespace siren

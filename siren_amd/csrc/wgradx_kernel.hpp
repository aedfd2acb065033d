#pragma once
// wgradx_kernel.hpp — the hidden-layer weight gradient of the bf16x6 training leg (siren_backward_split):
//   dW_l = delta_l^T a_{l-1},  db_l = sum delta_l        (l = 1..LH, hidden 256)
// on the bf16 matrix pipe in fp32-equivalent precision, as w1x_kernel.hpp does for the layer GEMMs: every fp32 tile
// value is split exactly into bf16 (hi, mid, lo) and each K-step of 32 coordinates sums the six products at or above
// 2^-16 of hi*hi on v_mfma_f32_16x16x32_bf16 (fp32 accumulation). Six 16-cycle MFMAs replace eight 32-cycle fp32
// 16x16x4 MFMAs per 32 coordinates: 2.67x less matrix time than wgrad_kernel (train_kernels.hpp), whose tiles,
// ring staging, grid and slab output it shares.
//   * grid (S, LH): block (s, l - 1) reduces the coordinate tiles [s tps, (s + 1) tps) of layer l (tps even: a
//     K-step is a PAIR of 16-coordinate tiles) into partial slab s; wave w owns the 128 x 128 sub-block (rows
//     128 (w >> 1), cols 128 (w & 1)), 64 accumulator blocks.
//   * A 4-slot glds ring of 32 KiB tiles (delta + a, swizzled as wgrad_kernel stages them); pair c lands in slots
//     2c, 2c + 1 (mod 4) while pair c - 1 computes.
//   * Operand lane (kg, m) = (lane >> 4, lane & 15) takes row m of a block at coordinates 8 kg .. 8 kg + 7 of the
//     pair (tile kg >> 1, quads 2 (kg & 1), 2 (kg & 1) + 1): two ds_read_b128, split in registers. The B pieces of the
//     wave's 8 column blocks are split once per pair and reused by all 8 row blocks.
//   * The bias sums accumulate from the delta rows already in registers (each lane: its 8 coordinates), combined over
//     the four K groups through the idle ring at the end in a fixed order, as wgrad_kernel.
#include "siren_params.h"
#include "w1x_kernel.hpp"

namespace siren {

constexpr int WX_NBUF = 4;                   // ring slots of one 16-coordinate tile each (delta 16 KiB + a 16 KiB)
constexpr int WX_TILE_FLOATS = H * 16;       // 256 neurons of one 16-coordinate tile
constexpr int WX_SLOT = 2 * WX_TILE_FLOATS;  // delta tile + activation tile
// wgrad_kernel's swizzled staging (train_kernels.hpp wg_swz_off): lane L fills LDS position L & 3 of row L >> 2 and
// fetches quad ((L & 3) - (L >> 3)) & 3 of that row, so row r keeps its quad c at position (c + (r >> 1)) & 3
__device__ __forceinline__ unsigned wx_swz_off(int lane) {
    const int rr = lane >> 2, p = lane & 3;
    return (unsigned)(rr * 64 + (((p - (rr >> 1)) & 3) * 16));
}

__device__ __forceinline__ void wx_issue(const float* __restrict__ dsrc, const float* __restrict__ asrc, float* ring,
                                         int64_t t, int slot, int wave, unsigned swz, int64_t tstride) {
    float* sl = ring + slot * WX_SLOT;
    const int wu = __builtin_amdgcn_readfirstlane(wave);
    // wave wu stages 8 chunks of 1 KiB: waves 0, 1 the delta tile, waves 2, 3 the activation tile
    const float* src = (wu < 2 ? dsrc + wu * 2048 : asrc + (wu - 2) * 2048) + t * tstride;
#pragma unroll
    for (int q = 0; q < 8; ++q) glds_x4(src + q * 256, swz, lds_addr(sl + (wu * 8 + q) * 256));
}

// coordinates 8 hq .. 8 hq + 7 of tile row R in a staged tile (row R keeps its quad c at 16 B position (c + (R >> 1)) & 3)
__device__ __forceinline__ void wx_row8(const float* tile, int R, int hq, f32x4& v0, f32x4& v1) {
    const float* row = tile + R * 16;
    v0 = *(const f32x4*)(row + (((2 * hq) + (R >> 1)) & 3) * 4);
    v1 = *(const f32x4*)(row + (((2 * hq + 1) + (R >> 1)) & 3) * 4);
}
// the exact (hi, mid, lo) bf16 pieces of 8 values as MFMA operands (element j of the lane = its j-th coordinate)
__device__ __forceinline__ void wx_split(const f32x4& v0, const f32x4& v1, u32x4 (&p)[3]) {
    unsigned h, m, l;
    split_pair(v0[0], v0[1], h, m, l);
    p[0][0] = h, p[1][0] = m, p[2][0] = l;
    split_pair(v0[2], v0[3], h, m, l);
    p[0][1] = h, p[1][1] = m, p[2][1] = l;
    split_pair(v1[0], v1[1], h, m, l);
    p[0][2] = h, p[1][2] = m, p[2][2] = l;
    split_pair(v1[2], v1[3], h, m, l);
    p[0][3] = h, p[1][3] = m, p[2][3] = l;
}

__global__ __launch_bounds__(THREADS, 1) void wgradx_kernel(const float* __restrict__ abuf,
                                                           const float* __restrict__ dbuf, int64_t n_pad, int64_t tps,
                                                           float* __restrict__ partial, int64_t P, int d, int o,
                                                           int lh) {
    __shared__ __attribute__((aligned(16))) float ring[WX_NBUF * WX_SLOT];
    const ParamOffsets off(d, o, lh, H);
    const int s = blockIdx.x, l = blockIdx.y + 1;
    const int64_t tstride = (int64_t)H * 16;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kg = lane >> 4, m = lane & 15;
    const int wr = wave >> 1, wc = wave & 1;
    const int64_t T = n_pad / 16;
    const int64_t t0 = (int64_t)s * tps, t1 = t0 + tps < T ? t0 + tps : T;
    const int64_t pairs = (t1 - t0) / 2;  // tps even and T a multiple of 4: whole pairs
    const float* dsrc = dbuf + (int64_t)l * n_pad * H;
    const float* asrc = abuf + (int64_t)(l - 1) * n_pad * H;
    const unsigned swz = wx_swz_off(lane);

    f32x4 acc[8][8];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

    if (pairs > 0) {
        wx_issue(dsrc, asrc, ring, t0, 0, wave, swz, tstride);
        wx_issue(dsrc, asrc, ring, t0 + 1, 1, wave, swz, tstride);
    }
    for (int64_t c = 0; c < pairs; ++c) {
        // pair c has landed (nothing younger is in flight); every wave is done with pair c - 1's slots, which pair
        // c + 1 overwrites
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_barrier" ::: "memory");  // also a compiler barrier for the LDS loads
        if (c + 1 < pairs) {
            wx_issue(dsrc, asrc, ring, t0 + 2 * c + 2, (int)((2 * c + 2) % WX_NBUF), wave, swz, tstride);
            wx_issue(dsrc, asrc, ring, t0 + 2 * c + 3, (int)((2 * c + 3) % WX_NBUF), wave, swz, tstride);
        }
        const float* tl = ring + ((2 * c + (kg >> 1)) % WX_NBUF) * WX_SLOT;  // this lane's tile of the pair
        const int hq = kg & 1;
        f32x4 braw[8][2];
#pragma unroll
        for (int cb = 0; cb < 8; ++cb) wx_row8(tl + WX_TILE_FLOATS, 128 * wc + 16 * cb + m, hq, braw[cb][0], braw[cb][1]);
        u32x4 bp[8][3];
#pragma unroll
        for (int rb = 0; rb < 8; ++rb) {
            f32x4 v0, v1;
            wx_row8(tl, 128 * wr + 16 * rb + m, hq, v0, v1);
            bs[rb] += ((v0[0] + v0[1]) + (v0[2] + v0[3])) + ((v1[0] + v1[1]) + (v1[2] + v1[3]));
            u32x4 ap[3];
            wx_split(v0, v1, ap);
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) {  // smallest products first
                if (rb == 0) wx_split(braw[cb][0], braw[cb][1], bp[cb]);  // split in the first row block's MFMA stream
                acc[rb][cb] = mfma_x(ap[2], bp[cb][0], acc[rb][cb]);
                acc[rb][cb] = mfma_x(ap[1], bp[cb][1], acc[rb][cb]);
                acc[rb][cb] = mfma_x(ap[0], bp[cb][2], acc[rb][cb]);
                acc[rb][cb] = mfma_x(ap[1], bp[cb][0], acc[rb][cb]);
                acc[rb][cb] = mfma_x(ap[0], bp[cb][1], acc[rb][cb]);
                acc[rb][cb] = mfma_x(ap[0], bp[cb][0], acc[rb][cb]);
            }
        }
        // every read of this pair's slots is retired before the next barrier (the next issue overwrites them)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    float* out = partial + (int64_t)s * P;
    float* dW = out + off.w(l);
    const int g = kg, i = m;  // C/D layout: lane (g, i) holds rows 4 g + q, column i of a block
#pragma unroll
    for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int cb = 0; cb < 8; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                dW[(int64_t)(128 * wr + 16 * rb + 4 * g + q) * H + 128 * wc + 16 * cb + i] = acc[rb][cb][q];
    // bias: lane (kg, m) holds row 128 wr + 16 rb + m over coordinates 8 kg .. 8 kg + 7 of every pair; the four K
    // groups of each row combined in a fixed order through the (now idle) ring
    __syncthreads();
    if (wc == 0) {
#pragma unroll
        for (int rb = 0; rb < 8; ++rb) ring[(128 * wr + 16 * rb + m) * 4 + kg] = bs[rb];
    }
    __syncthreads();
    const float* rw = ring + threadIdx.x * 4;
    out[off.b(l) + threadIdx.x] = (rw[0] + rw[1]) + (rw[2] + rw[3]);
}

}  // namespace siren

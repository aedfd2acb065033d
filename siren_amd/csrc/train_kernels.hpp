#pragma once
// train_kernels.hpp — weight-gradient stage of the W2 (image-fit train step) backward for gfx950.
//
// Replaces the reference's MmBackward grad-weight GEMMs ([H,N] x [N,H], K = N) and bias-grad sums that
// autograd runs for train_loss.backward() (training.py:95-96) on the BatchLinear stack (modules.py:23-24).
// Input: the per-layer sin activations a_l and deltas delta_l that the fused kernel wrote in STORE mode, in
// the coordinate-tile layout [l][tile][neuron][16 coords] (siren_fused.hip).
//   wgrad_kernel : dW_l = delta_l^T a_{l-1}, db_l = sum delta_l   (l = 1..LH), v_mfma_f32_16x16x4_f32, split-K
//   small_kernel : dW_0 = delta_0^T x, db_0, dW_out = gy^T a_LH, db_out  (VALU; K = d_in / d_out <= 4)
//   reduce_kernel: deterministic sum of the per-split partial slabs into the flat gradient (param order)
#include <type_traits>

#include "siren_common.h"
#include "siren_params.h"
#include "lds_ops.h"

namespace siren {

constexpr int WG_TILE_FLOATS = H * 16;          // 256 neurons of one 16-coordinate tile (16 KiB)
constexpr int WG_SLOT = 2 * WG_TILE_FLOATS;     // delta (half-)tile + activation (half-)tile
// Ring of 32 KiB slots (one 16-coordinate tile each). Round 6 A/B: 4 slots with one barrier per PAIR of tiles (and the
// pair's ring issue behind the first block's MFMAs) measured neutral to 0.7 % slower (video 12.46 vs 12.38 ms, Poisson
// 3.25 vs 3.23 ms per launch): the per-tile barrier is not what the kernel waits for.
constexpr int WG_NBUF = 3;


// Ring layout: a staged 1 KiB chunk is 16 neuron rows of 64 B (16 coordinates); row r keeps its coordinate quad c
// at 16 B position (c + (r >> 1)) & 3. The swizzle is applied by the global side of the load (lane L fills LDS
// position L & 3 of row L >> 2, so it fetches quad ((L & 3) - (L >> 3)) & 3 of that row), and with it the operand
// reads (lane (g, i) reads quad g of row i) put every 16-lane ds_read_b128 group on 16 distinct 16 B slots of the
// 256 B bank row: conflict-free (the linear layout was 2-way, 5.6 conflict cycles per LDS instruction).
__device__ __forceinline__ unsigned wg_swz_off(int lane) {
    const int rr = lane >> 2, p = lane & 3;
    return (unsigned)(rr * 64 + (((p - (rr >> 1)) & 3) * 16));
}

__device__ __forceinline__ void wg_issue(const float* __restrict__ dsrc, const float* __restrict__ asrc, float* ring,
                                         int64_t t, int64_t t1, int k, int wave, unsigned swz, int64_t tstride) {
    if (t < t1) {
        float* slot = ring + (k % WG_NBUF) * WG_SLOT;
        const int wu = __builtin_amdgcn_readfirstlane(wave);
        // wave wu stages 8 chunks of 1 KiB: waves 0, 1 the delta tile, waves 2, 3 the activation tile
        const float* src = (wu < 2 ? dsrc + wu * 2048 : asrc + (wu - 2) * 2048) + t * tstride;
#pragma unroll
        for (int q = 0; q < 8; ++q) glds_x4(src + q * 256, swz, lds_addr(slot + (wu * 8 + q) * 256));
    }
}

// grid (S, LH, (h/256)^2): block (s, l-1, q) reduces coordinate tiles [s*tps, min(T, (s+1)*tps)) of layer l
// into the 256x256 block q = (qr, qc) of dW_l (the whole dW_l for h = 256; a quadrant for h = 512, staging
// only the 256-neuron halves of the delta and activation tiles it needs).
// Wave w owns the 128x128 sub-block (rows 128*(w>>1), cols 128*(w&1)).
// Software-pipelined: a tile's 16 operand reads are issued into the second register set while the previous tile's
// 256 MFMAs run (the first version waited lgkmcnt(0) on them at the top of every tile, behind the barrier), and
// the bias gradient accumulates from the delta operands already in registers (no extra LDS row reads).
// JB = jet_bias at compile time (0 plain tiles; 1 jet tiles, value column 4g; 2 two-stream tiles, columns 4g, 4g + 2;
// 3 Q8 tile pairs), and the two waves that share a delta row half (wc = 0, 1) each sum the bias of every other block
// instead of both summing all eight: the runtime 0/1 masks and the duplicate sums were half of the loop's non-MFMA VALU
// (round 6; the waves meet at every tile's barrier, so the work is split evenly rather than given to one wave).
template <int JB>
__global__ __launch_bounds__(THREADS, 1) void wgrad_kernel(const float* __restrict__ abuf,
                                                          const float* __restrict__ dbuf, int64_t n_pad,
                                                          int64_t tps, float* __restrict__ partial, int64_t P,
                                                          int d, int o, int lh, int with_bias, int h,
                                                          int64_t bstride_act = 0,
                                                          int64_t bstride_part = 0) {
    __shared__ __attribute__((aligned(16))) float ring[WG_NBUF * WG_SLOT];
    const ParamOffsets off(d, o, lh, h);
    // grid (S, LH, batch x (h/256)^2 quadrants; grouped W2 over batched weights: per-element tiles / slabs)
    const int qn = h / 256, nq = qn * qn;
    int s = blockIdx.x, ly = blockIdx.y, zz = blockIdx.z;
    if (nq > 1) {
        // the quadrants (qr, qc) of one (split, layer) read the same delta half qr / activation half qc: the blocks are
        // renumbered so that those nq blocks are consecutive slots of ONE XCD (blocks are dealt round-robin over the 8
        // XCDs; MI355X_MICROARCH.md) and run together, so each half comes from HBM once and is re-read from that
        // XCD's L2 (the quadrant-major grid re-read every half from HBM: traffic 2x the tiles)
        const unsigned total = gridDim.x * gridDim.y * gridDim.z;
        unsigned q = xcd_slot(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), total);
        const unsigned quad = q % (unsigned)nq;
        q /= (unsigned)nq;
        s = (int)(q % gridDim.x);
        q /= gridDim.x;
        ly = (int)(q % gridDim.y);
        zz = (int)((q / gridDim.y) * nq + quad);
    }
    const int l = ly + 1;
    const int qz = zz % nq, bz = zz / nq;
    const int qr = qz / qn, qc = qz % qn;
    abuf += bz * bstride_act;
    dbuf += bz * bstride_act;
    partial += bz * bstride_part;
    const int64_t tstride = (int64_t)h * 16;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane >> 4, i = lane & 15;
    const int wr = wave >> 1, wc = wave & 1;
    const int64_t T = n_pad / 16;
    const int64_t t0 = (int64_t)s * tps, t1 = t0 + tps < T ? t0 + tps : T;
    const float* dsrc = dbuf + (int64_t)l * n_pad * h + qr * WG_TILE_FLOATS;
    const float* asrc = abuf + (int64_t)(l - 1) * n_pad * h + qc * WG_TILE_FLOATS;
    const unsigned swz = wg_swz_off(lane);
    // f32x4 index of this lane's operand reads inside a ring slot (block rb / cb adds 64, 1 KiB)
    const int rd = i * 4 + ((g + (i >> 1)) & 3);
    const int ra = rd + 512 * wr;
    const int rbv = rd + WG_TILE_FLOATS / 4 + 512 * wc;
    const f32x4* rv = (const f32x4*)ring;

    f32x4 acc[8][8];
#pragma unroll
    for (int a = 0; a < 8; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // bias partial sums: lane (g, i) accumulates the value columns of delta row 128 wr + 16 rb + i among
    // coordinates 4g..4g+3 (jet tiles: column 4g only; two-stream tiles: 4g, 4g + 2)
    float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // JB 3 (qf_kernel.hpp Q8 tiles: 8 coordinates x 4 streams over a tile pair): the value columns are columns 0..7 of
    // the even tile of each pair, i.e. lane groups g < 2 of even tiles (mt, per tile)
    float mt = 1.f;
    auto bias_of = [&](const f32x4& v) -> float {
        if constexpr (JB == 1) return v[0];
        else if constexpr (JB == 2) return v[0] + v[2];
        else if constexpr (JB == 3) return mt * ((v[0] + v[2]) + (v[1] + v[3]));
        else return (v[0] + v[2]) + (v[1] + v[3]);
    };

    f32x4 av[8], bv[8];
    // Operands are reloaded for the next tile as soon as their last MFMA of this tile has issued: A block rb after
    // its 32 MFMAs, B block cb inside the last A block (cb pairs outermost there). One register set, one loop body
    // (a double-buffered B set with a two-body loop spilled: the 256 accumulators fill the AGPR file). The reads are
    // plain LDS loads through an f32x4 pointer (ds_read_b128; hipcc counts and places their waits itself, so no
    // register of an in-flight load is ever copied -- inline-asm reads are invisible to its bookkeeping,
    // tools/check_asm_waits.py), read slot (k + 1) % 3 unconditionally (stale data after the last tile is never
    // used), and sched_barrier(0) keeps each reload between its block's MFMAs and the next block's.
    auto block = [&](auto RB, int vn, auto BIAS) {
        constexpr int rb = decltype(RB)::value;
        const f32x4 v = av[rb];
        if constexpr (decltype(BIAS)::value == 1 + (rb & 1)) bs[rb] += bias_of(v);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int cb = 0; cb < 8; ++cb) acc[rb][cb] = mfma4(v[r], bv[cb][r], acc[rb][cb]);
        av[rb] = rv[vn + ra + rb * 64];
        __builtin_amdgcn_sched_barrier(0);
    };
    auto last_block = [&](int vn, auto BIAS) {
        const f32x4 v = av[7];
        if constexpr (decltype(BIAS)::value == 2) bs[7] += bias_of(v);
        av[7] = rv[vn + ra + 7 * 64];
        __builtin_amdgcn_sched_barrier(0);
        // cb pairs outermost (a dependent MFMA two issues behind clears the 16x16x4 f32 latency); B block cb is
        // reloaded after its pair
#define WG_PAIR(CB)                                                                    \
    {                                                                                  \
        _Pragma("unroll") for (int r = 0; r < 4; ++r) {                                \
            acc[7][CB] = mfma4(v[r], bv[CB][r], acc[7][CB]);                           \
            acc[7][CB + 1] = mfma4(v[r], bv[CB + 1][r], acc[7][CB + 1]);               \
        }                                                                              \
        bv[CB] = rv[vn + rbv + (CB) * 64];                                             \
        bv[CB + 1] = rv[vn + rbv + (CB + 1) * 64];                                     \
        __builtin_amdgcn_sched_barrier(0);                                             \
    }
        WG_PAIR(0)
        WG_PAIR(2)
        WG_PAIR(4)
        WG_PAIR(6)
#undef WG_PAIR
    };

    wg_issue(dsrc, asrc, ring, t0, t1, 0, wave, swz, tstride);
    wg_issue(dsrc, asrc, ring, t0 + 1, t1, 1, wave, swz, tstride);
    wg_issue(dsrc, asrc, ring, t0 + 2, t1, 2, wave, swz, tstride);
    if (t0 < t1) {
        if (t0 + 2 < t1)
            asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else if (t0 + 1 < t1)
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_barrier" ::: "memory");  // also a compiler barrier for the LDS loads
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            av[q] = rv[ra + q * 64];
            bv[q] = rv[rbv + q * 64];
        }
    }
    auto tiles = [&](auto BIAS) {
        int k = 0;
        for (int64_t t = t0; t < t1; ++t, ++k) {
            // tile t + 1 has landed (tile t + 2 may still be in flight); the barrier also retires every wave's reads of
            // slot k % 3 (tile t, in registers), which the issue of tile t + 3 overwrites
            if (t + 2 < t1)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_barrier" ::: "memory");  // also a compiler barrier for the LDS loads
            wg_issue(dsrc, asrc, ring, t + 3, t1, k + 3, wave, swz, tstride);
            if (JB == 3) mt = ((t & 1) == 0 && g < 2) ? 1.f : 0.f;
            const int vn = ((k + 1) % WG_NBUF) * (WG_SLOT / 4);
            block(std::integral_constant<int, 0>{}, vn, BIAS);
            block(std::integral_constant<int, 1>{}, vn, BIAS);
            block(std::integral_constant<int, 2>{}, vn, BIAS);
            block(std::integral_constant<int, 3>{}, vn, BIAS);
            block(std::integral_constant<int, 4>{}, vn, BIAS);
            block(std::integral_constant<int, 5>{}, vn, BIAS);
            block(std::integral_constant<int, 6>{}, vn, BIAS);
            last_block(vn, BIAS);
            // every read of this tile's slot is retired before the next barrier (the next issue overwrites it)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    };
    // bias blocks: the even ones summed by the column-half-0 wave, the odd ones by its column-half-1 partner (same delta
    // rows); BIAS = 0 none, 1 even blocks, 2 odd blocks
    if (!with_bias)
        tiles(std::integral_constant<int, 0>{});
    else if (wc == 0)
        tiles(std::integral_constant<int, 1>{});
    else
        tiles(std::integral_constant<int, 2>{});

    float* out = partial + (int64_t)s * P;
    float* dW = out + off.w(l);
#pragma unroll
    for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int cb = 0; cb < 8; ++cb)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                dW[(int64_t)(256 * qr + 128 * wr + 16 * rb + 4 * g + q) * h + 256 * qc + 128 * wc + 16 * cb + i] =
                    acc[rb][cb][q];
    // bias: the value columns of lane group g (jet tiles: columns 0, 4, 8, 12; two-stream tiles: 0, 2, ..., 14),
    // then the four groups of each row combined in a fixed order through the (now idle) ring
    __syncthreads();
#pragma unroll
    for (int rb = 0; rb < 8; ++rb)
        if ((rb & 1) == wc) ring[(128 * wr + 16 * rb + i) * 4 + g] = bs[rb];
    __syncthreads();
    if (qc == 0) {
        const float* rw = ring + threadIdx.x * 4;
        out[off.b(l) + 256 * qr + threadIdx.x] = with_bias ? (rw[0] + rw[1]) + (rw[2] + rw[3]) : 0.f;
    }
}

// ---- first / output layer gradients ("edge" layers: K = d_in or d_out, VALU) ------------------------------------
// grid (S): block s reduces the coordinate tiles of split s (the same split as wgrad_kernel); thread t owns
// neurons t, t + 256, ... The per-column scalars of a chunk of 16 tiles (x, gy / v / glap) are staged in LDS and
// read as broadcasts; the tile loop is unrolled so each thread keeps several 64 B row loads in flight (the first
// version walked one tile at a time and was latency-bound at 7x its HBM time).
//   EDGE_W2 : rows delta_0, a_L:            dW0 = delta_0^T x, db0 = sum delta_0, dWout = gy^T a_L, dbout = sum gy
//   EDGE_W3 : rows zb_0, zdb_0, adot_L:     dW0 = zdb_0^T v + zb_0^T x, db0 = sum zb_0, dWout = u^T adot_L
//             (u = output weighting, ones when NULL), dbout = 0
//             (+ with a first-order seed gy, rows a_L: dWout += gy^T a_L, dbout = sum gy)
//   EDGE_JET: rows zb_0 jet, a_L jet (16 columns = 4 coordinates x 4 streams, scalars per coordinate):
//             dW0[:, k] = sum zb_0,value x_k + zb_0,tangent k, db0 = sum zb_0,value, dWout = sum glap a_L,second
//   EDGE_MIX: the mixed jet (third-order adjoint, jet_kernel.hpp MIX): rows as EDGE_JET, scalars x, v (sc), g (sgy)
//             (n, d) and u (su, (n, o), NULL = ones): dW0[:, k] = sum zb_0,value x_k + zb_0,v v_k + zb_0,g g_k,
//             db0 = sum zb_0,value, dWout_j = sum u_j a_L,second, dbout = 0; sc / sgy == NULL: v = e_1 / g = e_2 (the
//             QUAD jet of a Hessian node: tangents along the coordinate axes)
//   EDGE_J2 : two-stream jet tiles (wide_jet_kernel.hpp: 16 columns = 8 coordinates x (value, tangent along v)),
//             rows zb_0 jet, a_L jet; scalars x, v (sc), gy (sgy, nullable), u (su, NULL = ones):
//             dW0[:, k] = sum zb_0,val x_k + zb_0,tan v_k, db0 = sum zb_0,val, dWout_j = sum gy_j a_L,val + u_j a_L,tan,
//             dbout_j = sum gy_j
//   EDGE_Q8 : the Hessian node's backward on Q8 tile pairs (qf_kernel.hpp: 8 coordinates x 4 streams over two 16-column
//             tiles; pair p = tiles 2p (value | d/dx_1) and 2p + 1 (d/dx_2 | Q stream)), tangents along the axes:
//             dW0[:, k] = sum zb_0,value x_k + zb_0,k, db0 = sum zb_0,value, dWout_j = sum u_j a_L,Q, dbout = 0
enum { EDGE_W2 = 0, EDGE_W3 = 1, EDGE_JET = 2, EDGE_MIX = 3, EDGE_J2 = 4, EDGE_Q8 = 5 };
constexpr int EDGE_CHUNK = 16;  // tiles per LDS staging chunk
// Thread groups per workgroup: group g walks its own quarter of the split's tile range (the split is the wgrad
// kernel's, so one workgroup per split: 42 of them at hidden 512) and the groups' per-neuron sums are combined in
// LDS in a fixed order (deterministic). One 256-thread group per split reached 1.6 TB/s at hidden 512 (DESIGN.md
// §3.11); four keep 4x the row loads in flight.
// The jet kinds keep ~120 VGPRs at four groups; EDGE_W2 / EDGE_W3 (16 column scalars and up to four row streams per
// tile) need their 256-VGPR budget, so they run two groups (512 threads).
constexpr int edge_groups(int kind) { return kind == 2 || kind == 3 || kind == 5 ? 4 : 2; }
constexpr int edge_threads(int kind) { return edge_groups(kind) * THREADS; }
constexpr int EDGE_ACC = 14;  // per-thread sums: gw0[4], gb0, gwo[4], gbo, gbj[4]

template <int KIND>
__global__ __launch_bounds__(edge_threads(KIND)) void edge_kernel(const float* __restrict__ r0, const float* __restrict__ r1,
                                                            const float* __restrict__ r2, const float* __restrict__ r3,
                                                            const float* __restrict__ x, const float* __restrict__ sc,
                                                            const float* __restrict__ sgy, const float* __restrict__ su,
                                                            int64_t n, int64_t ntiles,
                                                            int64_t tps, float* __restrict__ eslab, int64_t E, int d,
                                                            int o, int lh, int h, int64_t bstride_act = 0,
                                                            int64_t bstride_e = 0) {
    // per-column scalars of one chunk (per group): [col][0..3] = x (d_in <= 4), [col][4..7] = gy / v / glap,
    // [col][8..11] = the first-order seed gy (n, o) of a seeded W3 (sgy != nullptr: rows r3 = a_L add gy^T a_L to
    // dWout, sum gy to dbout) / EDGE_MIX's g, [col][12..15] = W3's / EDGE_MIX's output weighting u (n, o) (ones when
    // su == nullptr)
    constexpr bool JETK = KIND == EDGE_JET || KIND == EDGE_MIX;
    constexpr int EDGE_GROUPS = edge_groups(KIND);
    constexpr bool Q8 = KIND == EDGE_Q8;  // a "tile" is a Q8 tile pair (8 coordinates)
    constexpr int CPT = JETK ? 4 : (KIND == EDGE_J2 || Q8 ? 8 : 16);  // coordinates per tile
    constexpr int NSC = (KIND == EDGE_W3 || KIND == EDGE_MIX || KIND == EDGE_J2 || Q8) ? 16 : 9;
    constexpr int SCAL = EDGE_CHUNK * CPT * NSC;  // floats of one group's staging area
    constexpr int SMEM = EDGE_GROUPS * SCAL > EDGE_GROUPS * THREADS * EDGE_ACC ? EDGE_GROUPS * SCAL
                                                                              : EDGE_GROUPS * THREADS * EDGE_ACC;
    __shared__ __attribute__((aligned(16))) float smem[SMEM];
    const int grp = threadIdx.x / THREADS, tl = threadIdx.x % THREADS;
    float (*scal)[NSC] = (float (*)[NSC])(smem + grp * SCAL);
    const bool seeded = KIND == EDGE_W3 && sgy != nullptr;
    const bool weighted = KIND == EDGE_W3 && su != nullptr;
    const ParamOffsets off(d, o, lh, h);
    const int s = blockIdx.x;
    const int64_t t0 = (int64_t)s * tps, t1 = t0 + tps < ntiles ? t0 + tps : ntiles;
    // this group's quarter [g0, g1) of the split; every group runs the same number of chunk trips (barriers)
    const int64_t q = (t1 - t0 + EDGE_GROUPS - 1) / EDGE_GROUPS;
    const int64_t g0 = t0 + grp * q < t1 ? t0 + grp * q : t1, g1 = g0 + q < t1 ? g0 + q : t1;
    const int64_t trips = (q + EDGE_CHUNK - 1) / EDGE_CHUNK;
    if (gridDim.z > 1) {  // grouped over batched weights (EDGE_W2: W2, EDGE_W3: second order): grid.z = element
        const int64_t b = blockIdx.z;
        r0 += b * bstride_act;
        r1 += b * bstride_act;
        x += b * n * d;
        if constexpr (KIND == EDGE_W3) {
            r2 += b * bstride_act;
            if (r3 != nullptr) r3 += b * bstride_act;
            sc += b * n * d;  // v
            if (sgy != nullptr) sgy += b * n * o;
            if (su != nullptr) su += b * n * o;
        } else {
            sc += b * n * o;  // gy
        }
        eslab += b * bstride_e;
    }
    const int64_t tstride = (int64_t)h * 16 * (Q8 ? 2 : 1);
    const int ns = KIND == EDGE_W2 ? o : ((KIND == EDGE_W3 || KIND == EDGE_MIX || KIND == EDGE_J2) ? d : 1);
    // this split's compact edge slab: [W0 (h, d) | b0 (h) | Wout (o, h) | bout (o)] (edge_reduce_kernel maps it back
    // to the parameter order); grid.y = the 256-neuron block
    float* out = eslab + (int64_t)s * E;
    const int64_t ewo = off.hidden0, ebo = off.hidden0 + (int64_t)o * h;
    {
        const int tb = blockIdx.y * THREADS;
        const int t = tb + tl;
        float gw0[MAXD] = {0.f, 0.f, 0.f, 0.f}, gb0 = 0.f;
        float gwo[MAXO] = {0.f, 0.f, 0.f, 0.f}, gbo = 0.f, gbj[MAXO] = {0.f, 0.f, 0.f, 0.f};
        for (int64_t it = 0; it < trips; ++it) {
            const int64_t c0 = g0 + it * EDGE_CHUNK;
            const int nt = (int)(g1 - c0 < 0 ? 0 : (g1 - c0 < EDGE_CHUNK ? g1 - c0 : EDGE_CHUNK));
            __syncthreads();
            for (int e = tl; e < EDGE_CHUNK * CPT; e += THREADS) {
                const int64_t cd = c0 * CPT + e;
                const bool ok = e < nt * CPT && cd < n;
#pragma unroll
                for (int k = 0; k < MAXD; ++k) scal[e][k] = (ok && k < d) ? x[cd * d + k] : 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if ((KIND == EDGE_MIX && sc == nullptr) || Q8)  // QUAD (Hessian node): v = e_1 everywhere
                        scal[e][4 + j] = (ok && j == 0) ? 1.f : 0.f;
                    else
                        scal[e][4 + j] = (ok && j < ns) ? sc[cd * ns + j] : 0.f;
                }
                if constexpr (KIND == EDGE_W3) {
#pragma unroll
                    for (int j = 0; j < MAXO; ++j) {
                        scal[e][8 + j] = (ok && seeded && j < o) ? sgy[cd * o + j] : 0.f;
                        scal[e][12 + j] = weighted ? ((ok && j < o) ? su[cd * o + j] : 0.f) : 1.f;
                    }
                } else if constexpr (KIND == EDGE_J2) {
#pragma unroll
                    for (int j = 0; j < MAXO; ++j) {
                        scal[e][8 + j] = (ok && sgy != nullptr && j < o) ? sgy[cd * o + j] : 0.f;
                        scal[e][12 + j] = (ok && j < o) ? (su != nullptr ? su[cd * o + j] : 1.f) : 0.f;
                    }
                } else if constexpr (Q8) {
#pragma unroll
                    for (int j = 0; j < MAXO; ++j)
                        scal[e][12 + j] = (ok && j < o) ? (su != nullptr ? su[cd * o + j] : 1.f) : 0.f;
                } else if constexpr (KIND == EDGE_MIX) {
#pragma unroll
                    for (int k = 0; k < MAXD; ++k)  // QUAD: g = e_2 (d = 2) when sgy == nullptr
                        scal[e][8 + k] = (ok && k < d) ? (sgy != nullptr ? sgy[cd * d + k] : (k == 1 ? 1.f : 0.f)) : 0.f;
#pragma unroll
                    for (int j = 0; j < MAXO; ++j)
                        scal[e][12 + j] = (ok && j < o) ? (su != nullptr ? su[cd * o + j] : 1.f) : 0.f;
                } else {
                    scal[e][8] = 0.f;
                }
            }
            __syncthreads();
            if (t < h) {
#pragma unroll(JETK ? 8 : (KIND == EDGE_J2 || Q8 ? 2 : 1))
                for (int i = 0; i < nt; ++i) {
                    const int64_t tile = c0 + i;
                    if constexpr (Q8) {
                        // row t of tile 2p: value (cols 0..7) | zb d/dx_1 (8..15); tile 2p + 1: zb d/dx_2 (0..7) and
                        // the a_L jet's Q stream (r1, cols 8..15)
                        const f32x4* za = (const f32x4*)(r0 + tile * tstride + t * 16);
                        const f32x4* zc = (const f32x4*)(r0 + tile * tstride + h * 16 + t * 16);
                        const f32x4* aq = (const f32x4*)(r1 + tile * tstride + h * 16 + t * 16 + 8);
                        f32x4 zv[2], z1[2], z2[2], a3[2];
#pragma unroll
                        for (int hh = 0; hh < 2; ++hh) {
                            zv[hh] = za[hh];
                            z1[hh] = za[2 + hh];
                            z2[hh] = zc[hh];
                            a3[hh] = aq[hh];
                        }
#pragma unroll
                        for (int e = 0; e < 8; ++e) {
                            const float* sv = scal[i * 8 + e];
                            const float v0 = zv[e >> 2][e & 3];
                            gb0 += v0;
                            gw0[0] += v0 * sv[0] + z1[e >> 2][e & 3];
                            gw0[1] += v0 * sv[1] + z2[e >> 2][e & 3];
#pragma unroll
                            for (int j = 0; j < MAXO; ++j) gwo[j] += sv[12 + j] * a3[e >> 2][e & 3];
                        }
                        continue;
                    }
                    const f32x4* a = (const f32x4*)(r0 + tile * tstride + t * 16);
                    const f32x4* b = (const f32x4*)(r1 + tile * tstride + t * 16);
                    f32x4 av[4], bv[4], cv[4], ev[4];
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq) {
                        av[qq] = a[qq];
                        bv[qq] = b[qq];
                        if (KIND == EDGE_W3) cv[qq] = ((const f32x4*)(r2 + tile * tstride + t * 16))[qq];
                        if (KIND == EDGE_W3) ev[qq] = seeded ? ((const f32x4*)(r3 + tile * tstride + t * 16))[qq] : f32x4{};
                    }
#pragma unroll
                    for (int qq = 0; qq < 4; ++qq) {
                        if constexpr (KIND == EDGE_JET) {
                            // columns 4q..4q+3 = coordinate q of the tile, streams (value, d/dx1, d/dx2, second)
                            const float* sv = scal[i * 4 + qq];
                            gb0 += av[qq][0];
                            gw0[0] += av[qq][0] * sv[0] + av[qq][1];
                            gw0[1] += av[qq][0] * sv[1] + av[qq][2];
                            gwo[0] += sv[4] * bv[qq][3];
                        } else if constexpr (KIND == EDGE_J2) {
                            // columns 4qq + r: coordinate 2qq + r / 2, stream r & 1
#pragma unroll
                            for (int rr = 0; rr < 2; ++rr) {
                                const float* sv = scal[i * 8 + 2 * qq + rr];
                                const float zv = av[qq][2 * rr], zt = av[qq][2 * rr + 1];
                                const float av_ = bv[qq][2 * rr], at_ = bv[qq][2 * rr + 1];
                                gb0 += zv;
#pragma unroll
                                for (int k = 0; k < MAXD; ++k) gw0[k] += zv * sv[k] + zt * sv[4 + k];
#pragma unroll
                                for (int j = 0; j < MAXO; ++j) {
                                    gwo[j] += sv[8 + j] * av_ + sv[12 + j] * at_;
                                    gbj[j] += sv[8 + j];
                                }
                            }
                        } else if constexpr (KIND == EDGE_MIX) {
                            const float* sv = scal[i * 4 + qq];
                            gb0 += av[qq][0];
#pragma unroll
                            for (int k = 0; k < MAXD; ++k)
                                gw0[k] += av[qq][0] * sv[k] + av[qq][1] * sv[4 + k] + av[qq][2] * sv[8 + k];
#pragma unroll
                            for (int j = 0; j < MAXO; ++j) gwo[j] += sv[12 + j] * bv[qq][3];
                        } else {
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                const float* sv = scal[i * 16 + 4 * qq + r];
                                gb0 += av[qq][r];
                                if constexpr (KIND == EDGE_W2) {
#pragma unroll
                                    for (int k = 0; k < MAXD; ++k) gw0[k] += av[qq][r] * sv[k];
#pragma unroll
                                    for (int j = 0; j < MAXO; ++j) gwo[j] += sv[4 + j] * bv[qq][r];
                                    gbo += t < MAXO ? sv[4 + (t & 3)] : 0.f;
                                } else {
#pragma unroll
                                    for (int k = 0; k < MAXD; ++k) gw0[k] += cv[qq][r] * sv[4 + k] + av[qq][r] * sv[k];
#pragma unroll
                                    for (int j = 0; j < MAXO; ++j) {
                                        gwo[j] += sv[12 + j] * bv[qq][r] + sv[8 + j] * ev[qq][r];
                                        gbj[j] += sv[8 + j];
                                    }
                                }
                            }
                        }
                    }
                }
            }
        }
        // combine the groups' sums in a fixed order (the staging area is reused)
        __syncthreads();
        {
            float* red = smem + (grp * THREADS + tl) * EDGE_ACC;
#pragma unroll
            for (int k = 0; k < MAXD; ++k) red[k] = gw0[k];
            red[4] = gb0;
#pragma unroll
            for (int j = 0; j < MAXO; ++j) {
                red[5 + j] = gwo[j];
                red[10 + j] = gbj[j];
            }
            red[9] = gbo;
        }
        __syncthreads();
        if (grp == 0 && t < h) {
#pragma unroll
            for (int gg = 1; gg < EDGE_GROUPS; ++gg) {
                const float* red = smem + (gg * THREADS + tl) * EDGE_ACC;
#pragma unroll
                for (int k = 0; k < MAXD; ++k) gw0[k] += red[k];
                gb0 += red[4];
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    gwo[j] += red[5 + j];
                    gbj[j] += red[10 + j];
                }
                gbo += red[9];
            }
#pragma unroll
            for (int k = 0; k < MAXD; ++k)
                if (k < d) out[off.w0 + (int64_t)t * d + k] = gw0[k];
            out[off.b0 + t] = gb0;
            if constexpr (KIND == EDGE_W2) {
#pragma unroll
                for (int j = 0; j < MAXO; ++j)
                    if (j < o) out[ewo + (int64_t)j * h + t] = gwo[j];
                if (t < o) out[ebo + t] = gbo;
            } else if constexpr (KIND == EDGE_W3 || KIND == EDGE_J2) {
#pragma unroll
                for (int j = 0; j < MAXO; ++j) {
                    if (j < o) out[ewo + (int64_t)j * h + t] = gwo[j];
                    if (j < o && t == j) out[ebo + t] = gbj[j];
                }
            } else if constexpr (KIND == EDGE_MIX || Q8) {
#pragma unroll
                for (int j = 0; j < MAXO; ++j)
                    if (j < o) out[ewo + (int64_t)j * h + t] = gwo[j];
                if (t < o) out[ebo + t] = 0.f;
            } else {
                for (int j = 0; j < o; ++j) out[ewo + (int64_t)j * h + t] = gwo[0];
                if (t < o) out[ebo + t] = 0.f;
            }
        }
    }
}

// gp[i] = sum over the partial slabs for i in [begin, end); indices in [lo, hi) (the hidden layers' W/b) sum S + S2
// slabs, the others S.
__global__ void reduce_kernel(const float* __restrict__ partial, int64_t S, int64_t P, float* __restrict__ gp,
                              int64_t S2 = 0, int64_t lo = 0, int64_t hi = 0, int64_t bstride_part = 0,
                              int64_t begin = 0, int64_t end = -1) {
    partial += (int64_t)blockIdx.y * bstride_part;  // grouped: grid.y = batch element, gp rows of P
    gp += (int64_t)blockIdx.y * P;
    if (end < 0) end = P;
    for (int64_t idx = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < end;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t ns = (idx >= lo && idx < hi) ? S + S2 : S;
        // 8 independent partial sums keep 8 slab loads in flight per thread (one dependent chain was
        // latency-bound); the combine order is fixed, so the result stays deterministic
        float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        const float* col = partial + idx;
        int64_t s = 0;
        for (; s + 8 <= ns; s += 8) {
#pragma unroll
            for (int q = 0; q < 8; ++q) a[q] += col[(s + q) * P];
        }
        for (; s < ns; ++s) a[0] += col[s * P];
        gp[idx] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    }
}

// The edge layers' gradient: sum of the SE compact edge slabs (edge_kernel) into the parameter order: compact index
// c < hidden0 is W0 / b0 (parameter c), the rest Wout / bout (parameter wout + c - hidden0). grid.y = batch element.
// The slabs are few columns (E ~ 1 K) deep (SE ~ 512): 16 columns per workgroup with 16 threads each over interleaved
// slabs (8 loads in flight per thread), combined through LDS in a fixed order — one thread per column walking all
// slabs was a latency-bound 30 us per step (profiles/r04g_paths_summary.log).
__global__ __launch_bounds__(256) void edge_reduce_kernel(const float* __restrict__ eslab, int64_t SE, int64_t E,
                                                          int64_t hidden0, int64_t wout, float* __restrict__ gp,
                                                          int64_t P, int64_t bstride_e) {
    __shared__ float red[16][17];
    eslab += (int64_t)blockIdx.y * bstride_e;
    gp += (int64_t)blockIdx.y * P;
    const int cl = threadIdx.x & 15, k = threadIdx.x >> 4;
    const int64_t c = (int64_t)blockIdx.x * 16 + cl;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (c < E) {
        const float* col = eslab + c;
        int64_t s = k;
        for (; s + 7 * 16 < SE; s += 8 * 16) {
#pragma unroll
            for (int q = 0; q < 8; ++q) a[q] += col[(s + 16 * q) * E];
        }
        for (; s < SE; s += 16) a[0] += col[s * E];
    }
    red[k][cl] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (k == 0 && c < E) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) t += red[j][cl];
        gp[c < hidden0 ? c : wout + (c - hidden0)] = t;
    }
}

}  // namespace siren

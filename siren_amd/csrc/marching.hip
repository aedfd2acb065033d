// marching.hip — device marching cubes for sdf_meshing.create_mesh (the reference: skimage
// marching_cubes_lewiner on the host, sdf_meshing.py:97-102). The volume the W0 kernel just evaluated stays in HBM;
// three passes over it build an indexed, welded, oriented mesh:
//   mc_count_kernel   per grid point: crossings on its +x/+y/+z grid edges (popcount) and, per cell, the number of
//                     triangles of its case (mc_table.h, tools/gen_mc_table.py)
//   exclusive scans   of both counts (scan_*_kernel: 4096 items per workgroup, block sums scanned by one workgroup)
//                     -> vertex and triangle offsets, totals
//   mc_emit_kernel    vertices (linear interpolation along the grid edge, one per crossing: welded) and faces
//                     (cube edges -> owning grid point + axis -> vertex number)
// Everything is HBM-streaming integer / byte work on ~4 B per voxel per pass; no MFMA.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "launch.h"
#include "mc_table.h"

namespace siren {

namespace {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_PER_THREAD = 16;
constexpr int SCAN_ITEMS = SCAN_THREADS * SCAN_PER_THREAD;

struct Grid {
    int64_t X, Y, Z;
    __device__ __forceinline__ int64_t idx(int64_t i, int64_t j, int64_t k) const { return (i * Y + j) * Z + k; }
};

// crossing bits of the three grid edges leaving point (i, j, k) in +axis0 / +axis1 / +axis2
__device__ __forceinline__ unsigned edge_bits(const float* __restrict__ v, const Grid& g, int64_t i, int64_t j,
                                              int64_t k, float level) {
    const int64_t p = g.idx(i, j, k);
    const bool in0 = v[p] < level;
    unsigned b = 0;
    if (i + 1 < g.X && (v[p + g.Y * g.Z] < level) != in0) b |= 1u;
    if (j + 1 < g.Y && (v[p + g.Z] < level) != in0) b |= 2u;
    if (k + 1 < g.Z && (v[p + 1] < level) != in0) b |= 4u;
    return b;
}

// One thread per grid point: blockIdx.z = axis-0 index, blockIdx.y = axis-1 index, axis 2 across the workgroup
// (coalesced rows, no index division). The 8 corner values of the point's cell are loaded once and give both the
// point's edge crossings and the cell's case.
struct Point {
    int64_t i, j, k, p;
    bool ok, cell;
    unsigned eb;
    int m;
};

__device__ __forceinline__ Point classify(const float* __restrict__ v, const Grid& g, float level) {
    Point q;
    q.k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    q.j = blockIdx.y;
    q.i = blockIdx.z;
    q.ok = q.k < g.Z;
    q.eb = 0;
    q.m = 0;
    q.cell = false;
    if (!q.ok) return q;
    q.p = g.idx(q.i, q.j, q.k);
    const int64_t si = g.Y * g.Z, sj = g.Z;
    const bool hi = q.i + 1 < g.X, hj = q.j + 1 < g.Y, hk = q.k + 1 < g.Z;
    q.cell = hi && hj && hk;
    float c[8];
    c[0] = v[q.p];
    c[1] = hi ? v[q.p + si] : c[0];
    c[2] = hj ? v[q.p + sj] : c[0];
    c[4] = hk ? v[q.p + 1] : c[0];
    const bool in0 = c[0] < level;
    q.eb = ((c[1] < level) != in0 ? 1u : 0u) | ((c[2] < level) != in0 ? 2u : 0u) | ((c[4] < level) != in0 ? 4u : 0u);
    if (q.cell) {
        c[3] = v[q.p + si + sj];
        c[5] = v[q.p + si + 1];
        c[6] = v[q.p + sj + 1];
        c[7] = v[q.p + si + sj + 1];
#pragma unroll
        for (int t = 0; t < 8; ++t)
            if (c[t] < level) q.m |= 1 << t;
    }
    return q;
}

__global__ __launch_bounds__(256) void mc_count_kernel(const float* __restrict__ v, Grid g, float level,
                                                       uint32_t* __restrict__ vcount, uint32_t* __restrict__ tcount) {
    const Point q = classify(v, g, level);
    if (!q.ok) return;
    vcount[q.p] = __builtin_popcount(q.eb);
    tcount[q.p] = q.cell ? (uint32_t)kMcCount[q.m] : 0u;
}

__global__ __launch_bounds__(256) void mc_emit_kernel(const float* __restrict__ v, Grid g, float level, float sx,
                                                      float sy, float sz, const uint32_t* __restrict__ voff,
                                                      const uint32_t* __restrict__ toff, float* __restrict__ verts,
                                                      int32_t* __restrict__ faces) {
    const Point q = classify(v, g, level);
    if (!q.ok) return;
    if (q.eb != 0) {
        const float v0 = v[q.p];
        uint32_t o = voff[q.p];
        const int64_t step[3] = {g.Y * g.Z, g.Z, 1};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (!(q.eb >> a & 1u)) continue;
            const float t = (level - v0) / (v[q.p + step[a]] - v0);
            float* w = verts + 3 * (int64_t)o;
            w[0] = ((float)q.i + (a == 0 ? t : 0.f)) * sx;
            w[1] = ((float)q.j + (a == 1 ? t : 0.f)) * sy;
            w[2] = ((float)q.k + (a == 2 ? t : 0.f)) * sz;
            ++o;
        }
    }
    const int nt = q.cell ? kMcCount[q.m] : 0;
    if (nt == 0) return;
    int32_t* f = faces + 3 * (int64_t)toff[q.p];
    for (int s = 0; s < 3 * nt; ++s) {
        const int e = kMcTri[q.m][s];
        const int a = e >> 2, kk = e & 3;
        // the edge's lower corner: bit (a+1)%3 = kk & 1, bit (a+2)%3 = kk >> 1
        int64_t c[3] = {q.i, q.j, q.k};
        c[(a + 1) % 3] += kk & 1;
        c[(a + 2) % 3] += kk >> 1;
        const unsigned qb = edge_bits(v, g, c[0], c[1], c[2], level);
        f[s] = (int32_t)(voff[g.idx(c[0], c[1], c[2])] + __builtin_popcount(qb & ((1u << a) - 1u)));
    }
}

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t x, uint32_t* lds_waves, uint32_t& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= off) incl += y;
    }
    if (lane == 63) lds_waves[wave] = incl;
    __syncthreads();
    uint32_t base = 0;
    total = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        const uint32_t s = lds_waves[w];
        if (w < wave) base += s;
        total += s;
    }
    __syncthreads();
    return base + incl - x;
}

// per workgroup: sum of its SCAN_ITEMS items
__global__ __launch_bounds__(SCAN_THREADS) void scan_reduce_kernel(const uint32_t* __restrict__ d, int64_t n,
                                                                   uint32_t* __restrict__ bsum) {
    __shared__ uint32_t w[SCAN_THREADS / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_ITEMS;
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < SCAN_PER_THREAD; ++r) {
        const int64_t e = base + r * SCAN_THREADS + threadIdx.x;
        if (e < n) s += d[e];
    }
    uint32_t total;
    (void)block_exclusive_scan(s, w, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// one workgroup: exclusive scan of the nb block sums in place, the grand total at bsum[nb] — saturated to 0xffffffff
// when it reaches 2^31 (the offsets are uint32 and the faces int32: siren_mc_count then refuses the volume instead of
// emitting wrapped indices; one pass's total is <= 1024 x 4096 x 5 items, so the 64-bit carry is exact)
__global__ __launch_bounds__(1024) void scan_blocks_kernel(uint32_t* __restrict__ bsum, int64_t nb) {
    __shared__ uint32_t w[16];
    uint32_t carry = 0;
    uint64_t carry64 = 0;
    for (int64_t b0 = 0; b0 < nb; b0 += blockDim.x) {
        const int64_t e = b0 + threadIdx.x;
        const uint32_t x = e < nb ? bsum[e] : 0u;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(x, w, total);
        if (e < nb) bsum[e] = carry + ex;
        carry += total;
        carry64 += total;
    }
    if (threadIdx.x == 0) bsum[nb] = carry64 >= (1ull << 31) ? 0xffffffffu : carry;
}

// per workgroup: its items -> exclusive prefix (in place), offset by the scanned block sum
__global__ __launch_bounds__(SCAN_THREADS) void scan_apply_kernel(uint32_t* __restrict__ d, int64_t n,
                                                                  const uint32_t* __restrict__ bsum) {
    __shared__ uint32_t tile[SCAN_ITEMS];
    __shared__ uint32_t w[SCAN_THREADS / 64];
    const int64_t base = (int64_t)blockIdx.x * SCAN_ITEMS;
#pragma unroll
    for (int r = 0; r < SCAN_PER_THREAD; ++r) {  // coalesced into LDS
        const int64_t e = base + r * SCAN_THREADS + threadIdx.x;
        tile[r * SCAN_THREADS + threadIdx.x] = e < n ? d[e] : 0u;
    }
    __syncthreads();
    uint32_t loc[SCAN_PER_THREAD];
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < SCAN_PER_THREAD; ++r) {  // thread t owns items [16 t, 16 t + 16)
        loc[r] = s;
        s += tile[threadIdx.x * SCAN_PER_THREAD + r];
    }
    uint32_t total;
    const uint32_t off = bsum[blockIdx.x] + block_exclusive_scan(s, w, total);
#pragma unroll
    for (int r = 0; r < SCAN_PER_THREAD; ++r) tile[threadIdx.x * SCAN_PER_THREAD + r] = off + loc[r];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SCAN_PER_THREAD; ++r) {
        const int64_t e = base + r * SCAN_THREADS + threadIdx.x;
        if (e < n) d[e] = tile[r * SCAN_THREADS + threadIdx.x];
    }
}

int64_t scan_blocks(int64_t n) { return (n + SCAN_ITEMS - 1) / SCAN_ITEMS; }

void scan_u32(uint32_t* d, int64_t n, uint32_t* bsum, hipStream_t st) {
    const int64_t nb = scan_blocks(n);
    hipLaunchKernelGGL(scan_reduce_kernel, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, d, n, bsum);
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(1024), 0, st, bsum, nb);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nb), dim3(SCAN_THREADS), 0, st, d, n, bsum);
}

dim3 point_grid(int64_t X, int64_t Y, int64_t Z) {
    return dim3((unsigned)((Z + 255) / 256), (unsigned)Y, (unsigned)X);
}

}  // namespace

// workspace (uint32): [vertex counts -> offsets: P][triangle counts -> offsets: P][block sums x 2: nb + 1 each]
int64_t mc_ws_words(int64_t X, int64_t Y, int64_t Z) {
    const int64_t P = X * Y * Z;
    return 2 * P + 2 * (scan_blocks(P) + 1);
}

void mc_count(const float* vol, int64_t X, int64_t Y, int64_t Z, float level, uint32_t* ws, hipStream_t st) {
    const int64_t P = X * Y * Z, nb = scan_blocks(P);
    uint32_t* vc = ws;
    uint32_t* tc = ws + P;
    uint32_t* vb = ws + 2 * P;
    uint32_t* tb = vb + nb + 1;
    hipLaunchKernelGGL(mc_count_kernel, point_grid(X, Y, Z), dim3(256), 0, st, vol, Grid{X, Y, Z}, level, vc, tc);
    scan_u32(vc, P, vb, st);
    scan_u32(tc, P, tb, st);
}

const uint32_t* mc_totals(const uint32_t* ws, int64_t X, int64_t Y, int64_t Z, int which) {
    const int64_t P = X * Y * Z, nb = scan_blocks(P);
    return ws + 2 * P + (which == 0 ? nb : 2 * nb + 1);
}

void mc_emit(const float* vol, int64_t X, int64_t Y, int64_t Z, float level, const float* spacing,
             const uint32_t* ws, float* verts, int32_t* faces, hipStream_t st) {
    const int64_t P = X * Y * Z;
    hipLaunchKernelGGL(mc_emit_kernel, point_grid(X, Y, Z), dim3(256), 0, st, vol, Grid{X, Y, Z}, level, spacing[0],
                       spacing[1], spacing[2], ws, ws + P, verts, faces);
}

}  // namespace siren

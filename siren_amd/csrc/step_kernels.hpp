// step_kernels.hpp — the per-step work around the fused network kernels, for gfx950:
//   sample_sdf_kernel   dataio.PointCloud.__getitem__ (dataio.py:420-442) on the device: K random on-surface
//                       points (coords + normals gathered from the resident point cloud, sdf 0) and K uniform
//                       off-surface points in [-1, 1]^3 (normals -1, sdf -1), from a counter-based RNG, so the
//                       per-step host sampling and H2D copy (training.py:53-54) disappear.
//   sumsq_kernel +      torch.nn.utils.clip_grad_norm_ (training.py:98-102) + torch.optim.Adam.step
//   adam_kernel         (training.py:17, 104) over the flat parameter bucket: the global norm never leaves the
//                       device (no host sync), one pass reads g, m, v, p and writes m, v, p (16 B + 12 B / param).
// All three are HBM-bound streaming kernels: grid-stride loops, 16 B vector accesses where the layout allows.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launch.h"

namespace siren {

// splitmix64 finaliser over (seed, step, i): a stateless counter RNG (the oracle restates it bit for bit)
__host__ __device__ inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t rng_key(uint64_t seed, uint64_t step) { return mix64(seed ^ mix64(step)); }
__host__ __device__ inline uint64_t rng64(uint64_t seed, uint64_t step, uint64_t i) {
    return mix64(rng_key(seed, step) + i);
}
// 24 high bits -> [0, 1) exactly representable; 2u - 1 in [-1, 1)
__host__ __device__ inline float unit24(uint64_t h) { return (float)(h >> 40) * 5.9604644775390625e-08f; }

// Counter layout: on-surface point i draws index rng64(seed, step, i); off-surface point i draws its three
// coordinates from rng64(seed, step, k + 3 i + c), c = 0..2. Index = floor(r * m / 2^64) (multiply-high: unbiased
// to 2^-64 / m, no modulo).
// key = rng_key(seed, step), hoisted to the host: one mix64 per random word in the kernel
__global__ void sample_sdf_kernel(const float* __restrict__ pc, const float* __restrict__ pn, int64_t m, int64_t k,
                                  uint64_t key, float* __restrict__ coords,
                                  float* __restrict__ normals, float* __restrict__ sdf) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * k; i += (int64_t)gridDim.x * blockDim.x) {
        float c[3], nv[3], s;
        if (i < k) {
            const uint64_t r = mix64(key + (uint64_t)i);
            const int64_t idx = (int64_t)__umul64hi(r, (uint64_t)m);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                c[q] = pc[idx * 3 + q];
                nv[q] = pn[idx * 3 + q];
            }
            s = 0.f;
        } else {
            const int64_t j = i - k;
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                c[q] = 2.f * unit24(mix64(key + (uint64_t)(k + 3 * j + q))) - 1.f;
                nv[q] = -1.f;
            }
            s = -1.f;
        }
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            coords[i * 3 + q] = c[q];
            normals[i * 3 + q] = nv[q];
        }
        sdf[i] = s;
    }
}

constexpr int STEP_THREADS = 256;  // STEP_BLOCKS (norm partials) lives in launch.h: the C ABI sizes scratch by it

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    float t = 0.f;
    for (int w = 0; w < STEP_THREADS / 64; ++w) t += red[w];
    return t;
}

// partial[b] = sum of g^2 over block b's grid-stride share
__global__ __launch_bounds__(STEP_THREADS) void sumsq_kernel(const float* __restrict__ g, int64_t p,
                                                             float* __restrict__ partial) {
    __shared__ float red[STEP_THREADS / 64];
    float acc = 0.f;
    const int64_t p4 = p / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p4; i += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = ((const float4*)g)[i];
        acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int64_t i = 4 * p4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < p; i += (int64_t)gridDim.x * blockDim.x)
        acc += g[i] * g[i];
    const float t = block_sum(acc, red);
    if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

// Adam (torch.optim.Adam, amsgrad off, no weight decay) with the clip coefficient of clip_grad_norm_:
//   c = min(1, max_norm / (||g|| + 1e-6)) (c = 1 when max_norm <= 0), g' = c g,
//   m = m + (1 - b1)(g' - m), v = b2 v + (1 - b2) g'^2, p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps)
// (torch's op order: lerp for m, mul + addcmul for v, sqrt(v) / sqrt(bc2) + eps, addcdiv)
__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float c, float b1, float b2, float step,
                                      float sqrt_bc2, float eps) {
    g *= c;
    m = m + (1.f - b1) * (g - m);
    v = b2 * v + (1.f - b2) * (g * g);
    p = p + (-step) * (m / (__builtin_sqrtf(v) / sqrt_bc2 + eps));
}

__global__ __launch_bounds__(STEP_THREADS) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                            float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                            const float* __restrict__ partial, int nparts, float lr,
                                                            float b1, float b2, float eps, float bc1, float bc2,
                                                            float max_norm, float* __restrict__ norm_out) {
    __shared__ float red[STEP_THREADS / 64];
    float c = 1.f;
    if (partial != nullptr) {
        float acc = 0.f;
        for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += partial[i];
        const float norm = __builtin_sqrtf(block_sum(acc, red));
        if (max_norm > 0.f) c = fminf(1.f, max_norm / (norm + 1e-6f));
        if (norm_out != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *norm_out = norm;
    }
    const float step = lr / bc1, isb = __builtin_sqrtf(bc2);
    const int64_t n4 = n / 4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
        float4 pv = ((float4*)p)[i], mv = ((float4*)m)[i], vv = ((float4*)v)[i];
        const float4 gv = ((const float4*)g)[i];
        adam1(pv.x, gv.x, mv.x, vv.x, c, b1, b2, step, isb, eps);
        adam1(pv.y, gv.y, mv.y, vv.y, c, b1, b2, step, isb, eps);
        adam1(pv.z, gv.z, mv.z, vv.z, c, b1, b2, step, isb, eps);
        adam1(pv.w, gv.w, mv.w, vv.w, c, b1, b2, step, isb, eps);
        ((float4*)p)[i] = pv;
        ((float4*)m)[i] = mv;
        ((float4*)v)[i] = vv;
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        adam1(p[i], g[i], m[i], v[i], c, b1, b2, step, isb, eps);
}

}  // namespace siren

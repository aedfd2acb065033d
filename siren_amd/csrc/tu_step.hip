// tu_step.hip — per-step kernels around the network: device point-cloud sampling, clip + Adam.
#include "launch.h"
#include <algorithm>

#include "step_kernels.hpp"

namespace siren {

void launch_sample_sdf(hipStream_t st, const float* pc, const float* pn, int64_t m, int64_t k, uint64_t seed,
                       uint64_t step, float* coords, float* normals, float* sdf) {
    const int64_t blocks = std::min<int64_t>((2 * k + 255) / 256, 8192);
    hipLaunchKernelGGL(sample_sdf_kernel, dim3((unsigned)blocks), dim3(256), 0, st, pc, pn, m, k, rng_key(seed, step),
                       coords, normals, sdf);
}

void launch_adam(hipStream_t st, float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                 float eps, float bc1, float bc2, float max_norm, float* scratch) {
    const int64_t want = (n / 4 + STEP_THREADS - 1) / STEP_THREADS;
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>(want, STEP_BLOCKS));
    if (max_norm > 0.f) {
        hipLaunchKernelGGL(sumsq_kernel, dim3(STEP_BLOCKS), dim3(STEP_THREADS), 0, st, g, n, scratch);
        hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(STEP_THREADS), 0, st, p, g, m, v, n, (const float*)scratch,
                           STEP_BLOCKS, lr, b1, b2, eps, bc1, bc2, max_norm, scratch + STEP_BLOCKS);
    } else {
        hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(STEP_THREADS), 0, st, p, g, m, v, n, (const float*)nullptr,
                           0, lr, b1, b2, eps, bc1, bc2, 0.f, (float*)nullptr);
    }
}

}  // namespace siren

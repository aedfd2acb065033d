// Microbenchmark: cycles per v_mfma_f32_16x16x4_f32 of the runtime-loop kernels' slice GEMM (lds_ops.h slice_mma:
// 16 output blocks x 4 K-steps per 16 KiB slice, A operands by ds_read_b128 one block pair ahead, counted lgkmcnt)
// against the same MFMA stream with register operands, with and without a workgroup barrier per slice, at one and two
// waves per SIMD (one / two 256-thread workgroups per CU). The slice stays resident in LDS (no global traffic).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I siren_amd/csrc tools/micro/slice_loop.hip -o /tmp/slice_loop
#include <hip/hip_runtime.h>
#include <cstdio>

#include "lds_ops.h"

using namespace siren;

template <int MODE, bool BAR>  // MODE 0: slice_mma (LDS operands); 1: register operands
__global__ __launch_bounds__(256, 2) void k(float* out, long long* cyc, int iters) {
    __shared__ __attribute__((aligned(16))) float lds[4 * 4096];
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4 * 4096; i += 256) lds[i] = 1e-3f * (i & 255);
    __syncthreads();
    f32x4 acc[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) acc[b] = f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 bop = {1.f, 0.5f, 0.25f, 0.125f};
    f32x4 ra0 = {lane * 1e-3f, 1.f, 2.f, 3.f}, ra1 = ra0 + 1.f;
    const unsigned va = lds_addr(lds) + 16u * lane;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (BAR) __builtin_amdgcn_s_barrier();
        if constexpr (MODE == 0) {
            slice_mma<16>(va, bop, acc);
        } else {
#pragma unroll
            for (int p = 0; p < 8; ++p)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    acc[2 * p] = mfma4(ra0[r], bop[r], acc[2 * p]);
                    acc[2 * p + 1] = mfma4(ra1[r], bop[r], acc[2 * p + 1]);
                }
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
#pragma unroll
    for (int b = 0; b < 16; ++b) s += acc[b][0] + acc[b][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, bool BAR>
void run(const char* name, int wgs_per_cu, float* out, long long* cyc, long long* h) {
    const int iters = 4000, blocks = 256 * wgs_per_cu;
    hipLaunchKernelGGL((k<MODE, BAR>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    hipLaunchKernelGGL((k<MODE, BAR>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += h[i];
    // per SIMD: wgs_per_cu waves share it, so the SIMD's cycles per MFMA = wave time / (wgs_per_cu * MFMAs per wave)
    printf("%-28s %d wave/SIMD: %.1f SIMD cycles per MFMA (ideal 32)\n", name, wgs_per_cu,
           s / blocks / (64.0 * iters) / wgs_per_cu);
}

int main() {
    float* out;
    long long *cyc, h[512];
    hipMalloc(&out, 512 * 256 * sizeof(float));
    hipMalloc(&cyc, 512 * sizeof(long long));
    for (int w = 1; w <= 2; ++w) {
        run<1, false>("register operands", w, out, cyc, h);
        run<1, true>("register operands + barrier", w, out, cyc, h);
        run<0, false>("slice_mma (LDS operands)", w, out, cyc, h);
        run<0, true>("slice_mma + barrier", w, out, cyc, h);
    }
    return 0;
}

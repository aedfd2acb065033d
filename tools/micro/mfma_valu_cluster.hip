// Microbenchmark: does the cost of VALU work next to v_mfma_f32_16x16x4_f32 depend on how it is grouped?
// Per iteration: 8 MFMAs (two accumulation chains) and 8*F independent v_fma_f32, either one group of F after every
// MFMA (interleaved, as mfma_valu_overlap.hip) or all 8*F in ONE cluster after the 8 MFMAs, or in two clusters of 4*F.
// One wave per SIMD, 4 waves per CU, every CU. Prints cycles per MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MF(ACC) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(ACC) : "v"(a), "v"(b));
#define FL(X) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(X) : "v"(b), "v"(a));

template <int N>
__device__ __forceinline__ void fill(float& f0, float& f1, float& f2, float& f3, float& f4, float& f5, float a, float b) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        switch (i % 6) {
            case 0: FL(f0) break;
            case 1: FL(f1) break;
            case 2: FL(f2) break;
            case 3: FL(f3) break;
            case 4: FL(f4) break;
            default: FL(f5) break;
        }
    }
}

// MODE 0: F after every MFMA; 1: 8F after the 8 MFMAs; 2: 4F after MFMA 4 and 4F after MFMA 8
template <int F, int MODE>
__global__ __launch_bounds__(256) void k(float* out, long long* cyc, int iters) {
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    float f0 = a, f1 = a + 1, f2 = a + 2, f3 = a + 3, f4 = a + 4, f5 = a + 5;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            MF(acc0) fill<F>(f0, f1, f2, f3, f4, f5, a, b); MF(acc1) fill<F>(f0, f1, f2, f3, f4, f5, a, b);
            MF(acc0) fill<F>(f0, f1, f2, f3, f4, f5, a, b); MF(acc1) fill<F>(f0, f1, f2, f3, f4, f5, a, b);
            MF(acc0) fill<F>(f0, f1, f2, f3, f4, f5, a, b); MF(acc1) fill<F>(f0, f1, f2, f3, f4, f5, a, b);
            MF(acc0) fill<F>(f0, f1, f2, f3, f4, f5, a, b); MF(acc1) fill<F>(f0, f1, f2, f3, f4, f5, a, b);
        } else if (MODE == 1) {
            MF(acc0) MF(acc1) MF(acc0) MF(acc1) MF(acc0) MF(acc1) MF(acc0) MF(acc1)
            fill<8 * F>(f0, f1, f2, f3, f4, f5, a, b);
        } else {
            MF(acc0) MF(acc1) MF(acc0) MF(acc1) fill<4 * F>(f0, f1, f2, f3, f4, f5, a, b);
            MF(acc0) MF(acc1) MF(acc0) MF(acc1) fill<4 * F>(f0, f1, f2, f3, f4, f5, a, b);
        }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc0[0] + acc1[1] + f0 + f1 + f2 + f3 + f4 + f5;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int F, int MODE>
void run(float* out, long long* cyc, long long* h) {
    const int iters = 2000, blocks = 256;
    hipLaunchKernelGGL((k<F, MODE>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    hipLaunchKernelGGL((k<F, MODE>), dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += h[i];
    const char* nm[] = {"interleaved (F after each MFMA)", "one cluster of 8F per 8 MFMAs", "two clusters of 4F"};
    printf("F=%2d %-34s %.1f cycles per MFMA\n", F, nm[MODE], s / blocks / (8.0 * iters));
}

int main() {
    float* out;
    long long *cyc, h[256];
    hipMalloc(&out, 256 * 256 * sizeof(float));
    hipMalloc(&cyc, 256 * sizeof(long long));
    run<0, 0>(out, cyc, h);
    run<1, 0>(out, cyc, h); run<1, 1>(out, cyc, h); run<1, 2>(out, cyc, h);
    run<2, 0>(out, cyc, h); run<2, 1>(out, cyc, h); run<2, 2>(out, cyc, h);
    run<4, 0>(out, cyc, h); run<4, 1>(out, cyc, h); run<4, 2>(out, cyc, h);
    return 0;
}

// Microbenchmark: can one wave issue VALU in the shadow of its own v_mfma_f32_16x16x4_f32 on gfx950?
// Each iteration: 8 MFMAs (two accumulation chains), each followed by F independent v_fma_f32 fillers, all in one
// asm block (no compiler scheduling). Prints cycles per MFMA for F = 0..12 (one wave per SIMD, 4 waves per CU).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int F>
__global__ __launch_bounds__(256) void k(float* out, long long* cyc, int iters) {
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    float a = threadIdx.x * 1e-3f, b = 1.0001f;
    float f0 = a, f1 = a + 1, f2 = a + 2, f3 = a + 3, f4 = a + 4, f5 = a + 5;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#define MF(ACC) asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(ACC) : "v"(a), "v"(b));
#define FL(X) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(X) : "v"(b), "v"(a));
#define FILL                                                   \
    if (F > 0) FL(f0) if (F > 1) FL(f1) if (F > 2) FL(f2)      \
    if (F > 3) FL(f3) if (F > 4) FL(f4) if (F > 5) FL(f5)      \
    if (F > 6) FL(f0) if (F > 7) FL(f1) if (F > 8) FL(f2)      \
    if (F > 9) FL(f3) if (F > 10) FL(f4) if (F > 11) FL(f5)
        MF(acc0) FILL MF(acc1) FILL MF(acc0) FILL MF(acc1) FILL
        MF(acc0) FILL MF(acc1) FILL MF(acc0) FILL MF(acc1) FILL
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc0[0] + acc1[1] + f0 + f1 + f2 + f3 + f4 + f5;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int F>
void run(float* out, long long* cyc, long long* h) {
    const int iters = 2000, blocks = 256;
    hipLaunchKernelGGL(k<F>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k<F>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters);
    hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += h[i];
    printf("F=%2d fillers per MFMA: %.1f cycles per MFMA (ideal 32 if hidden, %d if serial at 4/VALU)\n", F,
           s / blocks / (8.0 * iters), 32 + 4 * F);
}

int main() {
    float* out;
    long long *cyc, h[256];
    hipMalloc(&out, 256 * 256 * sizeof(float));
    hipMalloc(&cyc, 256 * sizeof(long long));
    run<0>(out, cyc, h);
    run<1>(out, cyc, h);
    run<2>(out, cyc, h);
    run<3>(out, cyc, h);
    run<4>(out, cyc, h);
    run<6>(out, cyc, h);
    run<8>(out, cyc, h);
    run<12>(out, cyc, h);
    return 0;
}

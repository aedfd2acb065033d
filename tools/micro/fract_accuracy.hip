// Micro-test: v_sin_f32 / v_cos_f32 of a phase u in revolutions (the phase-scaled pack's accumulators), reduced by
// u - rint(u) (two VALU: sincos_rev) against v_fract_f32 (one VALU), vs fp64 sin(2 pi u) of the same fp32 u.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__global__ void k(const float* t, float* s, float* c, float* s2, float* c2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float u = t[i];
    const float r = u - __builtin_rintf(u);
    s[i] = __builtin_amdgcn_sinf(r);
    c[i] = __builtin_amdgcn_cosf(r);
    const float f = __builtin_amdgcn_fractf(u);
    s2[i] = __builtin_amdgcn_sinf(f);
    c2[i] = __builtin_amdgcn_cosf(f);
}
int main() {
    const int n = 1 << 24;
    std::vector<float> t(n);
    for (int i = 0; i < n; ++i) t[i] = -128.f + 256.f * (float)i / n;
    t[0] = -1e-30f; t[1] = -1e-8f; t[2] = 1e-8f; t[3] = -0.f; t[4] = 0.5f; t[5] = -0.5f; t[6] = 0.99999994f;
    float *dt, *ds, *dc, *ds2, *dc2;
    hipMalloc(&dt, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&ds2, n * 4); hipMalloc(&dc2, n * 4);
    hipMemcpy(dt, t.data(), n * 4, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dt, ds, dc, ds2, dc2, n);
    std::vector<float> s(n), c(n), s2(n), c2(n);
    hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(s2.data(), ds2, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(c2.data(), dc2, n * 4, hipMemcpyDeviceToHost);
    double es = 0, ec = 0, es2 = 0, ec2 = 0, ms = 0, mc = 0;
    long nd = 0;
    for (int i = 0; i < n; ++i) {
        const double x = 2.0 * M_PI * (double)t[i];
        es = fmax(es, fabs(s[i] - sin(x))); ec = fmax(ec, fabs(c[i] - cos(x)));
        es2 = fmax(es2, fabs(s2[i] - sin(x))); ec2 = fmax(ec2, fabs(c2[i] - cos(x)));
        ms += fabs(s[i] - sin(x)); mc += fabs(s2[i] - sin(x));
        nd += (s[i] != s2[i]) || (c[i] != c2[i]);
    }
    printf("u - rint(u): sin max abs err %.3e cos %.3e mean(sin) %.3e | fract(u): sin %.3e cos %.3e mean(sin) %.3e | "
           "bitwise different %ld of %d\n", es, ec, ms / n, es2, ec2, mc / n, nd, n);
    return 0;
}

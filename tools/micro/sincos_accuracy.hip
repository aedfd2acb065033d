// Micro-test: sin/cos of a fp32 phase t in radians (t = fl(w z), the unscaled kernels' epilogues) by the Cody-Waite
// reduction (sincos_fast up to round 5: 5 VALU) and by the one-rounding reduction in revolutions (round 6: 3 VALU),
// both on v_sin_f32 / v_cos_f32, vs fp64 sin / cos of the same fp32 t; and the error the argument's own rounding already
// carries (fp64 sin(w z) vs sin(fl(w z)) for w = 30 and z = t / 30), the reference's fl(30 z) (modules.py:34).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__global__ void k(const float* t, float* s, float* c, float* s2, float* c2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float x = t[i];
    const float q = __builtin_rintf(x * 0.159154943091895336f);
    float r = __builtin_fmaf(-q, 6.28318548202514648f, x);
    r = __builtin_fmaf(-q, -1.74845553146951e-7f, r);
    const float u = r * 0.159154943091895336f;
    s[i] = __builtin_amdgcn_sinf(u);
    c[i] = __builtin_amdgcn_cosf(u);
    const float v = x * 0.159154943091895336f;
    const float u2 = v - __builtin_rintf(v);
    s2[i] = __builtin_amdgcn_sinf(u2);
    c2[i] = __builtin_amdgcn_cosf(u2);
}
int main() {
    const int n = 1 << 24;
    std::vector<float> t(n);
    for (int i = 0; i < n; ++i) t[i] = -100.f + 200.f * (float)i / n;
    float *dt, *ds, *dc, *ds2, *dc2;
    (void)hipMalloc(&dt, n * 4); (void)hipMalloc(&ds, n * 4); (void)hipMalloc(&dc, n * 4);
    (void)hipMalloc(&ds2, n * 4); (void)hipMalloc(&dc2, n * 4);
    (void)hipMemcpy(dt, t.data(), n * 4, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dt, ds, dc, ds2, dc2, n);
    std::vector<float> s(n), c(n), s2(n), c2(n);
    (void)hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(s2.data(), ds2, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(c2.data(), dc2, n * 4, hipMemcpyDeviceToHost);
    double es = 0, ec = 0, es2 = 0, ec2 = 0, ea = 0;
    for (int i = 0; i < n; ++i) {
        const double x = (double)t[i];
        es = fmax(es, fabs(s[i] - sin(x))); ec = fmax(ec, fabs(c[i] - cos(x)));
        es2 = fmax(es2, fabs(s2[i] - sin(x))); ec2 = fmax(ec2, fabs(c2[i] - cos(x)));
        const double z = x / 30.0;                       // a pre-activation whose fp32 phase is t
        ea = fmax(ea, fabs(sin((double)(float)(30.0f * (float)z)) - sin(30.0 * (double)(float)z)));
    }
    printf("|t| <= 100 rad: Cody-Waite sin %.3e cos %.3e | revolutions sin %.3e cos %.3e | argument rounding "
           "fl(30 z) alone %.3e\n", es, ec, es2, ec2, ea);
    return 0;
}

// Micro-test: accuracy of v_sin_f32 / v_cos_f32 (input in revolutions) after Cody-Waite reduction, vs fp64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
__global__ void k(const float* t, float* s, float* c, float* s2, float* c2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x = t[i];
  float q = __builtin_rintf(x * 0.159154943091895336f);           // revolutions
  float r = __builtin_fmaf(-q, 6.28125f, x);
  r = __builtin_fmaf(-q, 1.9353071795864769253e-3f, r);
  r = __builtin_fmaf(-q, 3.0199e-11f, r);
  float rv = r * 0.159154943091895336f;
  s[i] = __builtin_amdgcn_sinf(rv);
  c[i] = __builtin_amdgcn_cosf(rv);
  s2[i] = __builtin_amdgcn_sinf(x * 0.159154943091895336f);       // no reduction
  c2[i] = __builtin_amdgcn_cosf(x * 0.159154943091895336f);
}
int main() {
  const int n = 1 << 22;
  std::vector<float> t(n);
  for (int i = 0; i < n; ++i) t[i] = -100.f + 200.f * (float)i / n;
  float *dt, *ds, *dc, *ds2, *dc2;
  hipMalloc(&dt, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&ds2, n * 4); hipMalloc(&dc2, n * 4);
  hipMemcpy(dt, t.data(), n * 4, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dt, ds, dc, ds2, dc2, n);
  std::vector<float> s(n), c(n), s2(n), c2(n);
  hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost); hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(s2.data(), ds2, n * 4, hipMemcpyDeviceToHost); hipMemcpy(c2.data(), dc2, n * 4, hipMemcpyDeviceToHost);
  double es = 0, ec = 0, es2 = 0, ec2 = 0, ef = 0;
  for (int i = 0; i < n; ++i) {
    double x = t[i];
    es = fmax(es, fabs(s[i] - sin(x))); ec = fmax(ec, fabs(c[i] - cos(x)));
    es2 = fmax(es2, fabs(s2[i] - sin(x))); ec2 = fmax(ec2, fabs(c2[i] - cos(x)));
    ef = fmax(ef, fabs((double)sinf((float)x) - sin(x)));
  }
  printf("reduced v_sin max abs err %.3e  v_cos %.3e | unreduced v_sin %.3e v_cos %.3e | host sinf %.3e\n", es, ec, es2, ec2, ef);
  return 0;
}

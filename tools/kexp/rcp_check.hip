// rcp_check.hip -- accuracy of v_rcp_f64 alone and after one / two Newton steps (not product code).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__global__ void k(const double* x, double* r0, double* r1, double* r2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double d = x[i];
  double r = __builtin_amdgcn_rcp(d);
  r0[i] = r;
  r = fma(r, fma(-d, r, 1.0), r);
  r1[i] = r;
  r2[i] = fma(r, fma(-d, r, 1.0), r);
}
int main() {
  const int n = 1 << 20;
  std::vector<double> x(n);
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    x[i] = std::ldexp(1.0 + (double)(s >> 11) * 0x1.0p-53, (int)(s % 60) - 10);
  }
  double *dx, *d0, *d1, *d2;
  hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, d0, d1, d2, n);
  std::vector<double> r0(n), r1(n), r2(n);
  hipMemcpy(r0.data(), d0, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r1.data(), d1, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r2.data(), d2, n * 8, hipMemcpyDeviceToHost);
  double e0 = 0, e1 = 0, e2 = 0;
  for (int i = 0; i < n; ++i) {
    const long double ex = 1.0L / (long double)x[i];
    e0 = std::fmax(e0, (double)std::fabs((r0[i] - ex) / ex));
    e1 = std::fmax(e1, (double)std::fabs((r1[i] - ex) / ex));
    e2 = std::fmax(e2, (double)std::fabs((r2[i] - ex) / ex));
  }
  printf("v_rcp_f64 max rel err: raw %.3e  1 NR %.3e  2 NR %.3e  (2^-52 = %.3e)\n", e0, e1, e2, std::ldexp(1.0, -52));
  return 0;
}

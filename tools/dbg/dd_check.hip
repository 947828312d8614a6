// Diagnostic: large by-value kernel args + double-double primitives on device vs host.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#pragma clang fp contract(off)
struct dd { double hi, lo; };
struct cdd { dd re, im; };
__host__ __device__ inline dd two_sum(double a, double b) { const double s = a + b, bb = s - a; return {s, (a - (s - bb)) + (b - bb)}; }
__host__ __device__ inline dd quick_two_sum(double a, double b) { const double s = a + b; return {s, b - (s - a)}; }
__host__ __device__ inline dd dd_add(dd x, dd y) { dd s = two_sum(x.hi, y.hi), t = two_sum(x.lo, y.lo); s.lo += t.hi; s = quick_two_sum(s.hi, s.lo); s.lo += t.lo; return quick_two_sum(s.hi, s.lo); }
__host__ __device__ inline dd dd_mul(dd x, dd y) { const double p = x.hi * y.hi; double e = fma(x.hi, y.hi, -p); e += x.hi * y.lo + x.lo * y.hi; return quick_two_sum(p, e); }
#pragma clang fp contract(on)
struct Big { long long C, M, dec; cdd Vi[16]; cdd l[16]; };
__global__ void k(const Big f, double* out) {
  if (threadIdx.x) return;
  out[0] = f.Vi[0].re.hi; out[1] = f.Vi[0].re.lo; out[2] = f.Vi[15].im.hi; out[3] = f.l[15].im.lo; out[4] = (double)f.dec;
  dd a = {1.0 / 3.0, 1.8503717077085943e-17}, b = {3.14159265358979, 1.2e-16};
  dd s = dd_add(a, b), p = dd_mul(a, b);
  out[5] = s.hi; out[6] = s.lo; out[7] = p.hi; out[8] = p.lo;
}
int main() {
  Big f; f.C = 1; f.M = 2; f.dec = 1000;
  for (int i = 0; i < 16; ++i) { f.Vi[i] = {{i + 0.5, i * 1e-20}, {-i - 0.25, i * 2e-20}}; f.l[i] = {{i * 1.0, 0}, {0, i * 3e-20}}; }
  double* d; hipMalloc(&d, 64 * 8); double h[16];
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, f, d);
  hipMemcpy(h, d, 16 * 8, hipMemcpyDeviceToHost);
  printf("args: %g %g %g %g %g (want 0.5 0 -15.25 4.5e-19 1000)\n", h[0], h[1], h[2], h[3], h[4]);
  dd a = {1.0 / 3.0, 1.8503717077085943e-17}, b = {3.14159265358979, 1.2e-16};
  dd s = dd_add(a, b), p = dd_mul(a, b);
  printf("dd dev: %.17g %.5g %.17g %.5g\n", h[5], h[6], h[7], h[8]);
  printf("dd host: %.17g %.5g %.17g %.5g\n", s.hi, s.lo, p.hi, p.lo);
  return 0;
}

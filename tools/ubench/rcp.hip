// Microbenchmark (diagnostic tool): accuracy of the gfx950 fp64 hardware
// reciprocal / reciprocal-sqrt and of 0-3 Newton steps, in ulps against the
// correctly rounded host result, over log-uniform inputs.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

__global__ void k(const double* x, double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double b = x[i];
  double r = __builtin_amdgcn_rcp(b);
  out[8 * i + 0] = r;
  r = fma(r, fma(-b, r, 1.0), r);
  out[8 * i + 1] = r;
  r = fma(r, fma(-b, r, 1.0), r);
  out[8 * i + 2] = r;
  r = fma(r, fma(-b, r, 1.0), r);
  out[8 * i + 3] = r;
  const double y = __builtin_amdgcn_rsq(b);
  out[8 * i + 4] = y;
  // sqrt from rsq with one Goldschmidt/Newton refinement pair (as fsqrt_unit)
  double g = b * y, h = y * 0.5;
  const double rr = fma(-h, g, 0.5);
  g = fma(g, rr, g);
  h = fma(h, rr, h);
  double d = fma(-g, g, b);
  out[8 * i + 5] = fma(d, h, g);  // one correction
  g = fma(d, h, g);
  d = fma(-g, g, b);
  out[8 * i + 6] = fma(d, h, g);  // two corrections
  out[8 * i + 7] = b * y;          // raw b * rsq
}

static double ulps(double a, double ref) {
  if (a == ref) return 0;
  long long ia, ir;
  memcpy(&ia, &a, 8);
  memcpy(&ir, &ref, 8);
  return (double)llabs(ia - ir);
}

int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), o(8 * (size_t)n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-8, 8);
  for (auto& v : x) v = std::exp2(u(g));
  double *dx, *dout;
  hipMalloc(&dx, 8 * n);
  hipMalloc(&dout, 64 * (size_t)n);
  hipMemcpy(dx, x.data(), 8 * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
  hipMemcpy(o.data(), dout, 64 * (size_t)n, hipMemcpyDeviceToHost);
  const char* names[8] = {"rcp", "rcp+1N", "rcp+2N", "rcp+3N", "rsq", "sqrt 1c", "sqrt 2c", "b*rsq"};
  for (int c = 0; c < 8; ++c) {
    double mx = 0, mean = 0;
    int exact = 0;
    for (int i = 0; i < n; ++i) {
      const double ref = c < 4 ? 1.0 / x[i] : (c == 4 ? 1.0 / std::sqrt(x[i]) : std::sqrt(x[i]));
      const double e = ulps(o[8 * (size_t)i + c], ref);
      mx = e > mx ? e : mx;
      mean += e;
      exact += e == 0;
    }
    printf("%-8s max %.0f ulp  mean %.3f ulp  exact %.4f\n", names[c], mx, mean / n, (double)exact / n);
  }
  return 0;
}

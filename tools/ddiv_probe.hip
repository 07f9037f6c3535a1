// ddiv_probe.hip -- f64 division without v_div_scale / v_div_fixup, and f64
// square root without its scaling / class steps (the
// operands of the search's divisions are normal and their quotients far from
// overflow / underflow, where those two only pass values through): bit
// equality with a / b over random search-like operands, and cycles per
// division (s_memtime, one wave).  Not product code: a diagnostic.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/ddiv_probe tools/ddiv_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

__device__ __forceinline__ double ddiv_fast(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);               // v_rcp_f64
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = a * r;
  const double res = __builtin_fma(-b, q, a);
  return __builtin_fma(res, r, q);
}

__device__ __forceinline__ double dsqrt_fast(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  double g = x * r, h = r * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}

__global__ void k_check(const double* a, const double* b, unsigned long long* bad, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double x = a[i] / b[i], y = ddiv_fast(a[i], b[i]);
  if (__double_as_longlong(x) != __double_as_longlong(y)) atomicAdd(bad, 1ull);
  // square roots: the integers 1 .. n and |a| (wide exponents)
  const double s1 = (double)(i + 1), s2 = fabs(a[i]) + 1e-300;
  if (__double_as_longlong(sqrt(s1)) != __double_as_longlong(dsqrt_fast(s1))) atomicAdd(bad + 1, 1ull);
  if (__double_as_longlong(sqrt(s2)) != __double_as_longlong(dsqrt_fast(s2))) atomicAdd(bad + 1, 1ull);
}

template <int FAST>
__global__ void k_time(const double* a, const double* b, unsigned long long* cyc, double* sink) {
  double x = a[threadIdx.x], y = b[threadIdx.x], acc = 0.0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 4096; ++it) {
    const double q = FAST ? ddiv_fast(x, y) : x / y;
    acc += q;
    x = x + 1e-3;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  sink[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[FAST] = t1 - t0;
}

int main() {
  const int n = 1 << 24;
  std::vector<double> a(n), b(n);
  srand(11);
  auto rnd = [] { return (rand() + 0.5) / ((double)RAND_MAX + 1.0); };
  for (int i = 0; i < n; ++i) {
    switch (i % 4) {
      case 0: a[i] = (rnd() * 2 - 1) * 200.0; b[i] = 1 + rand() % 400; break;          // q = W / N
      case 1: a[i] = rnd() * rnd(); b[i] = rnd() * 1e-3 + 1e-12; break;                 // (q - lo) / (hi - lo)
      case 2: a[i] = 2.5 * rnd() * sqrt(1.0 + rand() % 1600); b[i] = 1 + rand() % 1600; break;   // u
      default: a[i] = (rnd() * 2 - 1) * pow(2.0, rand() % 60 - 30); b[i] = rnd() * pow(2.0, rand() % 60 - 30) + 1e-300; break;
    }
  }
  double *da, *db, *sink;
  unsigned long long *dbad, *dcyc;
  hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dbad, 16); hipMalloc(&dcyc, 16); hipMalloc(&sink, 64 * 8);
  hipMemcpy(da, a.data(), n * 8, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), n * 8, hipMemcpyHostToDevice);
  hipMemset(dbad, 0, 16);
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, da, db, dbad, n);
  hipLaunchKernelGGL(k_time<0>, dim3(1), dim3(64), 0, 0, da, db, dcyc, sink);
  hipLaunchKernelGGL(k_time<1>, dim3(1), dim3(64), 0, 0, da, db, dcyc, sink);
  hipLaunchKernelGGL(k_time<0>, dim3(1), dim3(64), 0, 0, da, db, dcyc, sink);
  hipLaunchKernelGGL(k_time<1>, dim3(1), dim3(64), 0, 0, da, db, dcyc, sink);
  unsigned long long bad[2] = {0, 0}, cyc[2];
  hipMemcpy(bad, dbad, 16, hipMemcpyDeviceToHost);
  hipMemcpy(cyc, dcyc, 16, hipMemcpyDeviceToHost);
  printf("{\"pairs\": %d, \"mismatches\": %llu, \"sqrt_mismatches\": %llu, \"cycles_per_div_ieee\": %.1f, \"cycles_per_div_fast\": %.1f}\n", n, bad[0], bad[1],
         cyc[0] / 4096.0, cyc[1] / 4096.0);
  return 0;
}

// Development probe: throughput of v_mfma_f32_16x16x4_f32 accumulation chains
// on gfx950 vs the number of independent chains per wave (XG) and waves per
// SIMD (W).  Registers only.  Prints cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int XG, int W>
__global__ void __launch_bounds__(256 * W) __attribute__((amdgpu_waves_per_eu(W, W)))
chain(float* out, unsigned long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  f4 acc[XG];
  for (int q = 0; q < XG; ++q) acc[q] = f4{0, 0, 0, 0};
  f4 a = f4{lane * 0.1f, 1.f, 2.f, 3.f}, b = f4{1.f, lane * 0.01f, 3.f, 4.f};
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int q = 0; q < XG; ++q) acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], b[(e + q) & 3], acc[q], 0, 0, 0);
    a += 1.0f;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int q = 0; q < XG; ++q) s += acc[q][0] + acc[q][3];
  out[blockIdx.x * 256 * W + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) atomicMax(cyc + blockIdx.x, t1 - t0);
}

template <int XG, int W>
void run() {
  const int blocks = 256, iters = 2000;
  float* out; unsigned long long* cyc;
  hipMalloc(&out, blocks * 256 * W * 4); hipMalloc(&cyc, blocks * 8);
  for (int rep = 0; rep < 2; ++rep) {
    hipMemset(cyc, 0, blocks * 8);
    hipLaunchKernelGGL((chain<XG, W>), dim3(blocks), dim3(256 * W), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
  }
  unsigned long long h[256]; hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0; for (int i = 0; i < blocks; ++i) m += h[i]; m /= blocks;
  printf("XG=%d W=%d: %.1f cycles per MFMA per SIMD\n", XG, W, m / ((double)iters * 4 * XG * W));
  hipFree(out); hipFree(cyc);
}

int main() {
  run<1, 1>(); run<2, 1>(); run<4, 1>(); run<8, 1>();
  run<1, 2>(); run<2, 2>(); run<4, 2>();
  run<1, 3>(); run<2, 3>(); run<4, 3>();
  return 0;
}

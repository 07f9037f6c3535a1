// Calibration probe for the conv's inner loop on gfx950 (development tool).
// One workgroup of 4 waves per CU, 256 workgroups, each wave runs ITER
// k-steps of 9 v_mfma_f32_16x16x4_f32 (3x3 accumulators, the 9x9 conv's
// job shape).  Variants: operands from registers; operands from LDS; with a
// workgroup barrier every KC k-steps.  Prints cycles per MFMA per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE, int KC, int NT = 256>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(NT / 256, NT / 256)))
probe(float* out, unsigned long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) float lds[96 * 112 + 8192];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 96 * 112 + 8192; i += NT) lds[i] = (float)(i & 7) * 0.001f;
  // gather offsets like the real conv: 16-cell tiles of a 9x9 board shifted by a tap
  int off[3]; bool ok[3];
  for (int i = 0; i < 3; ++i) {
    int cell = (i * 16 + (lane & 15)) % 81, y = cell / 9, x = cell % 9;
    int yy = y - 1, xx = x + 1;
    ok[i] = yy >= 0 && xx < 9;
    off[i] = ok[i] ? yy * 9 + xx : 0;
  }
  __syncthreads();
  f4 acc[3][3];
  for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) acc[a][b] = f4{0, 0, 0, 0};
  float ra[3] = {lane * 0.1f, lane * 0.2f, lane * 0.3f}, rb[3] = {1.f, 2.f, 3.f};
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it += KC) {
    if (MODE == 2) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); }
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      float a[3], b[3];
      if (MODE == 0) {
        for (int i = 0; i < 3; ++i) { a[i] = ra[i]; b[i] = rb[i]; }
      } else {
        const float4 av = *reinterpret_cast<const float4*>(lds + 96 * 112 + ((kk * 2) * 64 + lane) * 4);
        a[0] = av.x; a[1] = av.y; a[2] = av.z;
        if (MODE >= 3) {
          for (int i = 0; i < 3; ++i) {
            float v = lds[((it + kk) % 24 * 4 + (lane >> 4)) * 112 + off[i]];
            b[i] = ok[i] ? v : 0.f;
          }
        } else {
          for (int i = 0; i < 3; ++i) b[i] = lds[((it + kk) % 24 * 4 + (lane >> 4)) * 112 + (lane & 15) + 16 * i];
        }
      }
      for (int mi = 0; mi < 3; ++mi)
        for (int ni = 0; ni < 3; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int a = 0; a < 3; ++a) for (int b = 0; b < 3; ++b) s += acc[a][b][0] + acc[a][b][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int KC, int NT = 256>
void run(const char* name, float* out, unsigned long long* cyc, int iters) {
  // NT = 512: two waves per SIMD, each doing half of the per-CU work
  const int wi = NT == 512 ? iters / 2 : iters;
  hipLaunchKernelGGL((probe<MODE, KC, NT>), dim3(256), dim3(NT), 0, 0, out, cyc, wi);
  hipLaunchKernelGGL((probe<MODE, KC, NT>), dim3(256), dim3(NT), 0, 0, out, cyc, wi);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL((probe<MODE, KC, NT>), dim3(256), dim3(NT), 0, 0, out, cyc, wi);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  unsigned long long h[256];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  double avg = 0; for (int i = 0; i < 256; ++i) avg += h[i]; avg /= 256;
  double mfma = 9.0 * iters;   // per CU-quarter (one SIMD's share)
  printf("%-34s cycles/MFMA/SIMD %.1f  wall %.3f ms  TF/s %.1f\n", name, avg / mfma, ms,
         256.0 * 4 * mfma * 2048 / (ms * 1e-3) / 1e12);
}

int main() {
  float* out; unsigned long long* cyc;
  hipMalloc(&out, 256 * 256 * 4); hipMalloc(&cyc, 256 * 8);
  const int iters = 21600;
  run<0, 8>("registers", out, cyc, iters);
  run<1, 8>("lds operands", out, cyc, iters);
  run<2, 8>("lds + barrier/8 k-steps", out, cyc, iters);
  run<2, 4>("lds + barrier/4 k-steps", out, cyc, iters);
  run<3, 8>("lds gather+cndmask", out, cyc, iters);
  run<3, 8, 512>("lds gather+cndmask, 2 waves/SIMD", out, cyc, iters);
  run<1, 8, 512>("lds operands, 2 waves/SIMD", out, cyc, iters);
  return 0;
}

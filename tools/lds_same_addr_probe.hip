// lds_same_addr_probe.hip -- cost of a wave-uniform LDS store done by all 64
// lanes (same address, same value) against the same store by lane 0 only.
// Diagnostic for DESIGN.md §7 (select_leaf's t.leaf / t.depth / t.umask).
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_same_addr_probe tools/lds_same_addr_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 4096;

template <int MODE>
__global__ void __launch_bounds__(64) k_probe(unsigned long long* out, int seed) {
  __shared__ int s[64];
  __shared__ unsigned long long m[4];
  const int lane = threadIdx.x;
  int v = seed + lane;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    const int u = __builtin_amdgcn_readfirstlane(v + it);
    if constexpr (MODE == 0) {                    // all lanes, same address (int + u64)
      s[3] = u;
      m[1] = (unsigned long long)u << 7;
    } else if constexpr (MODE == 1) {             // lane 0 only
      if (lane == 0) {
        s[3] = u;
        m[1] = (unsigned long long)u << 7;
      }
    } else {                                      // all lanes, own addresses
      s[lane] = u;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    v += s[(it + lane) & 63] & 1;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[MODE] = t1 - t0 + (unsigned long long)(v & 1);
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 8 * 8);
  for (int r = 0; r < 2; ++r) {
    hipLaunchKernelGGL(k_probe<0>, dim3(1), dim3(64), 0, 0, d, 1);
    hipLaunchKernelGGL(k_probe<1>, dim3(1), dim3(64), 0, 0, d, 1);
    hipLaunchKernelGGL(k_probe<2>, dim3(1), dim3(64), 0, 0, d, 1);
    hipDeviceSynchronize();
  }
  unsigned long long h[3];
  hipMemcpy(h, d, 3 * 8, hipMemcpyDeviceToHost);
  printf("{\"all_lanes_same_addr\": %.1f, \"lane0_only\": %.1f, \"all_lanes_own_addr\": %.1f, \"unit\": \"cycles per iteration\"}\n",
         (double)h[0] / kIters, (double)h[1] / kIters, (double)h[2] / kIters);
  return 0;
}

// Residual-tower engine: board-size independent kernels and the table lookup.
#include "mzgo_tower_dispatch.hpp"

namespace mzgo {
extern const TowerSet tower_n5, tower_n9, tower_n19;

const TowerSet* find_tower(int N) {
  static const TowerSet* all[] = {&tower_n5, &tower_n9, &tower_n19};
  for (const TowerSet* t : all)
    if (t->N == N) return t;
  return nullptr;
}

__global__ void __launch_bounds__(256) k_tact(const int64_t* __restrict__ a, int* out, int B, int A, int* err) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B) return;
  const int64_t v = a[i];
  if (v < 0 || v >= A) { *err = 1; out[i] = 0; } else { out[i] = (int)v; }
}

hipError_t launch_tact(const int64_t* a, int* out, int B, int A, int* err, hipStream_t s) {
  hipLaunchKernelGGL(k_tact, dim3((B + 255) / 256), dim3(256), 0, s, a, out, B, A, err);
  return hipGetLastError();
}
}  // namespace mzgo

#ifdef MZGO_TCONV_STAMPS
// Diagnostic builds only: k_tconv's per-workgroup cycle sums, summed over
// workgroups (out[64] = [wave][field]), then zeroed.
extern "C" int mzgo_debug_tconv_stamps(unsigned long long* out) {
  // every instantiation has its own g_tstamps: read the 19x19 one
  return mzgo::tower_stamps_n19(out);
}
#endif

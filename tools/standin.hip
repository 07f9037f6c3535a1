// A stand-in for an RCCL collective's kernel (scripts/rccl_standin.py): W
// workgroups of one wave, each holding `lds` bytes of LDS and spinning for
// `cycles` shader-clock cycles (s_memtime), like a gather kernel waiting for
// a peer rank.  Used to measure whether such a kernel, ordered after epoch i
// on a second stream, delays epoch i + 1's whole-game launch (which puts one
// workgroup on every CU at ~159 KiB of LDS).
#include <hip/hip_runtime.h>

template <int LDS>
__global__ void __launch_bounds__(64) k_standin(long long cycles, int* sink) {
  __shared__ int buf[LDS / 4];
  for (int i = threadIdx.x; i < LDS / 4; i += 64) buf[i] = i;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0 && buf[blockIdx.x % (LDS / 4)] < 0) sink[0] = 1;   // (keeps buf live)
}

extern "C" int standin_launch(int workgroups, int lds_kb, long long cycles, int* sink, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (lds_kb <= 8) hipLaunchKernelGGL(k_standin<8192>, dim3(workgroups), dim3(64), 0, s, cycles, sink);
  else if (lds_kb <= 32) hipLaunchKernelGGL(k_standin<32768>, dim3(workgroups), dim3(64), 0, s, cycles, sink);
  else hipLaunchKernelGGL(k_standin<65536>, dim3(workgroups), dim3(64), 0, s, cycles, sink);
  return (int)hipGetLastError();
}

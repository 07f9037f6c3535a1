// l1_visibility_probe.hip -- which consumer-side reads see another CU's
// stores on the same XCC (the round-5 19x19 hand-off hang and
// the k_tconv_chain same-XCC path).  Not product code: a diagnostic.
//
// Pairs of workgroups: consumer c (blocks 0-7) and producer c + 8 (the
// dispatcher deals blocks to the 8 XCDs in turn, so b and b + 8 share one;
// both XCC ids are read and reported).  Per round r the consumer reads a 4 KiB
// buffer with plain loads (its L1 now holds the lines), then releases the
// producer; the producer stores r into every word (plain stores), drains them
// (s_waitcnt vmcnt(0)) and sets a flag (relaxed agent-scope store) -- the
// producer side of the chain's same-XCC path, no release.  The consumer polls
// the flag, applies the variant's invalidate and reads the buffer back with
// the variant's load; every word != r is stale.
//   variant 0: no invalidate,           plain global_load_dword
//   variant 1: buffer_inv sc0,          plain loads   (the round-5 helper experiment)
//   variant 2: fence(acquire, agent),   plain loads   (= buffer_inv sc1)
//   variant 3: no invalidate,           global_load_dword sc0
//   variant 4: no invalidate,           global_load_dword sc1
//   variant 5: no invalidate,           LDS-DMA global_load_lds_dwordx4 sc0 (k_tconv_chain's dma16_l2 to round 5)
//   variant 6: no invalidate,           LDS-DMA global_load_lds_dwordx4 sc1 (its round-6 form)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/l1_visibility_probe tools/l1_visibility_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kWords = 1024;     // 4 KiB per pair
constexpr int kRounds = 64;
constexpr long long kSpin = 1ll << 22;

__device__ __forceinline__ bool wait_ge(unsigned* p, unsigned v) {
  for (long long s = 0; s < kSpin; ++s) {
    if ((int)(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - v) >= 0) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

__device__ __forceinline__ unsigned ld_sc0(const unsigned* p) {
  unsigned v;
  asm volatile("global_load_dword %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
  unsigned v;
  asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
template <bool SC1>
__device__ __forceinline__ void dma16(const void* g, uint32_t lds) {
  uint32_t keep;
  if (SC1)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\t"
                 "s_mov_b32 m0, %0" : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc0\n\t"
                 "s_mov_b32 m0, %0" : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

// out[c * 4 + 0] stale words, [1] timeouts, [2] consumer XCC, [3] producer XCC
__global__ void __launch_bounds__(64) k_probe(unsigned* buf, unsigned* ready, unsigned* done, unsigned* xcc,
                                              unsigned long long* out, int variant) {
  __shared__ __attribute__((aligned(16))) unsigned lds[kWords];
  const int b = blockIdx.x, lane = threadIdx.x;
  const int pair = b & 7;
  unsigned* B = buf + pair * kWords;
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (lane == 0) xcc[b] = x & 0xF;
  unsigned long long stale = 0, tmo = 0;
  if (b < 8) {                                   // consumer
    for (int r = 1; r <= kRounds; ++r) {
      unsigned warm = 0;
      for (int i = lane; i < kWords; i += 64) warm += B[i];          // lines into this CU's L1
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      stale += warm == 0xFFFFFFFFu;                                  // (keeps the loads; never true)
      if (lane == 0) __hip_atomic_store(ready + pair, (unsigned)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bool ok = true;
      if (lane == 0) ok = wait_ge(done + pair, (unsigned)r);
      ok = __shfl(ok ? 1 : 0, 0) != 0;
      if (!ok) { ++tmo; break; }
      if (variant == 1) asm volatile("buffer_inv sc0" ::: "memory");
      if (variant == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (variant >= 5) {
        const uint32_t base = (uint32_t)(uintptr_t)lds;
        for (int k = 0; k < kWords * 4 / 1024; ++k) {
          const void* g = reinterpret_cast<const char*>(B) + k * 1024 + lane * 16;
          if (variant == 6) dma16<true>(g, base + k * 1024); else dma16<false>(g, base + k * 1024);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        for (int i = lane; i < kWords; i += 64) stale += lds[i] != (unsigned)r;
        __syncthreads();
      } else {
        for (int i = lane; i < kWords; i += 64) {
          const unsigned v = variant == 3 ? ld_sc0(B + i) : variant == 4 ? ld_sc1(B + i) : B[i];
          stale += v != (unsigned)r;
        }
      }
    }
  } else {                                       // producer
    for (int r = 1; r <= kRounds; ++r) {
      bool ok = true;
      if (lane == 0) ok = wait_ge(ready + pair, (unsigned)r);
      ok = __shfl(ok ? 1 : 0, 0) != 0;
      if (!ok) { ++tmo; break; }
      for (int i = lane; i < kWords; i += 64) B[i] = (unsigned)r;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(done + pair, (unsigned)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  for (int o = 32; o > 0; o >>= 1) stale += __shfl_xor(stale, o);
  if (lane == 0) {
    atomicAdd(out + pair * 4 + 0, stale);
    atomicAdd(out + pair * 4 + 1, tmo);
  }
}

int main() {
  unsigned *buf, *ready, *done, *xcc;
  unsigned long long* out;
  if (hipMalloc(&buf, 8 * kWords * 4) || hipMalloc(&ready, 64) || hipMalloc(&done, 64) || hipMalloc(&xcc, 64) ||
      hipMalloc(&out, 8 * 4 * 8))
    return 1;
  const char* names[] = {"no invalidate, plain loads", "buffer_inv sc0, plain loads",
                         "fence(acquire, agent), plain loads", "no invalidate, sc0 loads",
                         "no invalidate, sc1 loads", "no invalidate, LDS-DMA sc0", "no invalidate, LDS-DMA sc1"};
  printf("{\"words_per_round\": %d, \"rounds\": %d, \"pairs\": 8, \"variants\": [\n", kWords, kRounds);
  for (int v = 0; v < 7; ++v) {
    if (hipMemset(buf, 0, 8 * kWords * 4) || hipMemset(ready, 0, 64) || hipMemset(done, 0, 64) ||
        hipMemset(out, 0, 8 * 4 * 8))
      return 1;
    hipLaunchKernelGGL(k_probe, dim3(16), dim3(64), 0, 0, buf, ready, done, xcc, out, v);
    if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "launch failed\n"); return 1; }
    unsigned long long h[32];
    unsigned hx[16];
    if (hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost) || hipMemcpy(hx, xcc, sizeof(hx), hipMemcpyDeviceToHost))
      return 1;
    unsigned long long st = 0, tm = 0;
    int same = 0;
    for (int p = 0; p < 8; ++p) { st += h[p * 4]; tm += h[p * 4 + 1]; same += hx[p] == hx[p + 8]; }
    printf("  {\"variant\": %d, \"what\": \"%s\", \"stale_words\": %llu, \"of\": %d, \"timeouts\": %llu, "
           "\"pairs_same_xcc\": %d}%s\n",
           v, names[v], st, 8 * kWords * kRounds, tm, same, v < 6 ? "," : "");
  }
  printf("]}\n");
  return 0;
}

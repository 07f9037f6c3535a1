// mzgo_common.hpp -- shared device definitions for the MI355X MuZero-Go engine.
//
// Geometry, the counter-based RNG (restated in oracle/rng.py), wave64
// reductions and numpy's pairwise-sum order (restated in oracle/npsum.py).
// Everything here is gfx950 (CDNA4) device code: wave = 64 lanes, one
// workgroup of 4 waves per game.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mzgo {

// One workgroup per game.  9x9 runs 12 waves = 3 per SIMD (Winograd convs,
// one wave per cout tile and cin half); 5x5 and 6x6 run 8 waves = 2 per SIMD,
// the wave pairs splitting the direct conv's k-range; 19x19 runs 4 waves (its
// 4 cell jobs per wave need every register).

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// Board / latent geometry.  Cells are stored row-major (a = r*N + c, pass = N*N)
// exactly as GymGo flattens them (self_play.py:153).
// ---------------------------------------------------------------------------
template <int N_, int C_>
struct Geo {
  static constexpr int N = N_;
  static constexpr int C = C_;                    // latent_dim
  static constexpr int CELLS = N * N;
  static constexpr int A = CELLS + 1;             // action size (pass last)
  static constexpr int CT = (CELLS + 15) / 16;    // 16-cell MFMA column tiles
  static constexpr int CS = CT * 16;              // padded cell stride of pooled latents
  static constexpr int CPAD = (CS % 32 == 0) ? CS + 16 : CS;  // LDS row stride (== 16 mod 32)
  static constexpr int CINMAX = C > 64 ? C : 64;  // widest conv input staged in LDS
  static constexpr int NG = CT >= 3 ? 3 : CT;     // cell tiles per wave job
  static constexpr int NCG = (CT + NG - 1) / NG;  // cell groups
  static constexpr int AP = (A + 63) / 64;        // actions per lane (a = lane + 64*j)
  // 9x9 runs its latent convs as Winograd F(2,3)xF(3,3) GEMMs (mzgo_wino.hpp)
  static constexpr bool WINO = N == 9;
  static constexpr int WAVES = WINO ? 12 : (NCG <= 2 ? 8 : 4);  // waves per workgroup
  static constexpr int THREADS = WAVES * 64;
  static constexpr int WPE = WAVES / 4;           // waves per SIMD
  static constexpr int KSPLIT = WINO ? 2 : WAVES / 4;  // ring conv: k-range split over wave halves
  static constexpr int TREE_CAP = NCG <= 2 ? 512 : 0;  // nodes whose stats fit in LDS (0: HBM only)
  static_assert(C % 16 == 0, "latent_dim must be a multiple of 16");
};

// ---------------------------------------------------------------------------
// Counter-based RNG (oracle/rng.py):
//   key  = mix64(mix64(seed) ^ (game << 32 | move))
//   draw = mix64(key ^ (tag << 56) ^ idx)
// ---------------------------------------------------------------------------
enum : uint32_t { TAG_SELECT = 1, TAG_DIRICHLET = 2, TAG_ACTION = 3, TAG_WEIGHT = 4 };

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t stream_key(uint64_t seed, uint32_t game, uint32_t move) {
  return mix64(mix64(seed) ^ ((uint64_t)game << 32 | (uint64_t)move));
}
__host__ __device__ __forceinline__ uint64_t draw(uint64_t key, uint32_t tag, uint64_t idx) {
  return mix64(key ^ ((uint64_t)(tag & 0xFF) << 56) ^ (idx & ((1ull << 56) - 1)));
}
__host__ __device__ __forceinline__ double u01(uint64_t h) { return (double)(h >> 11) * 0x1.0p-53; }
__host__ __device__ __forceinline__ uint32_t randbelow(uint64_t h, uint32_t n) {
  return (uint32_t)(((h >> 32) * (uint64_t)n) >> 32);
}

// ---------------------------------------------------------------------------
// Diagnostic phase stamps (only in a -DMZGO_STAMPS build; see
// scripts/microbench.py).  Thread 0 of each workgroup adds shader-clock
// deltas per phase into mzgo_stamps[block][phase].
// ---------------------------------------------------------------------------
constexpr int kStampPhases = 24;   // 0-7 phases (thread 0), 8-19 per-wave conv loops
#ifdef MZGO_STAMPS
struct Stamp {
  unsigned long long* buf;
  unsigned long long t;
  __device__ explicit Stamp(unsigned long long* b) : buf(b) { t = __builtin_amdgcn_s_memtime(); }
  __device__ void lap(int phase) {
    unsigned long long now = __builtin_amdgcn_s_memtime();
    if (buf && threadIdx.x == 0) buf[blockIdx.x * kStampPhases + phase] += now - t;
    t = now;
  }
  __device__ void wave_add(int phase, unsigned long long cycles) {
    if (buf && (threadIdx.x & 63) == 0) buf[blockIdx.x * kStampPhases + phase] += cycles;
  }
};
#else
struct Stamp {
  __device__ explicit Stamp(unsigned long long*) {}
  __device__ void lap(int) {}
  __device__ void wave_add(int, unsigned long long) {}
};
#endif

// ---------------------------------------------------------------------------
// wave64 helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// Order LDS traffic between lanes of one wave (no workgroup barrier needed).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T w = __shfl_xor(v, o); v = w > v ? w : v; }
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T w = __shfl_xor(v, o); v = w < v ? w : v; }
  return v;
}

// ---------------------------------------------------------------------------
// numpy 2.2.6 pairwise_sum order (oracle/npsum.py), evaluated by one wave.
// Every lane returns the same value.  x lives in LDS.  Used wherever the
// reference calls ``.sum()`` on a prior vector (self_play.py:160,170,211,378)
// so that normalised priors are bit-identical to the reference's.
// ---------------------------------------------------------------------------
template <typename T, int N>
__device__ __forceinline__ T np_pairwise_sum(const T* x) {
  wave_lds_sync();
  if constexpr (N < 8) {
    T r = (T)0;
#pragma unroll
    for (int i = 0; i < N; ++i) r = r + x[i];
    return r;
  } else if constexpr (N <= 128) {
    constexpr int STOP = N - (N % 8);
    const int j = lane_id() & 7;
    T r = x[j];
    for (int i = 8; i < STOP; i += 8) r = r + x[i + j];
    T r0 = __shfl(r, 0), r1 = __shfl(r, 1), r2 = __shfl(r, 2), r3 = __shfl(r, 3);
    T r4 = __shfl(r, 4), r5 = __shfl(r, 5), r6 = __shfl(r, 6), r7 = __shfl(r, 7);
    T res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
#pragma unroll
    for (int i = STOP; i < N; ++i) res = res + x[i];
    return res;
  } else {
    constexpr int H = N / 2;
    constexpr int N2 = H - (H % 8);
    T lo = np_pairwise_sum<T, N2>(x);
    T hi = np_pairwise_sum<T, N - N2>(x + N2);
    return lo + hi;
  }
}

// f32 result of numpy's in-place ``f32_array *= f64_array`` element
__device__ __forceinline__ float mul_f32_by_f64(float p, double m) { return (float)((double)p * m); }

}  // namespace mzgo

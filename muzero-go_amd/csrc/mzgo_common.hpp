// mzgo_common.hpp -- shared device definitions for the MI355X MuZero-Go engine.
//
// Geometry, the counter-based RNG (restated in oracle/rng.py), wave64
// reductions and numpy's pairwise-sum order (restated in oracle/npsum.py).
// Everything here is gfx950 (CDNA4) device code: wave = 64 lanes, one
// workgroup of 4 waves per game.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Diagnostic switches that change results (stage knock-outs, timing
// ablations) exist only in diagnostic builds (mzgo_diag.hpp): the product
// library refuses to compile with any of them.
#if !defined(MZGO_DIAG_BUILD) && (defined(MZGO_TCONV_ABL_NODMA) || defined(MZGO_TCONV_ABL_NOBAR))
#error "wrong-result diagnostic switch without -DMZGO_DIAG_BUILD (diagnostic builds: scripts/build_variant.sh)"
#endif

namespace mzgo {

// One workgroup per game.  9x9 runs 12 waves = 3 per SIMD (Winograd convs,
// one wave per cout tile and cin half); 5x5 and 6x6 run 8 waves = 2 per SIMD,
// the wave pairs splitting the direct conv's k-range; 19x19 runs 4 waves (its
// 4 cell jobs per wave need every register).

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

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
  static constexpr bool WINO = N == 9 || N == 19;
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
// 0-7 phases (thread 0), 8-19 per-wave conv loops, 20-31 sub-phases,
// 40-43 shared batch jobs (publish, picks, own rounds, wait), 44-47 the
// 9x9 tail (a helper's unit cycles, units, jobs served; cycles in the tail
// phase), 52-54 shared
// conv jobs (publish + picks, own strips, wait), 56-63 factored simulation
// detail (see sim_loop), 64-71 batch_expand / expand_child detail,
// 72-82 verify_batch / parent conv detail, 83-87 self-play move phases,
// 88-90 representation convs, 91-95 select counts (levels at depth >= 2,
// selects, sequential-replay batches and their simulations, leaf depth sum)
constexpr int kStampPhases = 96;
constexpr int kStampLds = 91;          // phases >= this are thread 0's counters, kept in registers
#ifdef MZGO_STAMPS
// Phase sums accumulate in LDS (a global read-modify-write per lap would put
// an HBM round trip on the measured wave's critical path); flush() adds them
// to the global buffer once.
struct Stamp {
  unsigned long long* buf;
  unsigned long long* lds;
  unsigned long long t;
  __device__ explicit Stamp(unsigned long long* b) : buf(b) {
    __shared__ unsigned long long stamp_lds[kStampLds];
    lds = stamp_lds;
    if (threadIdx.x < kStampLds) lds[threadIdx.x] = 0;
    __syncthreads();
    t = __builtin_amdgcn_s_memtime();
  }
  __device__ void lap(int phase) {
    unsigned long long now = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) lds[phase] += now - t;
    t = now;
  }
  unsigned long long xr[kStampPhases - kStampLds] = {};
  __device__ void wave_add(int phase, unsigned long long cycles) {
    if (phase >= kStampLds) {
      if (threadIdx.x == 0) xr[phase - kStampLds] += cycles;
    } else if ((threadIdx.x & 63) == 0) {
      lds[phase] += cycles;   // one slot per wave
    }
  }
  __device__ unsigned long long now() const { return __builtin_amdgcn_s_memtime(); }
  __device__ void flush() {
    __syncthreads();
    if (buf && threadIdx.x < kStampLds) buf[blockIdx.x * kStampPhases + threadIdx.x] += lds[threadIdx.x];
    if (buf && threadIdx.x == 0)
      for (int k = 0; k < kStampPhases - kStampLds; ++k) buf[blockIdx.x * kStampPhases + kStampLds + k] += xr[k];
  }
};
#else
struct Stamp {
  __device__ explicit Stamp(unsigned long long*) {}
  __device__ void lap(int) {}
  __device__ void wave_add(int, unsigned long long) {}
  __device__ unsigned long long now() const { return 0; }
  __device__ void flush() {}
};
#endif

// ---------------------------------------------------------------------------
// wave64 helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// lane id that the compiler cannot hoist out of the simulation loop: values
// derived from it are recomputed (a few VALU ops) instead of being kept live
// across the whole loop and spilled at 168 VGPRs (3 waves per SIMD)
__device__ __forceinline__ int lane_id_local() {
  int l = threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
// thread index the compiler cannot hoist out of the move / simulation loops
// (as lane_id_local): IR-level LICM otherwise lifts every phase's
// threadIdx-derived LDS offsets to the kernel entry, where they stay live
// across the whole-game loop and spill (k_selfplay_move<9,96>: 236 -> 0 B
// scratch, 168 -> 160 VGPRs)
__device__ __forceinline__ int tid_local() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// a / b in f64, correctly rounded, for the search's divisions (q = W / N,
// (q - lo) / (hi - lo), c P sqrt(N) / (1 + n)): the reciprocal, two Newton
// steps, the product and one FMA correction -- the compiler's sequence for
// `/` without v_div_scale / v_div_fmas' scaling and v_div_fixup, which only
// pass values through when a, b and a / b are normal and far from overflow,
// as these always are (finite value sums, counts >= 1, a positive spread).
// Bit-identical to `/` there (tools/ddiv_probe.hip: 16.8 M search-like and
// wide-exponent pairs, no mismatch), 22 against 75 cycles per division; the
// sign of a zero quotient may differ, which no score, minimum or maximum
// sees.  9x9 epoch +1.3-1.5 % against plain `/` and sqrt (round 4, same call).
__device__ __forceinline__ double ddiv(double a, double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = a * r;
  return __builtin_fma(__builtin_fma(-b, q, a), r, q);
}

// sqrt in f64, correctly rounded, of the search's visit counts (integers
// >= 1): the reciprocal square root and the compiler's Newton / correction
// steps without the scaling of tiny arguments and the zero / infinity / NaN
// selects.  Bit-identical to sqrt for every integer 1 .. 2^24 and 16.8 M
// wide-exponent arguments (tools/ddiv_probe.hip).
__device__ __forceinline__ double dsqrt(double x) {
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

// Order LDS traffic between lanes of one wave (no workgroup barrier needed).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Cross-lane moves by DPP (no LDS round trip, unlike ds_bpermute): quad_perm
// xor-1 / xor-2 and row_ror 4 / 8 combine the 16 lanes of a row; the four row
// results are then read with v_readlane.  Valid for order-insensitive
// reductions (min, max, argmax) with all 64 lanes active.
namespace dpp {
enum : int { XOR1 = 0xB1, XOR2 = 0x4E, ROR4 = 0x124, ROR8 = 0x128 };
template <int C>
__device__ __forceinline__ int mov(int v) { return __builtin_amdgcn_update_dpp(0, v, C, 0xF, 0xF, false); }
template <int C>
__device__ __forceinline__ float mov(float v) { return __int_as_float(mov<C>(__float_as_int(v))); }
template <int C>
__device__ __forceinline__ double mov(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = mov<C>((int)x), hi = mov<C>((int)(x >> 32));
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ int lane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float lane(float v, int l) { return __int_as_float(lane(__float_as_int(v), l)); }
__device__ __forceinline__ double lane(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = lane((int)x, l), hi = lane((int)(x >> 32), l);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
}  // namespace dpp

// Wave-wide min / max of a float or double, every lane getting the result:
// permlane32 / permlane16 swaps (lanes i ^ 32, i ^ 16: each returns the own
// and the partner value, in some order -- min and max are commutative), then
// in-row DPP (xor 1, xor 2, half-row mirror, row mirror), with v_min / v_max.
// (tools/puct_probe.hip: the f64 min + max of a PUCT level 610 -> 365 cycles
// against the DPP + readlane version with compare-and-select.)  The values
// reduced here are finite; a -0 / +0 tie may come out with either sign,
// which changes no score the search forms from it.
// (v_min / v_max directly: fmin / fmax lower to llvm.minnum, which in IEEE
// mode quiets signalling NaNs with a v_max x, x, x on each operand first --
// two extra f64 operations per reduction step for values that are finite)
__device__ __forceinline__ float fmin_(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float fmax_(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double fmin_(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double fmax_(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <bool S32>
__device__ __forceinline__ void lane_swap(unsigned x, unsigned& a, unsigned& b) {
  const auto r = S32 ? __builtin_amdgcn_permlane32_swap(x, x, false, false)
                     : __builtin_amdgcn_permlane16_swap(x, x, false, false);
  a = r[0];
  b = r[1];
}
template <bool S32, class Op>
__device__ __forceinline__ float swap_op(float v, Op op) {
  unsigned a, b;
  lane_swap<S32>(__float_as_uint(v), a, b);
  return op(__uint_as_float(a), __uint_as_float(b));
}
template <bool S32, class Op>
__device__ __forceinline__ double swap_op(double v, Op op) {
  const unsigned long long x = (unsigned long long)__double_as_longlong(v);
  unsigned l0, l1, h0, h1;
  lane_swap<S32>((unsigned)x, l0, l1);
  lane_swap<S32>((unsigned)(x >> 32), h0, h1);
  return op(__longlong_as_double((long long)((unsigned long long)l0 | ((unsigned long long)h0 << 32))),
            __longlong_as_double((long long)((unsigned long long)l1 | ((unsigned long long)h1 << 32))));
}
template <typename T, class Op>
__device__ __forceinline__ T wave_reduce(T v, Op op) {
  v = swap_op<true>(v, op);
  v = swap_op<false>(v, op);
  v = op(v, dpp::mov<dpp::XOR1>(v));
  v = op(v, dpp::mov<dpp::XOR2>(v));
  v = op(v, dpp::mov<0x141>(v));                // row_half_mirror: lane i <-> 7 - i
  return op(v, dpp::mov<0x140>(v));             // row_mirror: lane i <-> 15 - i
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
  return wave_reduce(v, [](T a, T b) { return fmax_(a, b); });
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
  return wave_reduce(v, [](T a, T b) { return fmin_(a, b); });
}
// min of lo and max of hi over the wave
template <typename T>
__device__ __forceinline__ void wave_minmax(T& lo, T& hi) {
  lo = wave_min(lo);
  hi = wave_max(hi);
}

// v[i] + v[i ^ 32] and v[i] + v[i ^ 16] via the gfx950 permlane swaps
// (each returns both halves; addition is commutative, so the sum is the
// butterfly's exactly)
__device__ __forceinline__ unsigned bits_of(float v) { return __float_as_uint(v); }
__device__ __forceinline__ float from_bits(unsigned v, float) { return __uint_as_float(v); }
template <bool SWAP32>
__device__ __forceinline__ float swap_add(float v) {
  const auto r = SWAP32 ? __builtin_amdgcn_permlane32_swap(bits_of(v), bits_of(v), false, false)
                        : __builtin_amdgcn_permlane16_swap(bits_of(v), bits_of(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <bool SWAP32>
__device__ __forceinline__ double swap_add(double v) {
  const long long x = __double_as_longlong(v);
  const unsigned lo = (unsigned)x, hi = (unsigned)(x >> 32);
  const auto rl = SWAP32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                         : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto rh = SWAP32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                         : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double a = __longlong_as_double((long long)rl[0] | ((long long)rh[0] << 32));
  const double b = __longlong_as_double((long long)rl[1] | ((long long)rh[1] << 32));
  return a + b;
}

// Butterfly sum (xor 32, 16, 8, 4, 2, 1) without LDS traffic: permlane swaps
// for 32/16, DPP inside a row for the rest (row_ror 8 == xor 8; after it the
// row is 8-periodic, so row_ror 4 acts as xor 4).  Bit-identical to the
// __shfl_xor butterfly.  All 64 lanes active.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  v = swap_add<true>(v);
  v = swap_add<false>(v);
  v = v + dpp::mov<dpp::ROR8>(v);
  v = v + dpp::mov<dpp::ROR4>(v);
  v = v + dpp::mov<dpp::XOR2>(v);
  v = v + dpp::mov<dpp::XOR1>(v);
  return v;
}
// (score, action, payload) argmax, ties to the lower action; all lanes get it
__device__ __forceinline__ void wave_argmax(double& s, int& a, int& c) {
  auto step = [&](double os, int oa, int oc) {
    if (os > s || (os == s && oa < a)) { s = os; a = oa; c = oc; }
  };
  step(dpp::mov<dpp::XOR1>(s), dpp::mov<dpp::XOR1>(a), dpp::mov<dpp::XOR1>(c));
  step(dpp::mov<dpp::XOR2>(s), dpp::mov<dpp::XOR2>(a), dpp::mov<dpp::XOR2>(c));
  step(dpp::mov<dpp::ROR4>(s), dpp::mov<dpp::ROR4>(a), dpp::mov<dpp::ROR4>(c));
  step(dpp::mov<dpp::ROR8>(s), dpp::mov<dpp::ROR8>(a), dpp::mov<dpp::ROR8>(c));
  double rs[4];
  int ra[4], rc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { rs[r] = dpp::lane(s, 16 * r); ra[r] = dpp::lane(a, 16 * r); rc[r] = dpp::lane(c, 16 * r); }
  s = rs[0]; a = ra[0]; c = rc[0];
#pragma unroll
  for (int r = 1; r < 4; ++r) step(rs[r], ra[r], rc[r]);
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
    const int j = lane_id_local() & 7;
    T r = x[j];
    for (int i = 8; i < STOP; i += 8) r = r + x[i + j];
    // ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) of the 8 partials in
    // lanes 8k + j, by DPP within each 8-lane group (IEEE addition is
    // commutative, so a lane's b + a equals its partner's a + b bit for bit):
    // xor 1 pairs, xor 2 quads, half-row mirror (lane i <-> 7 - i) halves --
    // every lane ends with the sum, no readlane
    r = r + dpp::mov<dpp::XOR1>(r);
    r = r + dpp::mov<dpp::XOR2>(r);
    T res = r + dpp::mov<0x141>(r);
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

// position of the k-th (0-based) set bit of m (k < popcount(m)): binary search
// on popcounts of halves
__device__ __forceinline__ int kth_set_bit(uint64_t m, uint32_t k) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint64_t lo = m & ((1ull << w) - 1);
    const uint32_t c = (uint32_t)__popcll(lo);
    if (k >= c) { k -= c; m >>= w; pos += w; } else { m = lo; }
  }
  return pos;
}

// f32 result of numpy's in-place ``f32_array *= f64_array`` element
__device__ __forceinline__ float mul_f32_by_f64(float p, double m) { return (float)((double)p * m); }

}  // namespace mzgo

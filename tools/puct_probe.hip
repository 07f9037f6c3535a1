// puct_probe.hip -- microbenchmark of one PUCT level (mzgo_search.hpp:
// puct_pick, the select_leaf step of self_play.py:296-330) on one wave, as
// the 9x9 kernel runs it (wave 0 alone; the other waves wait at a barrier).
// Reports cycles per call (s_memtime) for the full function and for its
// pieces, on random child statistics of a 9x9 node (A = 82).  Not product
// code: a diagnostic for DESIGN.md §7.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I muzero-go_amd/csrc \
//         -o tools/puct_probe tools/puct_probe.hip && tools/puct_probe
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

#include "mzgo_search.hpp"

using namespace mzgo;
typedef Geo<9, 96> G9;

constexpr int kCalls = 4096;

// candidate: min / max of a double over the wave by permlane32 / permlane16
// swaps and in-row DPP (xor 1, xor 2, half-row mirror, row mirror): every lane
// ends with the result, no readlane
struct D2 {
  double a, b;
};
template <class Op>
__device__ __forceinline__ double wave_reduce_swap(double v, Op op) {
  auto dsw = [](double x, bool s32) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    const auto l = s32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                       : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = s32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                       : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const double a = __longlong_as_double((long long)l[0] | ((long long)h[0] << 32));
    const double c = __longlong_as_double((long long)l[1] | ((long long)h[1] << 32));
    return D2{a, c};
  };
  D2 p = dsw(v, true);
  v = op(p.a, p.b);
  p = dsw(v, false);
  v = op(p.a, p.b);
  v = op(v, dpp::mov<dpp::XOR1>(v));
  v = op(v, dpp::mov<dpp::XOR2>(v));
  v = op(v, dpp::mov<0x141>(v));
  v = op(v, dpp::mov<0x140>(v));
  return v;
}

// mode 0: puct_pick; 1: q + lo/hi only; 2: + wave_minmax; 3: scores only (no reductions)
template <int MODE>
__global__ void __launch_bounds__(64) k_probe(const double* P_in, const int* n_in, const double* w_in,
                                              unsigned long long* cycles, int* picks, SearchParams sp) {
  // (modes: 0 puct_pick; 1 q + per-lane lo/hi; 2 + wave_minmax; 3 + scores; 4-7 other min/max reductions)
  typedef G9 G;
  const int lane = threadIdx.x;
  double P[G::AP], w[G::AP];
  int n[G::AP], ch[G::AP];
  uint64_t elig[G::AP];
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    P[j] = a < G::A ? P_in[a] : 0.0;
    n[j] = a < G::A ? n_in[a] : 0;
    w[j] = a < G::A ? w_in[a] : 0.0;
    ch[j] = a;
    elig[j] = __ballot(a < G::A && P[j] > 0.0);
  }
  int acc = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kCalls; ++it) {
    // perturb the inputs per call so nothing is hoisted (a visit more on a child)
    const int k = it % G::A;
    int nn[G::AP];
    double ww[G::AP];
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      nn[j] = n[j] + ((lane + 64 * j) == k ? 1 : 0);
      ww[j] = w[j] + ((lane + 64 * j) == k ? 0.25 : 0.0);
    }
    const int nvis = 200 + it;
    if constexpr (MODE == 0) {
      int best_c;
      acc += puct_pick<G>(P, nn, ww, elig, ch, nvis, false, sp, best_c);
    } else {
      double q[G::AP];
      double lo = INFINITY, hi = -INFINITY;
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        q[j] = 0.0;
        if ((elig[j] >> lane) & 1ull) {
          q[j] = nn[j] > 0 ? ww[j] / (double)nn[j] : 0.0;
          lo = fmin(lo, q[j]);
          hi = fmax(hi, q[j]);
        }
      }
      if constexpr (MODE == 2 || MODE == 3) wave_minmax(lo, hi);
      if constexpr (MODE == 4) {
        lo = wave_reduce_swap(lo, [](double a, double b) { return b < a ? b : a; });
        hi = wave_reduce_swap(hi, [](double a, double b) { return b > a ? b : a; });
      }
      if constexpr (MODE == 5) { lo = wave_min(lo); hi = wave_max(hi); }
      if constexpr (MODE == 6) {
        lo = wave_reduce(lo, [](double a, double b) { return fmin(a, b); });
        hi = wave_reduce(hi, [](double a, double b) { return fmax(a, b); });
      }
      if constexpr (MODE == 7) {
        lo = wave_reduce_swap(lo, [](double a, double b) { return fmin(a, b); });
        hi = wave_reduce_swap(hi, [](double a, double b) { return fmax(a, b); });
      }
      if constexpr (MODE == 3) {
        const double sq = sqrt((double)nvis);
#pragma unroll
        for (int j = 0; j < G::AP; ++j) {
          const double qn = hi > lo ? (q[j] - lo) / (hi - lo) : q[j];
          const double u = ((double)((float)sp.c_puct * (float)P[j]) * sq) / (double)(1 + nn[j]);
          q[j] = qn + u;
        }
      }
      acc += (int)(q[0] + q[1] + lo + hi);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) { cycles[MODE] = t1 - t0; picks[MODE] = acc; }
}

int main() {
  typedef G9 G;
  std::vector<double> P(G::A), w(G::A);
  std::vector<int> n(G::A);
  srand(7);
  double s = 0;
  for (int a = 0; a < G::A; ++a) { P[a] = (rand() % 1000 + 1) / 1000.0; s += P[a]; }
  for (int a = 0; a < G::A; ++a) {
    P[a] /= s;
    n[a] = 1 + rand() % 5;
    w[a] = n[a] * ((rand() % 2001) - 1000) / 1000.0;
  }
  double *dP, *dw;
  int *dn, *dpicks;
  unsigned long long* dc;
  hipMalloc(&dP, G::A * 8); hipMalloc(&dw, G::A * 8); hipMalloc(&dn, G::A * 4);
  hipMalloc(&dc, 8 * 8); hipMalloc(&dpicks, 8 * 4);
  hipMemcpy(dP, P.data(), G::A * 8, hipMemcpyHostToDevice);
  hipMemcpy(dw, w.data(), G::A * 8, hipMemcpyHostToDevice);
  hipMemcpy(dn, n.data(), G::A * 4, hipMemcpyHostToDevice);
  SearchParams sp{};
  sp.c_puct = 2.5;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_probe<0>, dim3(1), dim3(64), 0, 0, dP, dn, dw, dc, dpicks, sp);
    hipLaunchKernelGGL(k_probe<1>, dim3(1), dim3(64), 0, 0, dP, dn, dw, dc, dpicks, sp);
    hipLaunchKernelGGL(k_probe<2>, dim3(1), dim3(64), 0, 0, dP, dn, dw, dc, dpicks, sp);
    hipLaunchKernelGGL(k_probe<3>, dim3(1), dim3(64), 0, 0, dP, dn, dw, dc, dpicks, sp);
    hipLaunchKernelGGL(k_probe<4>, dim3(1), dim3(64), 0, 0, dP, dn, dw, dc, dpicks, sp);
    hipLaunchKernelGGL(k_probe<5>, dim3(1), dim3(64), 0, 0, dP, dn, dw, dc, dpicks, sp);
    hipLaunchKernelGGL(k_probe<6>, dim3(1), dim3(64), 0, 0, dP, dn, dw, dc, dpicks, sp);
    hipLaunchKernelGGL(k_probe<7>, dim3(1), dim3(64), 0, 0, dP, dn, dw, dc, dpicks, sp);
    hipDeviceSynchronize();
  }
  unsigned long long c[8];
  hipMemcpy(c, dc, 8 * 8, hipMemcpyDeviceToHost);
  int pk[8];
  hipMemcpy(pk, dpicks, 8 * 4, hipMemcpyDeviceToHost);
  // s_memtime counts at the shader clock; per call
  printf("{\"puct_pick\": %.0f, \"q_lohi\": %.0f, \"q_lohi_minmax\": %.0f, \"q_minmax_scores\": %.0f, "
         "\"q_lohi_minmax_swap\": %.0f, \"q_lohi_min_max_separate\": %.0f, \"fminmax_dpp\": %.0f, "
         "\"fminmax_swap\": %.0f, \"same_results\": %d, "
         "\"unit\": \"s_memtime cycles per call, one wave, 9x9 (A = 82)\"}\n",
         (double)c[0] / kCalls, (double)c[1] / kCalls, (double)c[2] / kCalls, (double)c[3] / kCalls,
         (double)c[4] / kCalls, (double)c[5] / kCalls, (double)c[6] / kCalls, (double)c[7] / kCalls,
         (int)(pk[2] == pk[4] && pk[2] == pk[5] && pk[2] == pk[6] && pk[2] == pk[7]));
  return 0;
}

// mzgo_tower_dispatch.hpp -- host launchers of the residual-tower engine
// (mzgo_tower.hpp) for one board size, gathered in a table.
#pragma once
#include <cstdlib>

#include "mzgo_tower.hpp"

namespace mzgo {

// action i64 -> i32 with nn.Embedding's range check (err set on a bad index)
hipError_t launch_tact(const int64_t* a, int* out, int B, int A, int* err, hipStream_t s);

struct TowerSet {
  int N;
  hipError_t (*conv)(const TConvArgs&, hipStream_t);
  hipError_t (*chain)(const TConvChain&, int workgroups, hipStream_t);
  hipError_t (*obs)(const TowerArrays&, const SearchParams&, const PlayParams&, const EngineArrays&, int G,
                    hipStream_t);
  hipError_t (*obs_search)(const TowerArrays&, const SearchParams&, const float* obs, int game_base, int move,
                           int G, hipStream_t);
  hipError_t (*root)(const TowerArrays&, const SearchParams&, const EngineArrays&, const double* noise,
                     long long game_stride, int per_move, int G, hipStream_t);
  hipError_t (*select)(const TowerArrays&, const SearchParams&, const EngineArrays&, int G, hipStream_t);
  hipError_t (*expand)(const TowerArrays&, const SearchParams&, const EngineArrays&, int G, hipStream_t);
  // batched steps: k_tbatch (+ k_tboards: the step's board list and count), k_tbexpand
  hipError_t (*batch)(const TowerArrays&, const SearchParams&, const EngineArrays&, int G, int cap_root,
                      int cap_spec, hipStream_t);
  hipError_t (*bexpand)(const TowerArrays&, const SearchParams&, const EngineArrays&, int nb, hipStream_t);
  hipError_t (*choose)(const TowerArrays&, const SearchParams&, const PlayParams&, const EngineArrays&, int G,
                       hipStream_t);
  hipError_t (*search_out)(const TowerArrays&, const SearchParams&, const EngineArrays&, int G, int* visits,
                           double* value, hipStream_t);
  hipError_t (*tin)(const float* src, bf16* dst, int B, int C, int obs6, long long dst_stride, hipStream_t);
  hipError_t (*tout)(const bf16* src, float* dst, int B, int C, hipStream_t);
  hipError_t (*theads)(const TowerArrays&, int B, int has_reward, float* reward, float* value, float* logits,
                       hipStream_t);
};

const TowerSet* find_tower(int N);
#ifdef MZGO_TCONV_STAMPS
int tower_stamps_n19(unsigned long long* out);
#endif

template <int N>
struct TLaunch {
  static hipError_t conv(const TConvArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((k_tconv_ks<N>), dim3(a.nboards * a.co_chunks), dim3(512), 0, s, a);
    return hipGetLastError();
  }
  static hipError_t chain(const TConvChain& c, int workgroups, hipStream_t s) {
    hipLaunchKernelGGL((k_tconv_chain<N>), dim3(workgroups), dim3(512), 0, s, c, c.layers);
    return hipGetLastError();
  }
  static hipError_t obs(const TowerArrays& T, const SearchParams& sp, const PlayParams& pp, const EngineArrays& E,
                        int G, hipStream_t s) {
    hipLaunchKernelGGL((k_tobs<N>), dim3(G), dim3(64), 0, s, T, sp, pp, E);
    return hipGetLastError();
  }
  static hipError_t obs_search(const TowerArrays& T, const SearchParams& sp, const float* obs, int game_base,
                               int move, int G, hipStream_t s) {
    hipLaunchKernelGGL((k_tobs_search<N>), dim3(G), dim3(64), 0, s, T, sp, obs, game_base, move);
    return hipGetLastError();
  }
  static hipError_t root(const TowerArrays& T, const SearchParams& sp, const EngineArrays& E, const double* noise,
                         long long game_stride, int per_move, int G, hipStream_t s) {
    hipLaunchKernelGGL((k_troot<N>), dim3(G), dim3(64), 0, s, T, sp, E, noise, game_stride, per_move);
    return hipGetLastError();
  }
  static hipError_t select(const TowerArrays& T, const SearchParams& sp, const EngineArrays& E, int G,
                           hipStream_t s) {
    hipLaunchKernelGGL((k_tselect<N>), dim3(G), dim3(64), 0, s, T, sp, E);
    return hipGetLastError();
  }
  static hipError_t expand(const TowerArrays& T, const SearchParams& sp, const EngineArrays& E, int G,
                           hipStream_t s) {
    hipLaunchKernelGGL((k_texpand<N>), dim3(G), dim3(64), 0, s, T, sp, E);
    return hipGetLastError();
  }
  static hipError_t batch(const TowerArrays& T, const SearchParams& sp, const EngineArrays& E, int G, int cap_root,
                          int cap_spec, hipStream_t s) {
    hipLaunchKernelGGL((k_tbatch<N>), dim3(G), dim3(64), 0, s, T, sp, E, cap_root, cap_spec);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_tboards<N>), dim3(1), dim3(256), 0, s, T, E, G);
    return hipGetLastError();
  }
  static hipError_t bexpand(const TowerArrays& T, const SearchParams& sp, const EngineArrays& E, int nb,
                            hipStream_t s) {
    hipLaunchKernelGGL((k_tbexpand<N>), dim3(nb), dim3(64), 0, s, T, sp, E);
    return hipGetLastError();
  }
  static hipError_t choose(const TowerArrays& T, const SearchParams& sp, const PlayParams& pp,
                           const EngineArrays& E, int G, hipStream_t s) {
    hipLaunchKernelGGL((k_tchoose<N>), dim3(G), dim3(64), 0, s, T, sp, pp, E);
    return hipGetLastError();
  }
  static hipError_t search_out(const TowerArrays& T, const SearchParams& sp, const EngineArrays& E, int G,
                               int* visits, double* value, hipStream_t s) {
    hipLaunchKernelGGL((k_tsearch_out<N>), dim3(G), dim3(64), 0, s, T, sp, E, visits, value);
    return hipGetLastError();
  }
  static hipError_t tin(const float* src, bf16* dst, int B, int C, int obs6, long long dst_stride, hipStream_t s) {
    hipLaunchKernelGGL((k_tin<N>), dim3(B), dim3(256), 0, s, src, dst, C, obs6, dst_stride);
    return hipGetLastError();
  }
  static hipError_t tout(const bf16* src, float* dst, int B, int C, hipStream_t s) {
    hipLaunchKernelGGL((k_tout<N>), dim3(B), dim3(256), 0, s, src, dst, C);
    return hipGetLastError();
  }
  static hipError_t theads(const TowerArrays& T, int B, int has_reward, float* reward, float* value,
                           float* logits, hipStream_t s) {
    hipLaunchKernelGGL((k_theads<N>), dim3(B), dim3(64), 0, s, T, has_reward, reward, value, logits);
    return hipGetLastError();
  }
  static TowerSet table() {
    return TowerSet{N, &conv, &chain, &obs, &obs_search, &root, &select, &expand, &batch, &bexpand, &choose,
                    &search_out, &tin, &tout, &theads};
  }
};

}  // namespace mzgo

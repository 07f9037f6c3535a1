// mzgo_dispatch.hpp -- host launchers for one (N, C) instantiation of the
// kernels, gathered in a table so the C ABI can dispatch on runtime sizes.
#pragma once
#include "mzgo_kernels.hpp"

namespace mzgo {

struct KernelSet {
  int N, C;
  size_t lds_bytes;
  int rep_scratch;   // floats of HBM scratch per initial_inference item (strip boards), else 0
  int shared_batches;  // 1: the batch expansions stream Y from L2 and take helper workgroups (19x19)
  int tail_convs;      // 1: ended games' workgroups serve running games' parent convs (9x9, tail_help)
  hipError_t (*initial_inference)(const NetParams&, const float* obs, int B, float* lat, float* val,
                                  float* logits, float* scratch, hipStream_t);
  hipError_t (*recurrent_inference)(const NetParams&, const float* lat, const int64_t* act, int B,
                                    float* nlat, float* rew, float* val, float* logits, int* err,
                                    hipStream_t);
  hipError_t (*search)(const NetParams&, const SearchParams&, const EngineArrays&, const float* obs,
                       const double* noise, int G, int game_base, int move, int* visits,
                       double* value, hipStream_t);
  hipError_t (*board_reset)(const EngineArrays&, int G, hipStream_t);
  hipError_t (*board_step)(const EngineArrays&, int G, const int* act, int* status, double* winner,
                           double komi, hipStream_t);
  hipError_t (*board_planes)(const EngineArrays&, int G, double* planes, hipStream_t);
  hipError_t (*selfplay_move)(const NetParams& np, const NetParams& np_b, const SearchParams&,
                              const PlayParams&, const EngineArrays&, int G, hipStream_t);
  hipError_t (*selfplay_boards)(const SearchParams&, const PlayParams&, const EngineArrays&, int G, hipStream_t);
  hipError_t (*search_queue)(const NetParams& np, const SearchParams&, const PlayParams&, const EngineArrays&,
                             int G, int workgroups, hipStream_t);
};

const KernelSet* find_kernels(int N, int C);

template <int N, int C>
struct Launch {
  static hipError_t ii(const NetParams& np, const float* obs, int B, float* lat, float* val,
                       float* logits, float* scratch, hipStream_t s) {
    hipLaunchKernelGGL((k_initial_inference<N, C>), dim3(B), dim3(Geo<N, C>::THREADS), 0, s, np, obs, lat, val, logits,
                       scratch);
    return hipGetLastError();
  }
  static hipError_t ri(const NetParams& np, const float* lat, const int64_t* act, int B, float* nlat,
                       float* rew, float* val, float* logits, int* err, hipStream_t s) {
    hipLaunchKernelGGL((k_recurrent_inference<N, C>), dim3(B), dim3(Geo<N, C>::THREADS), 0, s, np, lat, act, nlat,
                       rew, val, logits, err);
    return hipGetLastError();
  }
  static hipError_t search(const NetParams& np, const SearchParams& sp, const EngineArrays& E,
                           const float* obs, const double* noise, int G, int game_base, int move,
                           int* visits, double* value, hipStream_t s) {
    hipLaunchKernelGGL((k_search<N, C>), dim3(G), dim3(Geo<N, C>::THREADS), 0, s, np, sp, E, obs, noise, game_base,
                       move, visits, value);
    return hipGetLastError();
  }
  static hipError_t breset(const EngineArrays& E, int G, hipStream_t s) {
    hipLaunchKernelGGL((k_board_reset<N, C>), dim3(G), dim3(Geo<N, C>::THREADS), 0, s, E);
    return hipGetLastError();
  }
  static hipError_t bstep(const EngineArrays& E, int G, const int* act, int* status, double* winner,
                          double komi, hipStream_t s) {
    hipLaunchKernelGGL((k_board_step<N, C>), dim3(G), dim3(Geo<N, C>::THREADS), 0, s, E, act, status, winner, komi);
    return hipGetLastError();
  }
  static hipError_t bplanes(const EngineArrays& E, int G, double* planes, hipStream_t s) {
    hipLaunchKernelGGL((k_board_planes<N, C>), dim3(G), dim3(Geo<N, C>::THREADS), 0, s, E, planes);
    return hipGetLastError();
  }
  static hipError_t move(const NetParams& np, const NetParams& np_b, const SearchParams& sp,
                         const PlayParams& pp, const EngineArrays& E, int G, hipStream_t s) {
    hipLaunchKernelGGL((k_selfplay_move<N, C>), dim3(G + sp.helpers), dim3(Geo<N, C>::THREADS), 0, s, np, np_b, sp,
                       pp, E);
    return hipGetLastError();
  }
  static hipError_t boards(const SearchParams& sp, const PlayParams& pp, const EngineArrays& E, int G, hipStream_t s) {
    hipLaunchKernelGGL((k_selfplay_boards<N, C>), dim3(G), dim3(BoardsGeo<Geo<N, C>>::THREADS), 0, s, sp, pp, E);
    return hipGetLastError();
  }
  static hipError_t queue(const NetParams& np, const SearchParams& sp, const PlayParams& pp, const EngineArrays& E,
                          int G, int workgroups, hipStream_t s) {
    hipLaunchKernelGGL((k_search_queue<N, C>), dim3(workgroups), dim3(Geo<N, C>::THREADS), 0, s, np, sp, pp, E, G);
    return hipGetLastError();
  }
  static KernelSet table() {
    typedef Geo<N, C> G;
    return KernelSet{N, C, sizeof(Smem<G>), rep_needs_scratch<G>() ? 64 * N * N : 0,
                     Smem<G>::GLOBAL_Y ? 1 : 0, TailConvs<G>::value ? 1 : 0, &ii, &ri, &search, &breset, &bstep,
                     &bplanes,
                     &move, &boards, &queue};
  }
};

}  // namespace mzgo

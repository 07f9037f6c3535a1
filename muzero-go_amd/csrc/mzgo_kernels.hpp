// mzgo_kernels.hpp -- the engine's kernels, templated on board size N and
// latent_dim C and instantiated per (N, C) in mzgo_kernels_N*.hip.
//
// Every kernel runs one workgroup (4 waves) per game / batch element; games
// never talk to each other, so there is no inter-workgroup synchronisation.
#pragma once
#include "mzgo_board.hpp"
#include "mzgo_conv.hpp"
#include "mzgo_expand.hpp"
#include "mzgo_search.hpp"
#include "mzgo_wino.hpp"

namespace mzgo {

// Network parameters on the device (packed by mzgo_capi.cpp).
struct NetParams {
  const float* w_conv1; const float* b_conv1;   // representation.conv1 (6 -> 64)
  const float* w_conv2; const float* b_conv2;   // representation.conv2 (64 -> 64)
  const float* w_conv3; const float* b_conv3;   // representation.conv3 (64 -> C)
  const float* w_dyn;   const float* b_dyn;     // dynamics.conv (C -> C)
  const float* emb;                             // dynamics.action_embedding [A][C]
  const float* head_w;                          // [3][C]: reward_conv, value_conv, policy_conv
  const float* etab;                            // [A][9][C] action-tap table (mzgo_expand.hpp)
  HeadScalars hs;
};

// b ? x : y, field by field (kernel-argument pointers stay known-global, so
// their loads are global loads, not flat ones)
__device__ __forceinline__ NetParams select_params(bool b, const NetParams& x, const NetParams& y) {
  NetParams n;
#define MZGO_SEL(f) n.f = b ? x.f : y.f;
  MZGO_SEL(w_conv1) MZGO_SEL(b_conv1) MZGO_SEL(w_conv2) MZGO_SEL(b_conv2) MZGO_SEL(w_conv3) MZGO_SEL(b_conv3)
  MZGO_SEL(w_dyn) MZGO_SEL(b_dyn) MZGO_SEL(emb) MZGO_SEL(head_w) MZGO_SEL(etab)
  MZGO_SEL(hs.reward_b) MZGO_SEL(hs.fc1_w) MZGO_SEL(hs.fc1_b) MZGO_SEL(hs.fc2_w) MZGO_SEL(hs.fc2_b)
  MZGO_SEL(hs.value_b) MZGO_SEL(hs.vfc_w) MZGO_SEL(hs.vfc_b) MZGO_SEL(hs.policy_b) MZGO_SEL(hs.pass_logit)
#undef MZGO_SEL
  return n;
}

// A kernel-argument pointer made opaque to the optimizer at this point of the
// program (an empty asm on its SGPR pair) and re-marked global: address
// arithmetic derived from it cannot be hoisted above the point.  The
// whole-game k_selfplay_move launders its arguments at the head of every move,
// so per-lane addresses are formed per move instead of once at the kernel
// entry and kept (spilled) across the whole game.
template <class T>
__device__ __forceinline__ T* launder_global(T* p) {
  unsigned long long x = reinterpret_cast<unsigned long long>(p);
  asm volatile("" : "+s"(x));
  return (T*)reinterpret_cast<__attribute__((address_space(1))) T*>(x);
}
// The search's f64 parameters made opaque per move as well: the constants
// derived from them (the Gamma sampler's d and 1 / sqrt(9 d), f32 1 - eps)
// are then formed per move instead of being hoisted to the kernel entry and
// kept (spilled, k_selfplay_move<19,96>) across the whole game
__device__ __forceinline__ double launder_f64(double v) {
  unsigned long long x = (unsigned long long)__double_as_longlong(v);
  asm volatile("" : "+s"(x));
  return __longlong_as_double((long long)x);
}
__device__ __forceinline__ SearchParams launder_search(const SearchParams& p) {
  SearchParams r = p;
  r.c_puct = launder_f64(p.c_puct);
  r.discount = launder_f64(p.discount);
  r.dirichlet_alpha = launder_f64(p.dirichlet_alpha);
  r.dirichlet_epsilon = launder_f64(p.dirichlet_epsilon);
  r.pass_epsilon = launder_f64(p.pass_epsilon);
  return r;
}
__device__ __forceinline__ NetParams launder_params(const NetParams& n) {
  NetParams r;
#define MZGO_L(f) r.f = launder_global(n.f);
  MZGO_L(w_conv1) MZGO_L(b_conv1) MZGO_L(w_conv2) MZGO_L(b_conv2) MZGO_L(w_conv3) MZGO_L(b_conv3)
  MZGO_L(w_dyn) MZGO_L(b_dyn) MZGO_L(emb) MZGO_L(head_w) MZGO_L(etab)
  MZGO_L(hs.reward_b) MZGO_L(hs.fc1_w) MZGO_L(hs.fc1_b) MZGO_L(hs.fc2_w) MZGO_L(hs.fc2_b)
  MZGO_L(hs.value_b) MZGO_L(hs.vfc_w) MZGO_L(hs.vfc_b) MZGO_L(hs.policy_b) MZGO_L(hs.pass_logit)
#undef MZGO_L
  return r;
}

constexpr int kCounters = 9;     // EngineArrays::counters

// Per-slot device state of an engine (sizes fixed at engine creation).
struct EngineArrays {
  int S;                 // simulations per move this engine was sized for
  int max_moves;
  // search state
  float* pool;           // [G][S+2][C*CS] per node: latent [C][CS] (direct dynamics) or conv
                         // output Y [CELLS][C] (factored); slot S+1: scratch latent
  float* prior;          // [G][S+1][A]
  int* child;            // [G][S+1][A]
  int* visits;           // [G][S+1]
  double* wsum;          // [G][S+1]
  double* root_prior;    // [G][A]
  int* path;             // [G][S+2]
  int* nodes;            // [G]  nodes used by the last search
  int* nact;             // [G][S+1] action that created each node (factored: rebuilds its latent)
  // boards
  int8_t* stones;        // [G][CELLS]
  uint8_t* invd;         // [G][CELLS]
  int* meta;             // [G][4] BoardMeta
  // self-play records
  int8_t* rec_stones;    // [G][M][CELLS]
  uint8_t* rec_invd;     // [G][M][CELLS]
  uint8_t* rec_flags;    // [G][M]   bit0 turn, bit1 passed, bit2 done
  int* rec_action;       // [G][M]
  double* rec_value;     // [G][M]
  double* rec_policy;    // [G][M][A]
  double* rec_reward;    // [G][M]
  int* game_len;         // [G]
  double* final_reward;  // [G]
  int* status;           // [G]  0 playing, 1 finished, >=16 error
  unsigned char* jobs;   // [G][job_bytes(A)] batch-expansion jobs shared with helper workgroups
  int* mpq;              // [2G + 1] move-parallel epoch (k_search_queue): per game (first move,
                         // moves played) of k_selfplay_boards, then the queue head
  unsigned long long* counters;  // [kCounters] 0: simulations run, 1: moves played, 2: games finished,
                                 //     3: dynamics convs run (factored: one per new parent; tower
                                 //     engines: towers evaluated, speculative ones included),
                                 //     4: of those, tail conv jobs (conv_tail), 5: prior rows formed,
                                 //     6: game workgroups started (k_selfplay_move), 7: tail helpers
                                 //     whose bounded wait for a job expired (tail_help), 8: expired
                                 //     mzgo_stream_wait_started gates (reported, then cleared)
  unsigned long long* stamps;    // [G][kStampPhases] phase cycles (MZGO_STAMPS builds only)
};

__device__ __forceinline__ EngineArrays launder_arrays(const EngineArrays& e) {
  EngineArrays r = e;
#define MZGO_L(f) r.f = launder_global(e.f);
  MZGO_L(pool) MZGO_L(prior) MZGO_L(child) MZGO_L(visits) MZGO_L(wsum) MZGO_L(root_prior) MZGO_L(path)
  MZGO_L(nodes) MZGO_L(nact) MZGO_L(stones) MZGO_L(invd) MZGO_L(meta) MZGO_L(rec_stones) MZGO_L(rec_invd)
  MZGO_L(rec_flags) MZGO_L(rec_action) MZGO_L(rec_value) MZGO_L(rec_policy) MZGO_L(rec_reward) MZGO_L(game_len)
  MZGO_L(final_reward) MZGO_L(status) MZGO_L(jobs) MZGO_L(mpq) MZGO_L(counters) MZGO_L(stamps)
#undef MZGO_L
  return r;
}

template <class G>
struct TreeViewOf {
  __device__ __forceinline__ static TreeView make(const EngineArrays& E, int g) {
    const size_t n1 = (size_t)E.S + 1;
    TreeView T;
    T.prior = E.prior + (size_t)g * n1 * G::A;
    T.child = E.child + (size_t)g * n1 * G::A;
    T.visits = E.visits + (size_t)g * n1;
    T.wsum = E.wsum + (size_t)g * n1;
    T.root_prior = E.root_prior + (size_t)g * G::A;
    T.path = E.path + (size_t)g * (n1 + 1);
    return T;
  }
};

// LDS of one game's workgroup: direct-conv boards (weight DMA rings) ...
template <class G, bool W = G::WINO>
struct Smem {
  union alignas(16) {
    float in[G::CINMAX * G::CPAD];                       // conv staging
    float hp[2 * 3 * G::CS];                             // head partials (after the conv loop)
    struct { int label[G::CELLS], libs[G::CELLS], gsize[G::CELLS]; } scr;  // board step
    ExpandLds<G, G::CINMAX * G::CPAD> f;   // factored expansion
  } u;
  alignas(16) float ring[RingBytes<G>::value / 4];       // weight DMA ring
  TreeLds<G> t;
  int8_t stone[G::CELLS];
  uint8_t invd[G::CELLS];
  int killed[4];
  int misc[8];
  int bc[8];                                             // broadcast slots
  // a batching configuration's buffers were sized to the union's budget
  // a batching configuration's buffers were sized to the union's budget (a
  // non-batching one may grow the union: the kernels assert the whole Smem
  // fits one CU's LDS)
  static_assert(!ExpandLds<G, G::CINMAX * G::CPAD>::BATCH ||
                    sizeof(ExpandLds<G, G::CINMAX * G::CPAD>) <= sizeof(float) * G::CINMAX * G::CPAD,
                "the batched expansion's LDS must fit the conv staging it overlays");
  __device__ float* heads() { return u.hp; }
  __device__ float* ulds() { return u.in; }             // the union as scratch
  static constexpr bool GLOBAL_Y = ExpandLds<G, G::CINMAX * G::CPAD>::GLOBAL_Y;
  static constexpr int HEAD_PARTS = ConvShape<G::C>::NCOG;
};

// ... and Winograd boards (transformed input; exchange buffer + head partials)
template <class G>
struct Smem<G, true> {
  union alignas(16) {
    float in[8 * G::CPAD];                               // conv1 input (6 planes + 2 zero)
    float v[Wino<G>::template v_floats<G::CINMAX>()];    // transformed conv input
    struct {
      float red[Wino<G>::template red_floats<G::C>()];
      float hp[(G::C / 16) * 3 * Wino<G>::HS];   // head partials of one strip
      alignas(16) float outs[G::C * Wino<G>::OUT_STRIDE];   // conv output staging
    } x;
    struct { int label[G::CELLS], libs[G::CELLS], gsize[G::CELLS]; } scr;  // board step
    ExpandLds<G, Wino<G>::template v_floats<G::CINMAX>()> f;
  } u;
  alignas(16) float raw[WinoRaw<G>::FLOATS];              // per-wave staging of conv input rows
  static constexpr bool STRIPS = Wino<G>::NSTRIP > 1;
  alignas(16) float hfin[STRIPS ? 3 * G::CS : 4];         // strip boards: summed head partials
  TreeLds<G> t;
  int8_t stone[G::CELLS];
  uint8_t invd[G::CELLS];
  int killed[4];
  int misc[8];
  int bc[8];
  static_assert(!ExpandLds<G, Wino<G>::template v_floats<G::CINMAX>()>::BATCH ||
                    sizeof(ExpandLds<G, Wino<G>::template v_floats<G::CINMAX>()>) <=
                        sizeof(float) * Wino<G>::template v_floats<G::CINMAX>(),
                "the batched expansion's LDS must fit the Winograd input it overlays");
  __device__ float* heads() { return STRIPS ? hfin : u.x.hp; }
  __device__ float* ulds() { return u.v; }              // the union as scratch
  static constexpr bool GLOBAL_Y = ExpandLds<G, Wino<G>::template v_floats<G::CINMAX>()>::GLOBAL_Y;
  static constexpr int HEAD_PARTS = STRIPS ? 1 : G::C / 16;
};

// One latent conv: src ([CIN][src_stride], global) (+ emb per channel) ->
// dst ([COUT][dst_stride], cells < out_cells), NH fused 1x1 head partials left
// in sm.heads().  All threads; returns synchronised.
// Factored Y of a conv (YM) written to LDS too, as the expansion's copy L.yc
// (CACHE boards, one strip): yc overlays only the exchange buffer, which is
// dead when the epilogue stores (wino_conv's YM store loop reads outs).
template <class G>
__device__ __forceinline__ float* y_lds_target(Smem<G>& sm) {
  if constexpr (G::WINO && decltype(sm.u.f)::CACHE && Wino<G>::NSTRIP == 1) {
    static_assert(sizeof(sm.u.f.yc) <= sizeof(sm.u.x.red), "the LDS Y copy overlays only the exchange buffer");
    return sm.u.f.yc;
  } else {
    return nullptr;
  }
}
// the head weights of the expansion (the rest of load_y, after a conv that
// left Y in L.yc)
template <class G>
__device__ __forceinline__ void load_hw(Smem<G>& sm, const float* head_w) {
  for (int i = tid_local(); i < 3 * G::C; i += G::THREADS) sm.u.f.hw[i] = head_w[i];
}

template <class G, int CIN, int COUT, int NH, bool YM = false>
__device__ __forceinline__ void latent_conv(Smem<G>& sm, const float* __restrict__ w, const float* __restrict__ b,
                                            const float* src, int src_stride, const float* emb, float* dst,
                                            int dst_stride, int out_cells, const float* head_w,
                                            Stamp* st = nullptr, float* ylds = nullptr) {
  if constexpr (G::WINO) {
    // row strips (19x19): strip s reads rows s*SROWS-1 .. (s+1)*SROWS of src,
    // so src must not alias dst (representation ping-pongs through scratch)
    for (int s = 0; s < Wino<G>::NSTRIP; ++s) {
      wino_input<G, CIN>(sm.u.v, sm.raw, src, src_stride, emb, s, st);
      if (st) st->lap(1);
      wino_conv<G, CIN, COUT, NH, YM>(sm.u.v, sm.u.x.red, sm.u.x.hp, sm.u.x.outs, sm.hfin, w, b, dst, dst_stride,
                                  out_cells, head_w, s, st, ylds);
    }
    if constexpr (Wino<G>::NSTRIP > 1) __syncthreads();   // hfin complete
  } else {
    stage_board<G>(sm.u.in, src, src_stride, CIN, emb);
    __syncthreads();
    if (st) st->lap(1);
    conv3x3_ring<G, CIN, COUT, NH, YM>(sm.u.in, sm.ring, w, b, dst, dst_stride, out_cells, head_w, sm.u.hp, st);
  }
}

// The dynamics conv of a node whose latent is rebuilt from its parent's Y
// and E[a] (Winograd boards): latent_conv with wino_input_rebuilt as the
// input transform -- no materialized copy of the latent.  All threads;
// returns synchronised (strip boards) / with the stores issued (one strip).
template <class G>
__device__ __forceinline__ void latent_conv_rebuilt(Smem<G>& sm, const NetParams& np, const float* ypar,
                                                    const float* ea, float* dst, Stamp* st = nullptr,
                                                    float* ylds = nullptr, bool par_in_lds = false) {
  if constexpr (G::WINO && Wino<G>::NSTRIP == 1) {
    // (the second channel slab transformed under the GEMM's first K half)
    wino_conv_rebuilt<G>(sm.u.v, sm.raw, sm.u.x.red, sm.u.x.hp, sm.u.x.outs, sm.hfin, ypar, ea, np.w_dyn, np.b_dyn,
                         dst, st, ylds, par_in_lds ? ylds : nullptr);
  } else if constexpr (G::WINO) {
    for (int s = 0; s < Wino<G>::NSTRIP; ++s)
      wino_conv_rebuilt<G>(sm.u.v, sm.raw, sm.u.x.red, sm.u.x.hp, sm.u.x.outs, sm.hfin, ypar, ea, np.w_dyn,
                           np.b_dyn, dst, st, ylds, par_in_lds ? ylds : nullptr, s);
    if constexpr (Wino<G>::NSTRIP > 1) __syncthreads();
  }
}

template <class G>
__device__ __forceinline__ BoardLds<G> board_lds(Smem<G>& sm) {
  BoardLds<G> b;
  b.stone = sm.stone; b.invd = sm.invd;
  b.label = sm.u.scr.label; b.libs = sm.u.scr.libs; b.gsize = sm.u.scr.gsize;
  b.killed = sm.killed; b.misc = sm.misc;
  return b;
}

// ---------------------------------------------------------------------------
// representation (self_play.py:70-74) + prediction heads (:104-113).
// planes(c, cell) gives the f32 observation.  The latent is written to
// ``lat`` ([C][lat_stride]), which also serves as scratch for conv1/conv2;
// strip boards put conv2's output in ``scr`` ([64][lat_stride]) instead (a
// strip conv cannot run in place).
// Leaves the logits in sm.t.logits and the value in sm.t.value.
// ---------------------------------------------------------------------------
template <class G>
constexpr bool rep_needs_scratch() {
  if constexpr (G::WINO) return Wino<G>::NSTRIP > 1;
  else return false;
}

// conv2 / conv3 of the representation as jobs (run_search's RepJobs on
// 19x19 with helper workgroups): jobs(k) runs conv k and returns true, or
// returns false for the workgroup's own latent_conv.
struct NoRepJobs {
  __device__ bool operator()(int) const { return false; }
};

template <class G, class PlaneFn, class Jobs = NoRepJobs>
__device__ __forceinline__ void representation(Smem<G>& sm, const NetParams& np, PlaneFn planes, float* lat,
                                      int lat_stride, float* scr, unsigned long long* ts = nullptr,
                                      Jobs jobs = Jobs{}) {
  float* mid = rep_needs_scratch<G>() ? scr : lat;
  for (int i = tid_local(); i < 6 * G::CELLS; i += G::THREADS) {
    const int c = i / G::CELLS, j = i - c * G::CELLS;
    sm.u.in[c * G::CPAD + j] = planes(c, j);
  }
  zero_channels<G>(sm.u.in, 6, 8);
  stage_head_scalars(np.hs, sm.t.hsc);
  __syncthreads();
  HeadPart<G> hp{nullptr};
  const int oc = lat_stride == G::CS ? G::CS : G::CELLS;   // pooled latents also write their 0 pads
  conv3x3_direct<G, 6, 64, 0, 1>(sm.u.in, np.w_conv1, np.b_conv1, lat, lat_stride, oc, nullptr, hp);
  __syncthreads();
#ifdef MZGO_STAMPS
  if (ts) ts[0] = __builtin_amdgcn_s_memtime();
#endif
  if (!jobs(2))
    latent_conv<G, 64, 64, 0>(sm, np.w_conv2, np.b_conv2, lat, lat_stride, nullptr, mid, lat_stride, oc, nullptr);
  __syncthreads();                                         // conv2's stores before conv3 reads them
#ifdef MZGO_STAMPS
  if (ts) ts[1] = __builtin_amdgcn_s_memtime();
#endif
  if (!jobs(3))
    latent_conv<G, 64, G::C, 2>(sm, np.w_conv3, np.b_conv3, mid, lat_stride, nullptr, lat, lat_stride, oc,
                                np.head_w + G::C);
  if (wave_id() == 0)
    finalize_heads<G, Smem<G>::HEAD_PARTS>(sm.heads(), false, sm.t.hsc, sm.t.logits, &sm.t.reward, &sm.t.value);
  __syncthreads();
}

// dynamics (self_play.py:85-95) + prediction: ``src`` latent + emb[action]
// -> ``dst`` latent; logits/reward/value left in sm.t.
template <class G>
__device__ __forceinline__ void dynamics(Smem<G>& sm, const NetParams& np, const float* src, int src_stride,
                                int action, float* dst, int dst_stride) {
  stage_head_scalars(np.hs, sm.t.hsc);
  latent_conv<G, G::C, G::C, 3>(sm, np.w_dyn, np.b_dyn, src, src_stride, np.emb + (size_t)action * G::C, dst,
                                dst_stride, dst_stride == G::CS ? G::CS : G::CELLS, np.head_w);
  if (wave_id() == 0)
    finalize_heads<G, Smem<G>::HEAD_PARTS>(sm.heads(), true, sm.t.hsc, sm.t.logits, &sm.t.reward, &sm.t.value);
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Batched drop-in inference (self_play.py:121-128)
// ---------------------------------------------------------------------------
template <int N, int C>
__global__ void __launch_bounds__((Geo<N, C>::THREADS)) __attribute__((amdgpu_waves_per_eu(Geo<N, C>::WPE, Geo<N, C>::WPE))) k_initial_inference(NetParams np, const float* __restrict__ obs,
                                                                 float* latent, float* value, float* logits,
                                                                 float* scratch) {
  typedef Geo<N, C> G;
  __shared__ Smem<G> sm;
  static_assert(sizeof(Smem<G>) <= 160 * 1024, "one workgroup per CU: the whole LDS at most");
  if constexpr (G::WINO) wino_raw_zero<G>(sm.raw);        // zero halo of the conv input planes
  const int b = blockIdx.x;
  const float* o = obs + (size_t)b * 6 * G::CELLS;
  float* lat = latent + (size_t)b * G::C * G::CELLS;
  float* scr = scratch ? scratch + (size_t)b * 64 * G::CELLS : nullptr;
  representation<G>(sm, np, [&](int c, int j) { return o[c * G::CELLS + j]; }, lat, G::CELLS, scr);
  for (int a = tid_local(); a < G::A; a += G::THREADS) logits[(size_t)b * G::A + a] = sm.t.logits[a];
  if (tid_local() == 0) value[b] = sm.t.value;
}

template <int N, int C>
__global__ void __launch_bounds__((Geo<N, C>::THREADS)) __attribute__((amdgpu_waves_per_eu(Geo<N, C>::WPE, Geo<N, C>::WPE))) k_recurrent_inference(NetParams np, const float* __restrict__ latent,
                                                                   const int64_t* __restrict__ action,
                                                                   float* next_latent, float* reward,
                                                                   float* value, float* logits, int* err) {
  typedef Geo<N, C> G;
  __shared__ Smem<G> sm;
  static_assert(sizeof(Smem<G>) <= 160 * 1024, "one workgroup per CU: the whole LDS at most");
  if constexpr (G::WINO) wino_raw_zero<G>(sm.raw);        // zero halo of the conv input planes
  const int b = blockIdx.x;
  int64_t a = action[b];
  if (a < 0 || a >= G::A) {            // nn.Embedding would raise IndexError
    if (tid_local() == 0) atomicOr(err, 1);
    a = 0;
  }
  dynamics<G>(sm, np, latent + (size_t)b * G::C * G::CELLS, G::CELLS, (int)a,
              next_latent + (size_t)b * G::C * G::CELLS, G::CELLS);
  for (int i = tid_local(); i < G::A; i += G::THREADS) logits[(size_t)b * G::A + i] = sm.t.logits[i];
  if (tid_local() == 0) { reward[b] = sm.t.reward; value[b] = sm.t.value; }
}

// ---------------------------------------------------------------------------
// One full MCTS.run (self_play.py:148-237) for game slot g.
// ---------------------------------------------------------------------------
// Game g's node slots: S+1 nodes + one scratch latent (slot S+1).
template <class G>
__device__ __forceinline__ float* pool_of(const EngineArrays& E, int g) {
  return E.pool + (size_t)g * ((size_t)E.S + 2) * G::C * G::CS;
}

// Batch expansion (factored dynamics): children i < B of one parent whose Y
// is in L.yc (and the head weights in L.hw), child i = node nid0 + i via
// action L.acts[i]; one wave per child: E[a] into LDS, heads, the child's
// prior row and child row (LAZY: neither -- the lazy policy head, see
// TreeLds::rawp), L.bv[i] = its backup value r + discount * v.  Each wave claims the next child
// (sm.t.ngrab, reset with sm.t.npick by the caller) and waits until
// sm.t.npick > k (wave 0 publishes the actions, pick_sequence, before it
// joins).  All threads; the caller synchronises.
template <class G, bool LAZY>
__device__ __forceinline__ void batch_expand(Smem<G>& sm, const NetParams& np, const SearchParams& sp,
                                             const TreeView& TV, int B, int nid0, const float* yg,
                                             Stamp* st = nullptr) {
  auto& L = sm.u.f;
  typedef decltype(sm.u.f) XL;
  if (st && tid_local() == 0) { st->wave_add(48, 1); st->wave_add(55, (unsigned long long)B); }   // batches, children
  if constexpr (XL::GLOBAL_Y && !LAZY) {
    // Y streamed from L2 (19x19): a wave claims two children at a time and
    // reads the parent's Y once for both (expand_wave2)
    const int wave = __builtin_amdgcn_readfirstlane(wave_id());
    const int lane = lane_id_local();
    auto& W = L.wv[wave];
    ExpandPlan<G> plan;
    plan.init(L.rpair);
    constexpr int E4N = 9 * G::C / 4;
    f32x4* ew0 = reinterpret_cast<f32x4*>(W.ew);
    f32x4* ew1 = reinterpret_cast<f32x4*>(W.ew2);
    // the child's heads, prior row and child row from its totals and the
    // policy sums in W.xw (as the one-child loop below)
    auto child_rows = [&](int k, float rsum, float vsum) {
      const int nid = nid0 + k;
      float r, v;
      heads_from_totals<G>(rsum, vsum, sm.t.hsc, r, v);
      float x[G::AP];
      policy_logits<G>(W.xw + XL::PROW, sm.t.hsc, x);
      int* crow = TV.child + (size_t)nid * G::A;
      for (int i = lane; i < G::A; i += 64) crow[i] = -1;
      child_priors<G>(sm.t, x, TV.prior + (size_t)nid * G::A, -1, sp.variant, W.fscratch(), W.dscratch());
      if (lane == 0) L.bv[k] = (double)r + sp.discount * (double)v;
    };
    // the lazy policy head (sp.lazy_rows; self-play): the totals only, and
    // the sentinel kLazyRow in child-row entry 0 -- a select that first
    // reaches the node forms its logits and priors (expand_child's LAZYH)
    auto lazy_child = [&](int k, float rsum, float vsum) {
      float r, v;
      heads_from_totals<G>(rsum, vsum, sm.t.hsc, r, v);
      if (lane == 0) {
        TV.child[(size_t)(nid0 + k) * G::A] = kLazyRow;
        L.bv[k] = (double)r + sp.discount * (double)v;
      }
    };
    const bool lazy = sp.lazy_rows != 0;
    for (;;) {
      int k = 0;
      if (lane == 0) k = atomicAdd(&sm.t.ngrab, 2);
      k = __builtin_amdgcn_readfirstlane(k);
      if (k >= B) break;
      const bool two = k + 1 < B;
      const int need = two ? k + 1 : k;
      while (__hip_atomic_load(&sm.t.npick, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= need)
        __builtin_amdgcn_s_sleep(2);
      const int a0 = __builtin_amdgcn_readfirstlane(L.acts[k]);
      const f32x4* e0 = reinterpret_cast<const f32x4*>(np.etab + (size_t)a0 * 9 * G::C);
      for (int i = lane; i < E4N; i += 64) ew0[i] = e0[i];
      if (two) {
        const int a1 = __builtin_amdgcn_readfirstlane(L.acts[k + 1]);
        const f32x4* e1 = reinterpret_cast<const f32x4*>(np.etab + (size_t)a1 * 9 * G::C);
        for (int i = lane; i < E4N; i += 64) ew1[i] = e1[i];
      }
      wave_lds_sync();
      if (lazy) {
        if (two) {
          float r0, v0, r1, v1;
          Pol2<G> pol;
          expand_wave2<G, XL::PROW, false>(W.xw, yg, W.ew, W.ew2, L.hw, plan, r0, v0, r1, v1, pol);
          lazy_child(k, r0, v0);
          lazy_child(k + 1, r1, v1);
        } else {
          float rsum, vsum;
          expand_wave<G, XL::PROW, false>(W.xw, yg, W.ew, L.hw, plan, rsum, vsum);
          lazy_child(k, rsum, vsum);
        }
      } else if (two) {
        float r0, v0, r1, v1;
        Pol2<G> pol;
        expand_wave2<G, XL::PROW>(W.xw, yg, W.ew, W.ew2, L.hw, plan, r0, v0, r1, v1, pol);
        wave_lds_sync();
        child_rows(k, r0, v0);
        wave_lds_sync();                     // child k's reads of W.xw / W.ew before child k + 1's
        store_policy2<G, XL::PROW>(W.xw, pol);
        wave_lds_sync();
        child_rows(k + 1, r1, v1);
      } else {
        float rsum, vsum;
        expand_wave<G, XL::PROW, true>(W.xw, yg, W.ew, L.hw, plan, rsum, vsum);
        wave_lds_sync();
        child_rows(k, rsum, vsum);
      }
      if (st) st->wave_add(68, two ? 2 : 1);
      wave_lds_sync();                       // W.ew / W.xw reused by the wave's next pair
    }
  } else if constexpr (XL::BATCH) {
    const int wave = __builtin_amdgcn_readfirstlane(wave_id());
    const int lane = lane_id_local();
    auto& W = L.wv[wave];
    ExpandPlan<G> plan;
    plan.init(L.rpair);
    // E[a] of the wave's next child, loaded into registers while the current
    // child's heads and rows are written (its action is published by then
    // unless the picks are late; the copy then reads E at the top)
    constexpr int E4N = 9 * G::C / 4, EP = (E4N + 63) / 64;
    f32x4 epre[EP];
    int epre_a = -1;
    f32x4* ewl = reinterpret_cast<f32x4*>(W.ew);
    // children are claimed one at a time (wave 0 joins late, after the picks)
    auto grab = [&]() {
      int v = 0;
      if (lane == 0) v = atomicAdd(&sm.t.ngrab, 1);
      return __builtin_amdgcn_readfirstlane(v);
    };
    for (int k = grab(), kn; k < B; k = kn) {
      while (__hip_atomic_load(&sm.t.npick, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= k)
        __builtin_amdgcn_s_sleep(2);
      unsigned long long t0 = st ? st->now() : 0, t1;
      const int a = __builtin_amdgcn_readfirstlane(L.acts[k]), nid = nid0 + k;
      if (a == epre_a) {
#pragma unroll
        for (int e = 0; e < EP; ++e)
          if (lane + 64 * e < E4N) ewl[lane + 64 * e] = epre[e];
      } else {
        const f32x4* e4 = reinterpret_cast<const f32x4*>(np.etab + (size_t)a * 9 * G::C);
        for (int i = lane; i < E4N; i += 64) ewl[i] = e4[i];
      }
      wave_lds_sync();
      if (st) { t1 = st->now(); st->wave_add(64, t1 - t0); t0 = t1; }
      float rsum, vsum;
      if constexpr (XL::GLOBAL_Y) expand_wave<G, XL::PROW, !LAZY>(W.xw, yg, W.ew, L.hw, plan, rsum, vsum);
      else expand_wave<G, XL::PROW, !LAZY>(W.xw, L.yc, W.ew, L.hw, plan, rsum, vsum);
      wave_lds_sync();
      epre_a = -1;
      kn = grab();
      {
        if (kn < B && __hip_atomic_load(&sm.t.npick, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) > kn) {
          epre_a = __builtin_amdgcn_readfirstlane(L.acts[kn]);
          const f32x4* e4 = reinterpret_cast<const f32x4*>(np.etab + (size_t)epre_a * 9 * G::C);
#pragma unroll
          for (int e = 0; e < EP; ++e) epre[e] = e4[lane + 64 * e < E4N ? lane + 64 * e : 0];
        }
      }
      if (st) { t1 = st->now(); st->wave_add(65, t1 - t0); t0 = t1; }
      float r, v;
      heads_from_totals<G>(rsum, vsum, sm.t.hsc, r, v);
      if (st) { t1 = st->now(); st->wave_add(66, t1 - t0); t0 = t1; }
      if constexpr (LAZY) {
        // no policy head: a select that first reaches the child forms its
        // logits (select_leaf -> kNeedLogits -> policy_sums_wg); most never do
        if (lane == 0) atomicOr(&sm.t.rawp[nid >> 5], 1u << (nid & 31));
      } else {
        float x[G::AP];
        policy_logits<G>(W.xw + XL::PROW, sm.t.hsc, x);
        int* crow = TV.child + (size_t)nid * G::A;
        for (int i = lane; i < G::A; i += 64) crow[i] = -1;
        child_priors<G>(sm.t, x, TV.prior + (size_t)nid * G::A, -1, sp.variant, W.fscratch(), W.dscratch());
      }
      if (lane == 0) L.bv[k] = (double)r + sp.discount * (double)v;
      wave_lds_sync();                     // W.ew / W.xw reused by the wave's next child
      if (st) { t1 = st->now(); st->wave_add(67, t1 - t0); st->wave_add(68, 1); }
    }
  }
}

// Node n's Y (global, [CELLS][C]) and the head weights into the LDS copies
// (GLOBAL_Y boards: the head weights and expand_wave's region-offset table
// only).  All threads; the caller synchronises.
template <class G>
__device__ __forceinline__ void load_y(Smem<G>& sm, const float* y, const float* head_w) {
  auto& L = sm.u.f;
  typedef decltype(sm.u.f) XL;
  if constexpr (XL::CACHE) {
    const f32x4* src = reinterpret_cast<const f32x4*>(y);
    f32x4* dst = reinterpret_cast<f32x4*>(L.yc);
    for (int i = tid_local(); i < G::CELLS * G::C / 4; i += G::THREADS) dst[i] = src[i];
  }
  if constexpr (XL::CACHE || XL::BATCH)
    for (int i = tid_local(); i < 3 * G::C; i += G::THREADS) L.hw[i] = head_w[i];
  if constexpr (XL::GLOBAL_Y)
    for (int i = tid_local(); i < XL::RPAIRS; i += G::THREADS) L.rpair[i] = ExpandPlan<G>::pair_entry(i >> 3, i & 7);
}

// ---------------------------------------------------------------------------
// Batch expansions shared with helper workgroups (GLOBAL_Y boards, 19x19).
// A 19x19 game has one workgroup, so with 64 games 192 CUs would idle; the
// self-play launch adds sp.helpers workgroups (3 per game), and a game's
// batch expansion (up to A children, each an L2 stream of its leaf's Y)
// becomes a job that its workgroup and its helpers share: the game's
// workgroup publishes the job (the actions, the leaf, the children's node
// ids), every workgroup claims children a round of WAVES at a time, computes
// them exactly as batch_expand does (the same function per child) and writes
// the rows and backup values to HBM; the game's workgroup waits until all B
// are done, then continues.  It never waits for a helper to START (it claims
// children itself until none are left), so nothing depends on helpers being
// resident.  Hand-offs: agent-scope release / relaxed flag / agent-scope
// acquire (cdna_hip_programming.md Guideline 16); claims: a CAS on one
// 64-bit word (batch number << 32 | next child), so a claim of a finished
// batch fails.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int job_bytes(int A) {
  return 512 + 2 * ((A * 8 + 255) / 256 * 256) + (A + 255) / 256 * 256 + ((A - 1 + 15) / 16 * 16 * 12 + 255) / 256 * 256;
}
constexpr unsigned kJobExit = 0xFFFFFFFFu;
// s_sleep units (64 clocks) between polls: a game waiting for its job's units,
// a helper waiting for the next job ((1, 2) measured the same)
constexpr int kJobWaitSleep = 4, kJobPollSleep = 8;
struct JobView {
  unsigned char* base;
  __device__ unsigned long long* claim() const { return reinterpret_cast<unsigned long long*>(base); }
  __device__ unsigned* seq() const { return reinterpret_cast<unsigned*>(base + 64); }
  __device__ unsigned* done() const { return reinterpret_cast<unsigned*>(base + 128); }
  // B, nid0 (conv: the parent), leaf, net, kind (0 batch, 1 conv of src, 2 conv of a rebuilt latent,
  // 3 replay checks), action (3: the root action), depth, batch size
  __device__ int* info() const { return reinterpret_cast<int*>(base + 192); }
  __device__ double* pass_prior() const { return reinterpret_cast<double*>(base + 224); }
  // replay checks: the failing simulations found by every workgroup (bit i)
  __device__ unsigned long long* failm() const { return reinterpret_cast<unsigned long long*>(base + 256); }
  // 1 once the game's workgroup runs (zeroed by the host before the launch):
  // tail helpers join only started games -- one not yet dispatched may be
  // waiting for the very CU a helper holds
  __device__ unsigned* started() const { return reinterpret_cast<unsigned*>(base + 384); }
  // tail helpers registered with this game (9x9 whole-game launches, tail_help)
  __device__ unsigned* nhelp() const { return reinterpret_cast<unsigned*>(base + 448); }
  // the actions, tagged: batch number << 32 | action (an entry is valid for
  // the batch whose number it carries: no separate progress counter)
  __device__ unsigned long long* acts() const { return reinterpret_cast<unsigned long long*>(base + 512); }
  __device__ double* bv(int A) const { return reinterpret_cast<double*>(base + 512 + (A * 8 + 255) / 256 * 256); }
  // the root's valid mask (child_priors reads it)
  __device__ uint8_t* valid(int A) const {
    return base + 512 + 2 * ((A * 8 + 255) / 256 * 256);
  }
  // representation conv3: the head sums per cell [3][CS] of every strip
  __device__ float* hfin(int A) const {
    return reinterpret_cast<float*>(base + 512 + 2 * ((A * 8 + 255) / 256 * 256) + (A + 255) / 256 * 256);
  }
};
template <class G>
__device__ __forceinline__ JobView job_of(const EngineArrays& E, int g) {
  return JobView{E.jobs + (size_t)g * job_bytes(G::A)};
}

// the parent convs and batch expansions go through jobs: 19x19 (Y streamed
// from L2, strip convs) with helper workgroups in the launch
template <class G>
__device__ __forceinline__ bool shared_jobs(const SearchParams& sp) {
  if constexpr (Smem<G>::GLOBAL_Y && G::WINO) return Wino<G>::NSTRIP > 1 && sp.helpers > 0;
  else return false;
}

// A job's batch number (unique within a launch: the host zeroes the jobs
// before it) with the claim word and the done counter reset for it.  Thread 0.
//
// The claim word is batch << 32 | total << 16 | next: a claim is decided by
// the word alone, never by the job's info block.  A helper that acquired
// batch s can read info rows the game's workgroup is already rewriting for
// s + 1 (the game claims every unit of s itself when no helper comes, waits
// for them and begins s + 1 at once); its CAS on the word of s then fails
// whatever total that info says, because s's word is exhausted (next >=
// total) before the game can begin s + 1, and the new word carries s + 1.
// A successful claim of s therefore means s is still open, so every info
// row the helper read belongs to s, and no stale done add can reach s + 1.
__device__ __forceinline__ unsigned job_begin(const JobView& J, int total, unsigned first = 0) {
  const unsigned bseq = __hip_atomic_load(J.seq(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  if (tid_local() == 0) {
    __hip_atomic_store(J.done(), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(J.claim(), (unsigned long long)bseq << 32 | (unsigned)total << 16 | first, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  return bseq;
}
// every store of the workgroup drained, then (release) the batch number.  All threads.
__device__ __forceinline__ void job_publish(const JobView& J, unsigned bseq) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid_local() == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (ROCm 7.2 may drop the fence's own wait)
    __hip_atomic_store(J.seq(), bseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// this workgroup's `mine` units added; wait until all `total` are done
// (every helper adds after its release), then acquire.  All threads.
__device__ __forceinline__ void job_wait(const JobView& J, int mine, int total) {
  if (tid_local() == 0) {
    unsigned d = __hip_atomic_fetch_add(J.done(), (unsigned)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + mine;
    while (d < (unsigned)total) {
      __builtin_amdgcn_s_sleep(kJobWaitSleep);
      d = __hip_atomic_load(J.done(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}
// claim the next unit of batch bseq (of total): -1 when none is left.  Thread 0
// claims, the workgroup gets it through LDS.  All threads.
template <class G>
__device__ __forceinline__ int job_claim(Smem<G>& sm, const JobView& J, unsigned bseq, int total, int step) {
  if (tid_local() == 0) {
    int c0 = -1;
    unsigned long long c = __hip_atomic_load(J.claim(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {                                       // (a failed CAS means another claim succeeded)
      // (the word's own total decides: see job_begin; `total` is the caller's copy)
      if ((unsigned)(c >> 32) != bseq || (int)(c & 0xFFFFu) >= (int)((c >> 16) & 0xFFFFu)) break;
      if (__hip_atomic_compare_exchange_strong(J.claim(), &c, c + step, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        c0 = (int)(c & 0xFFFFu);
        break;
      }
    }
    sm.bc[1] = c0;
  }
  __syncthreads();
  const int c0 = sm.bc[1];
  __syncthreads();                                   // (bc[1] is rewritten by the next claim)
  return c0;
}

// The dynamics conv of a parent as a job (19x19: 5 row strips, each strip
// independent given the input): its input -- src ([C][CS], the root's
// latent) or, with ypar, the latent rebuilt from the parent's Y and E[a]
// (wino_input_rebuilt: no materialized copy) -- -> dst (its Y, [CELLS][C]);
// strips claimed one at a time.  Returns this workgroup's strips.  All threads.
template <class G>
__device__ __forceinline__ int conv_strips(Smem<G>& sm, const NetParams& np, const JobView& J, unsigned bseq,
                                           const float* src, float* dst, const float* ypar = nullptr,
                                           const float* ea = nullptr) {
  int mine = 0;
  if constexpr (G::WINO) {
    for (int s; (s = job_claim(sm, J, bseq, Wino<G>::NSTRIP, 1)) >= 0; ++mine) {
      if (ypar) {
        // (the second channel slab transformed under the GEMM's first K half)
        wino_conv_rebuilt<G>(sm.u.v, sm.raw, sm.u.x.red, sm.u.x.hp, sm.u.x.outs, sm.hfin, ypar, ea, np.w_dyn,
                             np.b_dyn, dst, nullptr, nullptr, nullptr, s);
      } else {
        wino_input<G, G::C>(sm.u.v, sm.raw, src, G::CS, nullptr, s);
        wino_conv<G, G::C, G::C, 0, true>(sm.u.v, sm.u.x.red, sm.u.x.hp, sm.u.x.outs, sm.hfin, np.w_dyn, np.b_dyn,
                                           dst, G::CS, G::CS, nullptr, s);
      }
    }
  }
  __syncthreads();
  return mine;
}

// The game's workgroup: the conv of node `leaf` over the job machinery
// (dst = its pool slot).  Input: src (HBM, par < 0) or the latent rebuilt
// from parent par's Y and action act's E rows.  All threads; returns
// synchronised with dst complete and acquired.
// pre(bseq): work of the game's workgroup between the publish and its
// first strip claim (the next batch's picks: pick_all, wave 0), while the
// helpers start on the strips.
struct NoPre {
  __device__ void operator()(unsigned) const {}
};
template <class G, class Pre = NoPre>
__device__ __forceinline__ void conv_shared(Smem<G>& sm, const NetParams& np, const EngineArrays& E, int g,
                                            int leaf, int net, const float* src, float* dst,
                                            Stamp* st = nullptr, int par = -1, int act = 0, Pre pre = Pre{}) {
  const JobView J = job_of<G>(E, g);
  const unsigned bseq = job_begin(J, Wino<G>::NSTRIP);
  if (tid_local() == 0) {
    int* info = J.info();
    info[0] = Wino<G>::NSTRIP; info[1] = par; info[2] = leaf; info[3] = net; info[4] = par >= 0 ? 2 : 1;
    info[5] = act;
  }
  job_publish(J, bseq);                              // (src / the parent's Y reach the helpers)
  pre(bseq);
  if (st) st->lap(52);
  const float* ypar = par >= 0 ? pool_of<G>(E, g) + (size_t)par * G::C * G::CS : nullptr;
  const int mine = conv_strips<G>(sm, np, J, bseq, src, dst, ypar, np.etab + (size_t)act * 9 * G::C);
  if (st) st->lap(53);
  job_wait(J, mine, Wino<G>::NSTRIP);
  if (st) st->lap(54);
}

// ---------------------------------------------------------------------------
// The epoch tail at 9x9 (one-strip Winograd boards, the tree in LDS): in a
// whole-game launch the games end at different moves, and the last ones
// finish alone on their CUs (~29 % of an epoch's CU-time idle).  A workgroup
// whose game has ended registers (JobView::nhelp) with a running game that
// has fewer than kTailHelpers helpers and serves its parent convs: a game
// that sees a helper registered publishes its next parent conv as a job of
// kTailUnits units -- unit u = cout tiles 2u, 2u + 1 (wino_conv's m0 / nm) --
// claims units itself too (it never waits for a helper to start), waits for
// all, and loads the whole Y from L2 into its LDS copy.  Every workgroup
// computes the full Winograd input (from the parent's Y in the pool; the
// second slab under its first unit's GEMM, wino_conv_rebuilt) once per job and
// each unit's tiles' GEMM + epilogue exactly as the whole conv does,
// so the records do not depend on who computed what (MZGO_TAIL_HELPERS=0 A/B).
// Hand-offs: the job machinery above (release / relaxed flag / acquire).
// ---------------------------------------------------------------------------
constexpr int kTailUnits = 3;           // (granularity measured)
constexpr unsigned kTailHelpers = 2;
constexpr int kTailTiles = 6 / kTailUnits;     // cout tiles per unit
constexpr int kJobTailConv = 6;        // JobView info[4] of a tail conv job

template <class G>
struct TailConvs {
  static constexpr bool value = [] {
    if constexpr (G::WINO) return Wino<G>::NSTRIP == 1 && !Smem<G>::GLOBAL_Y && G::C == 6 * 16;
    else return false;
  }();
};

// Units of tail conv job bseq of game E/g claimed by this workgroup: V from
// the parent's Y once, then each unit's two cout tiles (red in the raw planes,
// whose zero halo is restored afterwards); Y stores drained.  All threads.
template <class G>
__device__ __forceinline__ int tail_conv_units(Smem<G>& sm, const NetParams& np, const JobView& J, unsigned bseq,
                                               const float* ypar, const float* ea, float* dst,
                                               const float* ylds_par = nullptr) {
  int mine = 0;
  if constexpr (TailConvs<G>::value) {
    for (int u; (u = job_claim(sm, J, bseq, kTailUnits, 1)) >= 0; ++mine) {
      if (mine == 0)   // (the second slab transformed under the first unit's GEMM, by every wave)
        wino_conv_rebuilt<G>(sm.u.v, sm.raw, sm.raw, sm.u.x.hp, sm.u.x.outs, sm.hfin, ypar, ea, np.w_dyn, np.b_dyn,
                             dst, nullptr, nullptr, ylds_par, 0, kTailTiles * u, kTailTiles);
      else
        wino_conv<G, G::C, G::C, 0, true>(sm.u.v, sm.raw, sm.u.x.hp, sm.u.x.outs, sm.hfin, np.w_dyn, np.b_dyn, dst,
                                          G::CS, G::CS, nullptr, 0, nullptr, nullptr, kTailTiles * u, kTailTiles);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this workgroup's Y stores done
    __syncthreads();
    if (mine > 0) wino_raw_zero<G>(sm.raw);
  }
  return mine;
}

// The game's workgroup: the parent conv of node `leaf` (its latent rebuilt
// from parent par's Y and action act's E rows) as a tail job; returns with
// Y in the pool slot and, when ylds, in the expansion's LDS copy.  All threads.
template <class G>
__device__ __forceinline__ void conv_tail(Smem<G>& sm, const NetParams& np, const EngineArrays& E, int g, int leaf,
                                          int par, int act, int net, float* dst, float* ylds, bool par_in_lds,
                                          Stamp* st = nullptr) {
  if constexpr (TailConvs<G>::value) {
    const JobView J = job_of<G>(E, g);
    const unsigned bseq = job_begin(J, kTailUnits);
    if (tid_local() == 0) {
      int* info = J.info();
      info[0] = kTailUnits; info[1] = par; info[2] = leaf; info[3] = net; info[4] = kJobTailConv; info[5] = act;
    }
    job_publish(J, bseq);                            // (the parent's Y in the pool reaches the helpers)
    if (st) st->lap(52);
    const float* ypar = pool_of<G>(E, g) + (size_t)par * G::C * G::CS;
    const int mine = tail_conv_units<G>(sm, np, J, bseq, ypar, np.etab + (size_t)act * 9 * G::C, dst,
                                        par_in_lds ? ylds : nullptr);
    if (st) st->lap(53);
    job_wait(J, mine, kTailUnits);
    if (st) st->lap(54);
    if (tid_local() == 0) atomicAdd(&E.counters[4], 1ull);
    if (ylds) {
      const f32x4* src = reinterpret_cast<const f32x4*>(dst);
      f32x4* d = reinterpret_cast<f32x4*>(ylds);
      for (int i = tid_local(); i < G::CELLS * G::C / 4; i += G::THREADS) d[i] = src[i];
    }
    __syncthreads();
  }
}

// A workgroup whose game has ended: serve running games' tail conv jobs until
// none is left to register with.  All threads.
template <class G>
__device__ __forceinline__ void tail_help(Smem<G>& sm, const NetParams& np_a, const NetParams& np_b,
                                          const EngineArrays& E, int self, int games) {
  if constexpr (TailConvs<G>::value) {
    wino_raw_zero<G>(sm.raw);                          // (an ended slot's workgroup never zeroed its planes)
    for (;;) {
      // a running game (its seq not kJobExit) with fewer than kTailHelpers
      // helpers, the nearest after this one
      if (tid_local() == 0) {
        int pick = -1;
        for (int k = 1; k < games && pick < 0; ++k) {
          const int t = (self + k) % games;
          const JobView Jt = job_of<G>(E, t);
          if (__hip_atomic_load(Jt.started(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 ||
              __hip_atomic_load(Jt.seq(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kJobExit)
            continue;
          unsigned c = __hip_atomic_load(Jt.nhelp(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          while (c < kTailHelpers &&
                 !__hip_atomic_compare_exchange_strong(Jt.nhelp(), &c, c + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)) {
          }
          if (c < kTailHelpers) pick = t;
        }
        sm.bc[2] = pick;
      }
      __syncthreads();
      const int t = sm.bc[2];
      __syncthreads();
      if (t < 0) return;
      const JobView J = job_of<G>(E, t);
      float* pool = pool_of<G>(E, t);
      unsigned last = 0;
      for (;;) {
        if (tid_local() == 0) {
          unsigned s = __hip_atomic_load(J.seq(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          for (long long spins = 0; (s == last || s == 0) && spins < (1ll << 24); ++spins) {
            __builtin_amdgcn_s_sleep(kJobPollSleep);
            s = __hip_atomic_load(J.seq(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          int expired = 0;
          if (s == last || s == 0) {                   // (bounded wait: leave, and exit -- no re-registering)
            __hip_atomic_fetch_sub(J.nhelp(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            atomicAdd(&E.counters[7], 1ull);           // (counted: bench lines report expiries)
            s = kJobExit;
            expired = 1;
          }
          if (s != kJobExit) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          sm.bc[2] = (int)s;
          sm.bc[4] = expired;
        }
        __syncthreads();
        const unsigned s = (unsigned)sm.bc[2];
        const int expired = sm.bc[4];
        __syncthreads();
        if (expired) return;
        if (s == kJobExit) break;
        last = s;
        const int* info = J.info();
        const int par = info[1], leaf = info[2], net = info[3], kind = info[4], act = info[5];
        if (kind != kJobTailConv) continue;
        const NetParams np = select_params(net != 0, np_b, np_a);
#ifdef MZGO_STAMPS
        const unsigned long long tu = __builtin_amdgcn_s_memtime();
#endif
        const int mine = tail_conv_units<G>(sm, np, J, s, pool + (size_t)par * G::C * G::CS,
                                            np.etab + (size_t)act * 9 * G::C, pool + (size_t)leaf * G::C * G::CS);
#ifdef MZGO_STAMPS
        // slots 44-46: a helper's cycles computing tail units, units, jobs served
        if (tid_local() == 0 && E.stamps) {
          unsigned long long* sl = E.stamps + (size_t)blockIdx.x * kStampPhases;
          sl[44] += __builtin_amdgcn_s_memtime() - tu;
          sl[45] += (unsigned long long)mine;
          sl[46] += mine > 0 ? 1ull : 0ull;
        }
#endif
        if (tid_local() == 0 && mine > 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (ROCm 7.2 may drop the fence's own wait)
          __hip_atomic_fetch_add(J.done(), (unsigned)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
}

// The representation's conv2 (CIN 64 -> 64) and conv3 (64 -> C, value and
// policy head sums per cell into hfin) of a 19x19 root as strip jobs (kinds
// 4, 5): src -> dst, both [CIN][CS] / [COUT][CS] in HBM (factored search:
// the scratch slot and node 0's slot).  Returns this workgroup's strips.
template <class G, int CIN, int COUT, int NH>
__device__ __forceinline__ int rep_strips(Smem<G>& sm, const JobView& J, unsigned bseq, const float* w,
                                          const float* b, const float* src, float* dst, const float* head_w,
                                          float* hfin) {
  int mine = 0;
  if constexpr (G::WINO) {
    for (int s; (s = job_claim(sm, J, bseq, Wino<G>::NSTRIP, 1)) >= 0; ++mine) {
      wino_input<G, CIN>(sm.u.v, sm.raw, src, G::CS, nullptr, s);
      wino_conv<G, CIN, COUT, NH>(sm.u.v, sm.u.x.red, sm.u.x.hp, sm.u.x.outs, hfin, w, b, dst, G::CS, G::CS,
                                  head_w, s);
    }
  }
  __syncthreads();
  return mine;
}

// The game's workgroup: representation conv k (2 or 3) over the job
// machinery; conv3's head sums come back into sm.hfin.  All threads;
// returns synchronised.
template <class G>
__device__ __forceinline__ void rep_shared(Smem<G>& sm, const NetParams& np, const EngineArrays& E, int g, int net,
                                           int k) {
  if constexpr (G::WINO && Wino<G>::NSTRIP > 1) {
  const JobView J = job_of<G>(E, g);
  float* pool = pool_of<G>(E, g);
  float* lat = pool + (size_t)(E.S + 1) * G::C * G::CS;
  const unsigned bseq = job_begin(J, Wino<G>::NSTRIP);
  if (tid_local() == 0) {
    int* info = J.info();
    info[0] = Wino<G>::NSTRIP; info[1] = 0; info[2] = 0; info[3] = net; info[4] = k == 2 ? 4 : 5;
  }
  job_publish(J, bseq);                              // (conv k's input reaches the helpers)
  const int mine = k == 2 ? rep_strips<G, 64, 64, 0>(sm, J, bseq, np.w_conv2, np.b_conv2, lat, pool, nullptr, sm.hfin)
                          : rep_strips<G, 64, G::C, 2>(sm, J, bseq, np.w_conv3, np.b_conv3, pool, lat,
                                                       np.head_w + G::C, J.hfin(G::A));
  job_wait(J, mine, Wino<G>::NSTRIP);
  if (k == 3)
    for (int i = tid_local(); i < 2 * G::CS; i += G::THREADS) sm.hfin[i] = J.hfin(G::A)[i];
  __syncthreads();
  }
}

// One child of a batch by ONE wave (batch_expand's per-child work): E[a]
// into W.ew, expand_wave over Y, the heads, the child's prior row and child
// row; returns the backup value r + discount * v (every lane).  Lazy policy
// head: LAZY (LDS trees) writes neither row (TreeLds::rawp), LAZYH (HBM
// trees, the shared batches) only the sentinel kLazyRow into child-row entry
// 0; a select that first reaches the node forms its logits and priors (most
// never are).
template <class G, bool LAZY, bool LAZYH = false>
__device__ __forceinline__ double expand_child(Smem<G>& sm, const NetParams& np, const SearchParams& sp,
                                               const TreeView& TV, const float* yg, const ExpandPlan<G>& plan,
                                               int a, int nid, Stamp* st = nullptr) {
  // (st: wave 0's phase cycles in slots 64-66, 68)
  unsigned long long t0 = st ? st->now() : 0, t1;
  auto& L = sm.u.f;
  typedef decltype(sm.u.f) XL;
  const int lane = lane_id_local();
  auto& W = L.wv[__builtin_amdgcn_readfirstlane(wave_id())];
  constexpr int E4N = 9 * G::C / 4;
  f32x4* ewl = reinterpret_cast<f32x4*>(W.ew);
  const f32x4* e4 = reinterpret_cast<const f32x4*>(np.etab + (size_t)a * 9 * G::C);
  for (int i = lane; i < E4N; i += 64) ewl[i] = e4[i];
  wave_lds_sync();
  if (st && wave_id() == 0) { t1 = st->now(); st->wave_add(64, t1 - t0); t0 = t1; }
  float rsum, vsum;
  constexpr bool POL = !LAZY && !LAZYH;
  if constexpr (XL::GLOBAL_Y) expand_wave<G, XL::PROW, POL>(W.xw, yg, W.ew, L.hw, plan, rsum, vsum);
  else expand_wave<G, XL::PROW, POL>(W.xw, L.yc, W.ew, L.hw, plan, rsum, vsum);
  wave_lds_sync();
  if (st && wave_id() == 0) { t1 = st->now(); st->wave_add(65, t1 - t0); t0 = t1; }
  float r, v;
  heads_from_totals<G>(rsum, vsum, sm.t.hsc, r, v);
  if (st && wave_id() == 0) { t1 = st->now(); st->wave_add(66, t1 - t0); t0 = t1; }
  if constexpr (LAZY) {
    if (lane == 0) atomicOr(&sm.t.rawp[nid >> 5], 1u << (nid & 31));
  } else if constexpr (LAZYH) {
    if (lane == 0) TV.child[(size_t)nid * G::A] = kLazyRow;
  } else {
    float x[G::AP];
    policy_logits<G>(W.xw + XL::PROW, sm.t.hsc, x);
    int* crow = TV.child + (size_t)nid * G::A;
    for (int i = lane; i < G::A; i += 64) crow[i] = -1;
    child_priors<G>(sm.t, x, TV.prior + (size_t)nid * G::A, -1, sp.variant, W.fscratch(), W.dscratch());
  }
  wave_lds_sync();                     // W.ew / W.xw reused by the wave's next child
  if (st && wave_id() == 0) { st->wave_add(68, st->now() - t0); }
  return (double)r + sp.discount * (double)v;
}

// The children of job J (batch bseq, B children, node ids nid0 + k, actions
// in L.acts) a round of WAVES at a time, claimed by CAS; each child's backup
// value goes to J.bv (HBM).  Returns this workgroup's count.  All threads.
template <class G, bool LAZY, bool LAZYH = false>
__device__ __forceinline__ int job_rounds(Smem<G>& sm, const NetParams& np, const SearchParams& sp,
                                          const TreeView& TV, const float* yg, const JobView& J, unsigned bseq,
                                          int B, int nid0, bool helper = false, Stamp* st = nullptr) {
  auto& L = sm.u.f;
  const int wave = __builtin_amdgcn_readfirstlane(wave_id());
  ExpandPlan<G> plan;
  plan.init(L.rpair);
  double* bvg = J.bv(G::A);
  int mine = 0;
  for (;;) {
    const int c0 = job_claim(sm, J, bseq, B, G::WAVES);
    if (c0 < 0) break;
    const int k = c0 + wave;
    if (k < B) {
      int a;
      if (helper) {                                  // (a helper may claim before the game's wave 0 picked it)
        unsigned long long t = __hip_atomic_load(J.acts() + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while ((unsigned)(t >> 32) != bseq) {
          __builtin_amdgcn_s_sleep(2);
          t = __hip_atomic_load(J.acts() + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        a = __builtin_amdgcn_readfirstlane((int)(unsigned)t);
      } else {
        a = __builtin_amdgcn_readfirstlane(L.acts[k]);
      }
      const double bv = expand_child<G, LAZY, LAZYH>(sm, np, sp, TV, yg, plan, a, nid0 + k, st);
      if (lane_id_local() == 0) bvg[k] = bv;
    }
    mine += (B - c0 < G::WAVES ? B - c0 : G::WAVES);
  }
  return mine;
}

// The game's workgroup: batch_expand over the job machinery (B children of
// leaf `leaf` whose Y is yg, actions in L.acts, node ids nid0 + k); L.bv
// gets every child's backup value.
struct NoWait {
  __device__ void operator()() const {}
};
template <class G, bool LAZY, class Wait = NoWait>
__device__ __forceinline__ void batch_expand_shared(Smem<G>& sm, const NetParams& np, const SearchParams& sp,
                                                    const EngineArrays& E, int g, const TreeView& TV, int B,
                                                    int nid0, int leaf, int net, const float* yg,
                                                    const uint64_t (&m)[G::AP], int n, int i0, uint64_t key,
                                                    int sim0, Stamp* st = nullptr, bool prepicked = false,
                                                    Wait pre_wait = Wait{}) {
  auto& L = sm.u.f;
  const JobView J = job_of<G>(E, g);
  const unsigned bseq = job_begin(J, B);
  // the job first (geometry, the root's mask, the actions known already:
  // i0 of them), then the picks (pick_all, wave 0; tagged entries: a helper
  // that claims a round before they are out waits for its entry)
  for (int a = tid_local(); a < G::A; a += G::THREADS) J.valid(G::A)[a] = sm.t.valid[a];
  if (tid_local() == 0) {
    int* info = J.info();
    info[0] = B; info[1] = nid0; info[2] = leaf; info[3] = net; info[4] = 0;
    *J.pass_prior() = sm.t.pass_prior;
    for (int k = 0; k < i0; ++k)
      __hip_atomic_store(J.acts() + k, (unsigned long long)bseq << 32 | (unsigned)L.acts[k], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  job_publish(J, bseq);
  if (st) st->lap(40);
  // (prepicked: the actions i0.. went out during the parent's conv job,
  // tagged for this batch; the workgroup reads them from the job like a
  // helper and copies them back into L.acts, which the conv overwrote)
  if (!prepicked && wave_id() == 0)
    pick_all<G>(m, n, i0, B - i0, key, sim0, L.acts, st, J.acts(), bseq);
  __syncthreads();                                   // every pick made (in LDS too)
  if (st) st->lap(41);
  const int mine = job_rounds<G, LAZY, !LAZY>(sm, np, sp, TV, yg, J, bseq, B, nid0, prepicked, st);
  if (st) st->lap(42);
  if (prepicked)
    for (int k = tid_local(); k < B; k += G::THREADS)
      L.acts[k] = (int)(unsigned)__hip_atomic_load(J.acts() + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  pre_wait();                                        // (the replay checks' first level rows, verify_preload)
  job_wait(J, mine, B);
  const double* bvg = J.bv(G::A);
  for (int k = tid_local(); k < B; k += G::THREADS) L.bv[k] = bvg[k];
  __syncthreads();
  if (st) st->lap(43);
}

// dst[0] = w0, dst[k + 1] = dst[k] + (neg ? -v[k] : v[k]) for k < B: the
// sequential f64 sums (lane 0), 8 at a time without branches, the next 8
// loads in flight: v is read up to 15 and dst written up to 7 entries past B
// (those sums are never read).  Wave-level.
template <class G>
__device__ __forceinline__ double prefix_sums(double w0, const double* __restrict__ v, int B, bool neg,
                                              double* __restrict__ dst) {
  double w = w0;
  if (lane_id_local() == 0) {
    if (dst) dst[0] = w;
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = v[u];
    for (int k0 = 0; k0 < B; k0 += 8) {
      double y[8];                                 // the next chunk's loads, in flight during the chain
#pragma unroll
      for (int u = 0; u < 8; ++u) y[u] = v[k0 + 8 + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        if (k0 + u < B) w = w + (neg ? -x[u] : x[u]);
        if (dst) dst[k0 + u + 1] = w;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = y[u];
    }
  }
  return w;                                        // lane 0: the sum over all B
}

// Batched root phase.  While the root has unexpanded eligible children,
// select_leaf (self_play.py:283-287; main.py's select the same) picks one of
// them by the simulation's draw alone -- no value enters the choice -- so the
// first K = min(S, #eligible root children) simulations expand K distinct
// root children in an order fixed before any of them is evaluated.  They run
// as one batch: the root's conv once, batch_expand, then the K backups in
// simulation order, so every sum is the sequential one and the tree is the
// same node for node.  Returns K (0: no batch).
template <class G, class Acc>
__device__ __forceinline__ int root_batch(Smem<G>& sm, const NetParams& np, const SearchParams& sp,
                                          const EngineArrays& E, int g, const TreeView& TV, Acc& T, float* pool,
                                          float* scratch, int* nact, uint64_t key, Stamp* st = nullptr) {
  auto& L = sm.u.f;
  if constexpr (!decltype(sm.u.f)::BATCH) {
    return 0;
  } else {
    const int S = sp.num_simulations;
    // eligible root children (prior > 0, as select_leaf decides)
    if (wave_id() == 0) {
      int n = 0;
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane_id_local() + 64 * j;
        n += __popcll(__ballot(a < G::A && T.root_prior(a) > 0.0));
      }
      if (lane_id_local() == 0) sm.t.bcast = n < S ? n : S;
    }
    __syncthreads();
    const int K = sm.t.bcast;
    if (K == 0) return 0;
    // the simulations' choices: sim k takes the r_k-th (ascending) of the
    // n - k eligible root children not taken yet, r_k = randbelow(draw_k, n - k)
    uint64_t el[G::AP];
    int n = 0;
    if (wave_id() == 0) {
      const int lane = lane_id_local();
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane + 64 * j;
        el[j] = __ballot(a < G::A && T.root_prior(a) > 0.0);
        n += __popcll(el[j]);
      }
    }
    // the root's conv Y (its latent is in the scratch slot), then Y and the
    // head weights into LDS.  The conv overwrites the whole union, so the
    // batch's LDS buffers are filled only after it.  (Shared jobs: the picks
    // go out while the helpers run the conv's strips.)
    if (shared_jobs<G>(sp)) {
      conv_shared<G>(sm, np, E, g, 0, sp.net, scratch, pool, st, -1, 0, [&](unsigned cb) {
        if (wave_id() == 0) pick_all<G>(el, n, 0, K, key, 0, L.acts, st, job_of<G>(E, g).acts(), cb + 1);
      });
    } else {
      latent_conv<G, G::C, G::C, 0, true>(sm, np.w_dyn, np.b_dyn, scratch, G::CS, nullptr, pool, G::CS, G::CS,
                                          nullptr, nullptr, y_lds_target<G>(sm));
    }
    __syncthreads();
    if (st) st->lap(60);
    if (y_lds_target<G>(sm) != nullptr && !shared_jobs<G>(sp)) load_hw<G>(sm, np.head_w);   // (Y in L.yc already)
    else load_y<G>(sm, pool, np.head_w);
    if (tid_local() == 0) { sm.t.npick = 0; sm.t.ngrab = 0; }
    __syncthreads();
    if (st) st->lap(61);
    if (shared_jobs<G>(sp)) {
      batch_expand_shared<G, Acc::LDS>(sm, np, sp, E, g, TV, K, 1, 0, sp.net, pool, el, n, 0, key, 0, nullptr, true);
    } else {
      if (wave_id() == 0) pick_sequence<G>(el, n, 0, K, key, 0, L.acts, &sm.t.npick, G::WAVES);
      batch_expand<G, Acc::LDS>(sm, np, sp, TV, K, 1, pool, st);
    }
    __syncthreads();
    if (st) st->lap(62);
    if (wave_id() == 0) {
      const int lane = lane_id_local();
      // the K backups of backpropagate(path + [child], v) (self_play.py:337-343)
      for (int k = lane; k < K; k += 64) {
        const int a = L.acts[k], nid = 1 + k;
        const double v = L.bv[k];
        T.init(nid);
        T.add(nid, v);
        T.set_child(0, a, nid);
        T.add_root_child(a, v);
        nact[nid] = a;
      }
      if (lane == 0) {
        const bool alt = sp.variant == 0;   // main.py:366-368 does not alternate
        // the root's sum in simulation order: the same f64 additions, the
        // running sum in a register (prefix_sums' chain) instead of LDS
        const double wroot = prefix_sums<G>(T.ws(0), L.bv, K, alt, nullptr);
        T.set(0, T.vis(0) + K, wroot);
        sm.t.newest = -1;                    // every prior row is in HBM already
        sm.t.ycache = 0;                     // L.yc holds the root's Y
      }
    }
    __syncthreads();
    return K;
  }
}

// Parallel replay of a speculative batch (factored dynamics, LDS trees).
//
// The batch's B children of `leaf` (depth D, path p_0 = root .. p_D = leaf)
// stand for simulations sim .. sim + B - 1; simulation sim + i (i >= 1)
// reaches the leaf again iff, at every level l < D, p_l's PUCT still picks
// the path child x_l = p_(l+1) after the i earlier simulations were backed
// up (it then takes acts[i] at the leaf: its draw, by construction).  Those
// i backups are known in advance (their values are the batch's), so every
// check (i, l) is independent: the state it sees is p_l's children as they
// are now, except x_l with n_x + i visits and value sum W_x(i) (the prefix
// sum, in simulation order, of its shares), and p_l with N + i visits.  All
// (i, l) checks run at once over the workgroup with puct_pick's operations
// and first-maximum rule; the batch is accepted up to the first failing i,
// and the tree takes the accepted simulations' sums.  Returns the number of
// accepted simulations m >= 1 (all threads; synchronised).
template <class G, int DMAX>
struct VerifyLds {
  double cP[DMAX][64 * G::AP];      // c_puct * P as puct_pick forms it
  double q[DMAX][64 * G::AP];       // W / N of every child, now
  double inv1n[DMAX][64 * G::AP];   // 1 / (1 + N) of every child, now (the screening pass)
  int n[DMAX][64 * G::AP];
  // per (level, i): x's q after i accepted simulations, 1 / (hi - lo) of the
  // level's q range then (0: no spread), the sqrt term, and x's exact score
  double qx[DMAX][G::A + 1], invr[DMAX][G::A + 1], sq[DMAX][G::A + 1], sx[DMAX][G::A + 1];
  uint64_t elig[DMAX][G::AP];
  double lo_o[DMAX], hi_o[DMAX];    // min / max of q over eligible children other than x
  double cpx[DMAX];                 // x's c_puct * P
  int x[DMAX], n0[DMAX], N0[DMAX];
  double wpre[DMAX][G::A + 9];      // x_l's value sum after i accepted simulations (+ prefix_sums' tail)
  double wroot[G::A + 9];           // the root's value sum after i
  uint64_t failm[G::AP];            // simulations i whose walk leaves the batch (bit i)
  uint64_t exactm[DMAX][G::AP];     // (level, i) checks the screening left open
  int fail;
};
// levels verify_batch holds at once (its arrays are per level; a deeper path
// is checked in groups of this many levels): 8 at 9x9 and below, 2 at 19x19
template <class G>
constexpr int verify_depth() { return G::AP > 2 ? 2 : 8; }
// A speculative batch of B children of a leaf at depth D is replayed one
// select at a time (B - 1 walks of D + 1 levels) while (B - 1) * (D + 1) <
// kSeqK, else by the parallel replay (verify_batch; the trees are the same
// either way).  Measured, 9x9 / 256 / 200 epoch, same call: K = 8 / 12 / 16 /
// 24: 77.1 / 78.1 / 79.0 / 77.8 M sims/s (a minimum-B rule at its best, 6:
// 77.0-77.2); HBM trees with helper workgroups (shared jobs, 19x19): K = 0 /
// 8 / 16 / 32 / 64: 37.8 / 37.8 / 38.0 / 38.3 / 37.7 M
// (profiles/r4x_shared_seq_ab.txt)
constexpr int kSeqK = 16, kSharedSeqK = 32;
__device__ __forceinline__ bool replay_sequential(int B, int depth) { return (B - 1) * (depth + 1) < kSeqK; }
__device__ __forceinline__ bool replay_parallel(bool shared, int B, int depth) {
  if (shared) return (B - 1) * (depth + 1) >= kSharedSeqK;
  return !replay_sequential(B, depth);
}

// Phase 1a of verify_batch for one path level l (row k of vl): its
// children's c_puct * P, q, 1 / (1 + n), n and eligibility, the min / max of
// q over the eligible children other than x_l, and x_l's terms.  Reads the
// tree only (not the batch's values), so it may run before the batch is
// done.  Wave-level.
template <class G, class Acc, class V>
__device__ __forceinline__ void verify_load_level(Smem<G>& sm, const SearchParams& sp, const TreeView& TV,
                                                  const Acc& T, const int* nact, V& vl, int k, int l, int ract) {
  const int lane = lane_id_local();
  const int p = T.path(l);
  const int xa = l == 0 ? ract : nact[T.path(l + 1)];
  double lo = INFINITY, hi = -INFINITY, cpx = 0.0;
  int nx = 0;
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    const bool in = a < G::A;
    double P, w = 0.0;
    int n = 0;
    if (l == 0) {
      P = in ? T.root_prior(a) : 0.0;
      if constexpr (Acc::LDS) {
        if (in) { n = sm.t.rvis[a]; w = sm.t.rws[a]; }     // the root-child mirror
      } else {
        const int c = in ? T.child(0, a) : -1;
        if (c >= 0) { n = T.vis(c); w = T.ws(c); }
      }
    } else {
      P = in ? (double)TV.prior[(size_t)p * G::A + a] : 0.0;
      const int c = in ? TV.child[(size_t)p * G::A + a] : -1;
      if (c >= 0) { n = T.vis(c); w = T.ws(c); }
    }
    const bool e = P > 0.0;
    const uint64_t el = __ballot(e);
    const double q = e ? (n > 0 ? ddiv(w, (double)n) : 0.0) : 0.0;
    const double cp = l == 0 ? sp.c_puct * P : (double)((float)sp.c_puct * (float)P);
    vl.cP[k][a] = cp;
    vl.q[k][a] = q;
    vl.inv1n[k][a] = 1.0 / (double)(1 + n);
    vl.n[k][a] = n;
    if (lane == 0) vl.elig[k][j] = el;
    if (e && a != xa) { lo = fmin_(lo, q); hi = fmax_(hi, q); }
    if (j == (xa >> 6)) {
      nx = __builtin_amdgcn_readlane(n, xa & 63);
      cpx = dpp::lane(cp, xa & 63);
    }
  }
  wave_minmax(lo, hi);
  if (lane == 0) {
    vl.lo_o[k] = lo;
    vl.hi_o[k] = hi;
    vl.x[k] = xa;
    vl.n0[k] = nx;
    vl.N0[k] = T.vis(p);
    vl.cpx[k] = cpx;
  }
}

// verify_batch's checks of path levels l0 .. l0 + nl - 1 (nl <= DV): phases
// 1a-2 and the exact fallback; failing simulations are OR-ed into vl.failm
// (the caller zeroes it once).  with_root: also the root's value sums
// (vl.wroot) on a spare wave.  ract: the root action on the path.  loaded:
// the levels' rows are in vl already (verify_preload).  All threads;
// returns synchronised.
template <class G, class Acc>
__device__ __forceinline__ void verify_levels(Smem<G>& sm, const SearchParams& sp, const TreeView& TV, const Acc& T,
                                              const int* nact, int D, int B, int l0, int nl, int ract,
                                              bool with_root, Stamp* st = nullptr, bool loaded = false) {
  constexpr int DV = verify_depth<G>();
  typedef VerifyLds<G, DV> V;
  V& vl = *reinterpret_cast<V*>(&sm.u.f.wv[0]);
  const int wave = __builtin_amdgcn_readfirstlane(wave_id());
  const int lane = lane_id_local();
  const bool alt = sp.variant == 0;
  const double* bv = sm.u.f.bv;
  if (tid_local() < DV * G::AP) (&vl.exactm[0][0])[tid_local()] = 0;
  // ---- 1a. jobs 0..nl-1: level l0 + k's children (one wave each); jobs
  // nl..2nl-1: x's sequential value sums for those levels, and in the first
  // group job 2nl: the root's, on other waves at the same time ----
  const int njobs = 2 * nl + (with_root ? 1 : 0);
  for (int job = wave; job < njobs; job += G::WAVES) {
    if (job == 2 * nl) {                          // the root's value sum after i simulations
      prefix_sums<G>(T.ws(0), bv, B, alt && ((D + 1) & 1), vl.wroot);
      continue;
    }
    if (job >= nl) {                              // x_l = p_(l+1), depth l + 1
      const int k = job - nl, l = l0 + k;
      prefix_sums<G>(T.ws(T.path(l + 1)), bv, B, alt && ((D - l) & 1), vl.wpre[k]);
      continue;
    }
    if (!loaded) verify_load_level<G, Acc>(sm, sp, TV, T, nact, vl, job, l0 + job, ract);
    if (st) st->lap(75);
  }
  __syncthreads();
  if (st) st->lap(76);
  // ---- 1b. per level, per simulation i (lane i = lane + 64 j): the level
  // as simulation i's select finds it, and x's score exactly as puct_pick
  // forms it; a score that is not finite fails i ----
  for (int k = wave; k < nl; k += G::WAVES) {
    const int nx = vl.n0[k], N0 = vl.N0[k];
    const double lo = vl.lo_o[k], hi = vl.hi_o[k], cpx = vl.cpx[k];
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const int i = lane + 64 * j;
      bool bad = false;
      if (i <= B) {
        const int n1 = nx + i, Ni = N0 + i;
        const double qxi = n1 > 0 ? ddiv(vl.wpre[k][i], (double)n1) : 0.0;
        const double loi = fmin_(lo, qxi), hii = fmax_(hi, qxi);
        const double sqi = dsqrt((double)(sp.variant == 1 ? Ni + 1 : (Ni > 1 ? Ni : 1)));
        const double sxi = (hii > loi ? ddiv(qxi - loi, hii - loi) : qxi) + ddiv(cpx * sqi, (double)(1 + n1));
        vl.qx[k][i] = qxi;
        vl.invr[k][i] = hii > loi ? 1.0 / (hii - loi) : 0.0;
        vl.sq[k][i] = sqi;
        vl.sx[k][i] = sxi;
        bad = i >= 1 && i < B && !(sxi > -INFINITY);
      }
      const uint64_t bb = __ballot(bad);
      if (lane == 0 && bb) atomicOr(reinterpret_cast<unsigned long long*>(&vl.failm[j]), (unsigned long long)bb);
    }
    if (st) st->lap(77);
  }
  __syncthreads();
  if (st) st->lap(72);
  // ---- 2. every (i, l) check at once, transposed: lanes are simulations
  // i = lane + 64 j, each wave takes every WAVES-th child a of each level.
  // Screening: the two divisions of a's score as products with reciprocals
  // (a few ulp off); a decides (l, i) only if its score is clear of x's by
  // far more than that, else (l, i) is redone below with puct_pick's exact
  // operations.  i fails if any eligible a != x beats x (puct_pick's first
  // maximum: a higher score, or an equal one at a lower action). ----
  const unsigned long long ts0 = st ? st->now() : 0;
  for (int k = 0; k < nl; ++k) {
    const int xa = vl.x[k];
    const double lo_o = vl.lo_o[k], hi_o = vl.hi_o[k];
    double loi[G::AP], invr[G::AP], sqi[G::AP], sxi[G::AP], tol[G::AP];
    bool spread[G::AP];
    uint64_t beaten[G::AP], close[G::AP];
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const int i = lane + 64 * j;
      const int ii = i <= B ? i : B;
      const double qxi = vl.qx[k][ii];
      loi[j] = fmin_(lo_o, qxi);
      spread[j] = fmax_(hi_o, qxi) > loi[j];
      invr[j] = vl.invr[k][ii];
      sqi[j] = vl.sq[k][ii];
      sxi[j] = vl.sx[k][ii];
      tol[j] = 1e-12 * (1.0 + fabs(sxi[j]));
      beaten[j] = 0;
      close[j] = 0;
    }
    // the wave's children a = wave + WAVES k, one per lane k, loaded in one
    // round trip; the loop broadcasts them with readlane
    constexpr int KW = (G::A + G::WAVES - 1) / G::WAVES;
    static_assert(KW <= 64, "one lane per child of the wave");
    const int amine = wave + G::WAVES * lane;
    const bool mine = lane < KW && amine < G::A && amine != xa &&
                      ((vl.elig[k][(amine < G::A ? amine : 0) >> 6] >> (amine & 63)) & 1ull);
    const int ac = mine ? amine : 0;
    const double qa_l = vl.q[k][ac], cpa_l = vl.cP[k][ac], ia_l = vl.inv1n[k][ac];
    const uint64_t todo = __ballot(mine);
    for (uint64_t mm = todo; mm; mm &= mm - 1) {
      const int kk = __builtin_ctzll(mm);
      const double qa = dpp::lane(qa_l, kk), cpa = dpp::lane(cpa_l, kk), ia = dpp::lane(ia_l, kk);
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        if (64 * j >= B) break;                     // (uniform) no simulation i in this register
        const double sc = (spread[j] ? (qa - loi[j]) * invr[j] : qa) + (cpa * sqi[j]) * ia;
        beaten[j] |= __ballot(sc > sxi[j] + tol[j]);
        close[j] |= __ballot(!(fabs(sc - sxi[j]) > tol[j]));
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        if (beaten[j]) atomicOr(reinterpret_cast<unsigned long long*>(&vl.failm[j]), (unsigned long long)beaten[j]);
        if (close[j] & ~beaten[j])
          atomicOr(reinterpret_cast<unsigned long long*>(&vl.exactm[k][j]), (unsigned long long)(close[j] & ~beaten[j]));
      }
    }
  }
  if (st) st->wave_add(80, st->now() - ts0);
  __syncthreads();
  if (st) st->lap(78);
  // the open (l, i) checks with puct_pick's exact operations (rare)
  for (int k = 0; k < nl; ++k) {
    uint64_t open[G::AP];
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const uint64_t o = vl.exactm[k][j] & ~vl.failm[j];
      open[j] = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(o >> 32)) << 32) |
                __builtin_amdgcn_readfirstlane((uint32_t)o);
    }
    int c = 0;
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      for (uint64_t mm = open[j]; mm; mm &= mm - 1, ++c) {
        if (c % G::WAVES != wave) continue;
        const int i = 64 * j + __builtin_ctzll(mm);
        if (i < 1 || i >= B) continue;
        const int xa = vl.x[k];
        const int nx = vl.n0[k] + i;
        const double qx = vl.qx[k][i];
        const double lo = fmin_(vl.lo_o[k], qx), hi = fmax_(vl.hi_o[k], qx);
        const double sq = vl.sq[k][i], sx = vl.sx[k][i];
        uint64_t beat = 0;
#pragma unroll
        for (int jj = 0; jj < G::AP; ++jj) {
          const int a = lane + 64 * jj;
          const bool el = (vl.elig[k][jj] >> lane) & 1ull;
          const bool isx = a == xa;
          const double q = isx ? qx : vl.q[k][a];
          const int n = isx ? nx : vl.n[k][a];
          const double qn = hi > lo ? ddiv(q - lo, hi - lo) : q;
          const double sc = qn + ddiv(vl.cP[k][a] * sq, (double)(1 + n));
          beat |= __ballot(el && !isx && (sc > sx || (sc == sx && a < xa)));
        }
        if (beat && lane == 0)
          atomicOr(reinterpret_cast<unsigned long long*>(&vl.failm[i >> 6]), 1ull << (i & 63));
      }
    }
  }
  __syncthreads();
  if (st) st->lap(79);
}

// How verify_batch splits a depth-D path: groups of gs levels; shared: the
// groups are a job (HBM trees with helper workgroups): one level per group
// while the groups do not outnumber the 4 workgroups, else DV; otherwise
// the game's workgroup checks groups of DV itself.  g0: group 0's levels.
struct VerifyPlan {
  int gs, ngroups, g0;
  bool shared;
};
template <class G, class Acc>
__device__ __forceinline__ VerifyPlan verify_plan(const SearchParams& sp, int D) {
  constexpr int DV = verify_depth<G>();
  VerifyPlan v;
  v.gs = D <= 4 ? 1 : DV;
  v.ngroups = (D + v.gs - 1) / v.gs;
  v.shared = !Acc::LDS && shared_jobs<G>(sp) && v.ngroups > 1;
  if (!v.shared) { v.gs = DV; v.ngroups = (D + DV - 1) / DV; }
  v.g0 = D < v.gs ? D : v.gs;
  return v;
}

// verify_batch's group-0 level rows (phase 1a's tree loads), made while the
// batch's last children are still being expanded (they read the tree, not
// the batch's values; vl overlays the batch's wave buffers, which the game's
// workgroup is done with).  All threads; no barrier.
template <class G, class Acc>
__device__ __forceinline__ void verify_preload(Smem<G>& sm, const SearchParams& sp, const TreeView& TV, const Acc& T,
                                               const int* nact, int D) {
  if constexpr (decltype(sm.u.f)::BATCH) {
    typedef VerifyLds<G, verify_depth<G>()> V;
    V& vl = *reinterpret_cast<V*>(&sm.u.f.wv[0]);
    const VerifyPlan v = verify_plan<G, Acc>(sp, D);
    for (int k = __builtin_amdgcn_readfirstlane(wave_id()); k < v.g0; k += G::WAVES)
      verify_load_level<G, Acc>(sm, sp, TV, T, nact, vl, k, k, sm.t.ract);
  }
}

template <class G, class Acc>
__device__ __forceinline__ int verify_batch(Smem<G>& sm, const SearchParams& sp, const EngineArrays& E, int g,
                                            const TreeView& TV, Acc& T, int* nact, int leaf, int D, int B, int nid,
                                            Stamp* st = nullptr, bool preloaded = false) {
  if constexpr (!decltype(sm.u.f)::BATCH) {
    return 0;                                       // (no speculative batches without the batch LDS)
  } else {
  constexpr int DV = verify_depth<G>();
  typedef VerifyLds<G, DV> V;
  static_assert(sizeof(V) <= sizeof(sm.u.f.wv), "verification arrays overlay the batch buffers");
  V& vl = *reinterpret_cast<V*>(&sm.u.f.wv[0]);
  const int lane = lane_id_local();
  const bool alt = sp.variant == 0;
  const double* bv = sm.u.f.bv;
  // the node at depth d takes the share v (-1)^(D + 1 - d) of a batch child's backup
  if (tid_local() < G::AP) vl.failm[tid_local()] = 0;
  // Levels l0 .. l0 + nl - 1 at a time (every (i, l) check is independent of
  // the others; a failing i is recorded in failm whichever group finds it).
  // With helper workgroups (HBM trees), several groups are a job: each
  // workgroup claims groups and ORs its failing simulations into J.failm.
  // (preloaded: group 0's level rows are in vl already -- the game's
  // workgroup checks group 0 itself, first)
  const VerifyPlan vp = verify_plan<G, Acc>(sp, D);
  const int gs = vp.gs, ngroups = vp.ngroups;
  const bool shared = vp.shared;
  if (shared) {
    const JobView J = job_of<G>(E, g);
    const unsigned bseq = job_begin(J, ngroups, preloaded ? 1u : 0u);
    if (tid_local() == 0) {
      int* info = J.info();
      info[0] = ngroups; info[1] = nid; info[2] = leaf; info[3] = gs; info[4] = 3;
      info[5] = sm.t.ract; info[6] = D; info[7] = B;
    }
    if (tid_local() < G::AP) __hip_atomic_store(J.failm() + tid_local(), 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    job_publish(J, bseq);                          // (J.bv holds the batch's values already)
    int mine = 0;
    if (preloaded) {
      verify_levels<G, Acc>(sm, sp, TV, T, nact, D, B, 0, vp.g0, sm.t.ract, false, st, true);
      ++mine;
    }
    for (int grp; (grp = job_claim(sm, J, bseq, ngroups, 1)) >= 0; ++mine)
      verify_levels<G, Acc>(sm, sp, TV, T, nact, D, B, grp * gs, min(gs, D - grp * gs), sm.t.ract, false, st);
    if (mine > 0 && tid_local() < G::AP && vl.failm[tid_local()])
      __hip_atomic_fetch_or(J.failm() + tid_local(), (unsigned long long)vl.failm[tid_local()], __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    job_wait(J, mine, ngroups);
    if (tid_local() < G::AP)
      vl.failm[tid_local()] = __hip_atomic_load(J.failm() + tid_local(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    for (int l0 = 0; l0 < D; l0 += DV)
      verify_levels<G, Acc>(sm, sp, TV, T, nact, D, B, l0, D - l0 < DV ? D - l0 : DV, sm.t.ract, l0 == 0, st,
                            preloaded && l0 == 0);
  }
  if ((D == 0 || shared) && tid_local() == 0) prefix_sums<G>(T.ws(0), bv, B, alt && ((D + 1) & 1), vl.wroot);
  if (tid_local() == 0) {
    int f = B;
#pragma unroll
    for (int j = G::AP - 1; j >= 0; --j) {
      uint64_t mm = vl.failm[j];
      if (j == 0) mm &= ~1ull;                         // (simulation i = 0 reached the leaf already)
      if (mm) f = 64 * j + __builtin_ctzll(mm);
    }
    vl.fail = f < B ? f : B;
  }
  __syncthreads();
  if (st) st->lap(73);
  const int m = vl.fail;
  // ---- 3. the tree takes the m accepted simulations: path node p_d (d >= 1)
  // gets m visits and the first m of its shares, summed in simulation order
  // (prefix_sums' f64 chain, one lane per node) ----
  if (wave_id() == 0) {
    for (int d = lane; d <= D; d += 64) {
      if (d == 0) {
        T.set(0, T.vis(0) + m, vl.wroot[m]);
      } else {
        const int p = T.path(d);
        const bool neg = alt && ((D + 1 - d) & 1);
        double w = T.ws(p);
#pragma unroll 8
        for (int k = 0; k < m; ++k) w = w + (neg ? -bv[k] : bv[k]);
        const int n = T.vis(p) + m;
        T.set(p, n, w);
        if constexpr (Acc::LDS)
          if (d == 1) { sm.t.rvis[sm.t.ract] = n; sm.t.rws[sm.t.ract] = w; }
      }
    }
    wave_lds_sync();
    for (int i = lane; i < m; i += 64) {            // the new children
      const int ai = sm.u.f.acts[i], n2 = nid + i;
      const double v = 0.0 + bv[i];
      T.set(n2, 1, v);
      nact[n2] = ai;
      T.set_child(leaf, ai, n2);
      if (leaf == 0) T.add_root_child(ai, v);       // (set_child zeroed the mirror)
    }
    if (lane == 0) { sm.t.newest = -1; sm.t.ycache = leaf; }
  }
  __syncthreads();
  if (st) st->lap(74);
  return m;
  }
}

// A helper workgroup of game g (k_selfplay_move's blocks past the games):
// jobs until the game's workgroup posts kJobExit (or none comes for ~seconds):
// batch expansions, parent convs and replay checks.
template <class G>
__device__ __forceinline__ void helper_loop(Smem<G>& sm, const NetParams& np_a, const NetParams& np_b,
                                            const SearchParams& sp, const EngineArrays& E, int g) {
  const JobView J = job_of<G>(E, g);
  const TreeView TV = TreeViewOf<G>::make(E, g);
  float* pool = pool_of<G>(E, g);
  unsigned last = 0;
  for (;;) {
    if (tid_local() == 0) {
      unsigned s = __hip_atomic_load(J.seq(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (long long spins = 0; (s == last || s == 0) && spins < (1ll << 26); ++spins) {
        __builtin_amdgcn_s_sleep(kJobPollSleep);
        s = __hip_atomic_load(J.seq(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (s == last || s == 0) s = kJobExit;           // (bounded wait: give up)
      if (s != kJobExit) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      sm.bc[2] = (int)s;
    }
    __syncthreads();
    const unsigned s = (unsigned)sm.bc[2];
    if (s == kJobExit) return;
    last = s;
    const int* info = J.info();
    const int B = info[0], nid0 = info[1], leaf = info[2], net = info[3], kind = info[4];
    const NetParams np = select_params(net != 0, np_b, np_a);
    if (kind == 3) {                                   // replay checks of a batch (verify_batch)
      constexpr int DV = verify_depth<G>();
      typedef VerifyLds<G, DV> V;
      V& vl = *reinterpret_cast<V*>(&sm.u.f.wv[0]);
      const int ngroups = B, gs = info[3], ract = info[5], D = info[6], nb = info[7];
      const double* bvg = J.bv(G::A);
      for (int k = tid_local(); k < nb; k += G::THREADS) sm.u.f.bv[k] = bvg[k];
      if (tid_local() < G::AP) vl.failm[tid_local()] = 0;
      __syncthreads();
      const TreeAcc<G, false> T(TV, sm.t);
      const int* nact = E.nact + (size_t)g * ((size_t)E.S + 1);
      int mine = 0;
      for (int grp; (grp = job_claim(sm, J, s, ngroups, 1)) >= 0; ++mine)
        verify_levels<G, TreeAcc<G, false>>(sm, sp, TV, T, nact, D, nb, grp * gs, min(gs, D - grp * gs), ract,
                                            false);
      if (mine > 0 && tid_local() < G::AP && vl.failm[tid_local()])
        __hip_atomic_fetch_or(J.failm() + tid_local(), (unsigned long long)vl.failm[tid_local()], __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid_local() == 0 && mine > 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (ROCm 7.2 may drop the fence's own wait)
        __hip_atomic_fetch_add(J.done(), (unsigned)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      continue;
    }
    if (kind == 4 || kind == 5) {                      // the representation's conv2 / conv3
      float* lat = pool + (size_t)(E.S + 1) * G::C * G::CS;
      const int mine = kind == 4 ? rep_strips<G, 64, 64, 0>(sm, J, s, np.w_conv2, np.b_conv2, lat, pool, nullptr,
                                                            sm.hfin)
                                 : rep_strips<G, 64, G::C, 2>(sm, J, s, np.w_conv3, np.b_conv3, pool, lat,
                                                              np.head_w + G::C, J.hfin(G::A));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid_local() == 0 && mine > 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (ROCm 7.2 may drop the fence's own wait)
        __hip_atomic_fetch_add(J.done(), (unsigned)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      continue;
    }
    if (kind != 0) {                                   // a parent's conv
      const int par = info[1], act = info[5];
      const int mine = conv_strips<G>(sm, np, J, s, pool + (size_t)(E.S + 1) * G::C * G::CS,
                                      pool + (size_t)leaf * G::C * G::CS,
                                      kind == 2 ? pool + (size_t)par * G::C * G::CS : nullptr,
                                      np.etab + (size_t)act * 9 * G::C);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid_local() == 0 && mine > 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (ROCm 7.2 may drop the fence's own wait)
        __hip_atomic_fetch_add(J.done(), (unsigned)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      continue;
    }
    for (int a = tid_local(); a < G::A; a += G::THREADS) sm.t.valid[a] = J.valid(G::A)[a];
    if (tid_local() == 0) sm.t.pass_prior = *J.pass_prior();
    stage_head_scalars(np.hs, sm.t.hsc);
    load_y<G>(sm, nullptr, np.head_w);                 // (GLOBAL_Y: the head weights only)
    __syncthreads();
    const float* yg = pool + (size_t)leaf * G::C * G::CS;
    const int mine = job_rounds<G, false, true>(sm, np, sp, TV, yg, J, s, B, nid0, true);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's row and value stores
    __syncthreads();
    if (tid_local() == 0 && mine > 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (ROCm 7.2 may drop the fence's own wait)
      __hip_atomic_fetch_add(J.done(), (unsigned)mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// 19x19 epoch tail (sp.tail, whole-game launches): a helper workgroup whose
// game has ended -- and the game's own workgroup -- move on to the running
// game with the fewest re-assigned helpers (JobView::nhelp; the nearest after
// `hint` among ties) and serve its jobs.  Every job kind takes any number of
// workgroups (claims are dynamic), so this changes who computes, not what.
// Returns the game or -1 when none is running.  All threads.
template <class G>
__device__ __forceinline__ int join_running_game(Smem<G>& sm, const EngineArrays& E, int games, int hint) {
  if (wave_id() == 0) {
    const int lane = lane_id_local();
    unsigned best = 0xFFFFFFFFu;
    int pick = -1;
    for (int k0 = 1; k0 <= games; k0 += 64) {
      const int k = k0 + lane;
      const int t = (hint + k) % games;
      unsigned key = 0xFFFFFFFFu;
      if (k <= games) {
        const JobView Jt = job_of<G>(E, t);
        if (__hip_atomic_load(Jt.started(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 &&
            __hip_atomic_load(Jt.seq(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kJobExit)
          key = __hip_atomic_load(Jt.nhelp(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      // (helpers, distance) lexicographic: the fewest helpers, then the nearest
      unsigned long long v = (unsigned long long)key << 32 | (unsigned)k;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = __shfl_xor(v, o);
        v = w < v ? w : v;
      }
      if ((unsigned)(v >> 32) < best) { best = (unsigned)(v >> 32); pick = (hint + (int)(v & 0xFFFFFFFFu)) % games; }
    }
    if (lane == 0) {
      if (pick >= 0) __hip_atomic_fetch_add(job_of<G>(E, pick).nhelp(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      sm.bc[2] = pick;
    }
  }
  __syncthreads();
  const int t = sm.bc[2];
  __syncthreads();
  return t;
}

// The simulations of one search with the tree accessor Acc (LDS or HBM stats).
//
// Factored dynamics also batch SPECULATIVELY: once a simulation's select ends
// at a leaf with u >= 2 unexpanded eligible children, the next simulations
// will pick further unexpanded children of the same leaf -- in an order fixed
// by their draws -- as long as the select walk from the root reaches that
// leaf again.  In the reference's trees it does ~99 % of the time (the same
// depth-1 node keeps the root's PUCT maximum).  So B children of the leaf are
// expanded as one batch (batch_expand), and wave 0 then replays the
// simulations one by one: select from the root (exactly as the sequential
// loop would, on the tree as it stands); if it reaches the predicted (leaf,
// action), the precomputed child is attached and backed up; at the first
// miss the batch's remaining children are dropped (their node ids and rows
// are reused) and the loop continues from that select.  The tree is the
// sequential one node for node.
template <class G, class Acc>
__device__ __forceinline__ void sim_loop(Smem<G>& sm, const NetParams& np, const SearchParams& sp,
                                         const EngineArrays& E, int g, const TreeView& TV, uint64_t key) {
  float* pool = pool_of<G>(E, g);
  const size_t node_floats = (size_t)G::C * G::CS;
  float* scratch = pool + (size_t)(E.S + 1) * node_floats;
  int* nact = E.nact + (size_t)g * ((size_t)E.S + 1);
  const int S = sp.num_simulations;
  const bool factored = sp.factored != 0;
  constexpr bool BATCH = decltype(sm.u.f)::BATCH;
  Acc T(TV, sm.t);
  tree_reset_root<G>(T);
  if (tid_local() == 0) {
    sm.t.newest = -1; sm.t.newp_node = -1; sm.t.ycache = -1; sm.t.rowc_node = -1; sm.t.lognode = -1;
  }
  __syncthreads();

  int nodes = 1, convs = 0;
  // prior rows formed (HBM writes of a node's priors + child row): eager
  // expansions, and lazily expanded nodes on a select's first arrival
  int rows = 0;
  // (batched children with eager rows: the HBM trees' non-shared batches
  // unless self-play keeps their policy head lazy, sp.lazy_rows)
  const bool eager_rows = !(Acc::LDS || shared_jobs<G>(sp) || (decltype(sm.u.f)::GLOBAL_Y && sp.lazy_rows));
  Stamp st(E.stamps);
  int sim = 0;
  if (factored) {
    sim = root_batch<G, Acc>(sm, np, sp, E, g, TV, T, pool, scratch, nact, key, &st);
    if (eager_rows) rows += sim;
    nodes += sim;
    convs += sim > 0 ? 1 : 0;
    st.lap(4);
  }
  bool pending = false;                                   // a select for `sim` is already in sm.t
  while (sim < S) {
    if (!pending) {
      if (wave_id() == 0) {
        const int a = select_leaf<G>(sm.t, T, sp, key, sim, &st);
        if (lane_id_local() == 0) sm.t.action = a;
        st.wave_add(92, 1);
        st.wave_add(95, (unsigned long long)sm.t.depth);
      }
      __syncthreads();
    }
    pending = false;
    // the walk reached a lazily expanded node for the first time: its policy
    // sums from its parent's Y and E[a] by the whole workgroup, then wave 0
    // resumes the walk there (it settles the node's priors and goes on)
    while (sm.t.action == kNeedLogits) {
      const int xn = sm.t.leaf, xd = sm.t.depth;
      st.lap(0);
      policy_sums_wg<G>(sm.t.logits, pool + (size_t)sm.t.lpar * node_floats,
                        np.etab + (size_t)sm.t.lact * 9 * G::C, np.head_w);
      if (tid_local() == 0) sm.t.lognode = xn;
      ++rows;
      __syncthreads();
      st.lap(32);
      if (tid_local() == 0) st.wave_add(34, 1);
      if (wave_id() == 0) {
        const int a = select_leaf<G>(sm.t, T, sp, key, sim, &st, xn, xd);
        if (lane_id_local() == 0) sm.t.action = a;
      }
      __syncthreads();
      st.lap(33);
    }
    st.lap(0);
    const int a = sm.t.action, leaf = sm.t.leaf, depth = sm.t.depth;
    if (a < 0) {                                         // terminal leaf: backup 0 (:188-191)
      // self_play.py: terminal leaf -> backup 0 (:188-191); main.py: nothing (:296)
      if (wave_id() == 0 && a == -1) backup<G>(T, depth, -1, 0.0);
      __syncthreads();
      ++sim;
      continue;
    }
    const float* heads;
    const int nid = nodes;
    if (factored) {
      // the leaf's conv Y exists once it has a child; otherwise compute it now
      // (from its latent, rebuilt from its parent's Y unless it is the root)
      float* yleaf = pool + (size_t)leaf * node_floats;
      int yc = sm.t.ycache;
      bool prepicked = false;                            // the batch's picks went out during the conv job
      static_assert(!decltype(sm.u.f)::CACHE || 3 * G::C <= G::THREADS, "one head weight per thread");
      float hwpre = 0.f;                                 // this thread's head weight, fetched before the conv
      bool hwready = false;
      if (!sm.t.yready) {
        const bool sj = shared_jobs<G>(sp);
        // Winograd boards rebuild the latent inside the conv's input
        // transform (wino_input_rebuilt); the others materialize it first
        if (leaf != 0 && !sj && !G::WINO) {
          const int par = T.path(depth - 1);
          materialize<G>(scratch, pool + (size_t)par * node_floats, np.etab + (size_t)nact[leaf] * 9 * G::C,
                         sm.ulds());
        }
        st.lap(81);
        if (sj) {
          // (the strips read the parent's Y and E rows themselves; the batch's
          // picks are made while the helpers start on them)
          const int nun0 = sm.t.nunexp, B0 = BATCH ? (nun0 < S - sim ? nun0 : S - sim) : 1;
          prepicked = BATCH && B0 >= 2;
          conv_shared<G>(sm, np, E, g, leaf, sp.net, scratch, yleaf, &st, leaf != 0 ? T.path(depth - 1) : -1,
                         leaf != 0 ? nact[leaf] : 0, [&](unsigned cb) {
                           if (prepicked && wave_id() == 0) {
                             uint64_t um0[G::AP];
#pragma unroll
                             for (int j = 0; j < G::AP; ++j)
                               um0[j] = sm.t.umask[j] & ((a >> 6) == j ? ~(1ull << (a & 63)) : ~0ull);
                             pick_all<G>(um0, nun0 - 1, 1, B0 - 1, key, sim + 1, sm.u.f.acts, &st,
                                         job_of<G>(E, g).acts(), cb + 1);
                           }
                         });
        } else if (G::WINO && leaf != 0) {
          const int par = T.path(depth - 1);
          // the expansion's head weights (L.hw, which the conv overwrites) are
          // fetched before the conv and stored after it: the L2 round trip
          // runs under the conv instead of after it
          if constexpr (decltype(sm.u.f)::CACHE) hwpre = tid_local() < 3 * G::C ? np.head_w[tid_local()] : 0.f;
          // a tail helper registered with this game: the conv as a tail job
          bool tail = false;
          if constexpr (TailConvs<G>::value) {
            if (sp.tail) {
              if (tid_local() == 0)
                sm.bc[3] = __hip_atomic_load(job_of<G>(E, g).nhelp(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > 0;
              __syncthreads();
              tail = sm.bc[3] != 0;
            }
          }
          if (tail) {
            conv_tail<G>(sm, np, E, g, leaf, par, nact[leaf], sp.net, yleaf, y_lds_target<G>(sm),
                         y_lds_target<G>(sm) != nullptr && yc == par, &st);
          } else {
            latent_conv_rebuilt<G>(sm, np, pool + (size_t)par * node_floats, np.etab + (size_t)nact[leaf] * 9 * G::C,
                                   yleaf, &st, y_lds_target<G>(sm), y_lds_target<G>(sm) != nullptr && yc == par);
          }
          hwready = true;
        } else {
          latent_conv<G, G::C, G::C, 0, true>(sm, np.w_dyn, np.b_dyn, scratch, G::CS, nullptr, yleaf, G::CS,
                                              G::CS, nullptr, &st, G::WINO ? y_lds_target<G>(sm) : nullptr);
        }
        __syncthreads();                                 // Y stores before the expansion reads them
        st.lap(82);
        // the conv overwrote the union; one-strip Winograd boards got the
        // leaf's Y into L.yc by the conv itself (only the head weights reload)
        if (!sj && G::WINO && y_lds_target<G>(sm) != nullptr) {
          if (hwready) {
            if (tid_local() < 3 * G::C) sm.u.f.hw[tid_local()] = hwpre;
          } else {
            load_hw<G>(sm, np.head_w);
          }
          if (tid_local() == 0) sm.t.ycache = leaf;
          yc = leaf;
          __syncthreads();
        } else {
          yc = -1;
        }
        if (tid_local() == 0) { st.wave_add(59, 1); ++convs; }   // convs run
      }
      const int nun = sm.t.nunexp;
      const int B = BATCH ? (nun < S - sim ? nun : S - sim) : 1;
      if (BATCH && B >= 2) {
        // ---- speculative batch of B children of `leaf` ----
        st.lap(69);
        if (yc != leaf) load_y<G>(sm, yleaf, np.head_w);
        if constexpr (Acc::LDS) {
          if (leaf != 0 && sm.t.rowc_node != leaf) {      // the replay's selects read leaf's rows from LDS
            for (int i = tid_local(); i < G::A; i += G::THREADS) {
              sm.t.rowc_child[i] = TV.child[(size_t)leaf * G::A + i];
              sm.t.rowc_prior[i] = TV.prior[(size_t)leaf * G::A + i];
            }
            __syncthreads();
            if (tid_local() == 0) sm.t.rowc_node = leaf;
          }
        }
        if (tid_local() == 0) { sm.u.f.acts[0] = a; sm.t.npick = 1; sm.t.ngrab = 0; }
        __syncthreads();
        st.lap(70);
        uint64_t um[G::AP];
#pragma unroll
        for (int j = 0; j < G::AP; ++j) um[j] = sm.t.umask[j];
#pragma unroll
        for (int j = 0; j < G::AP; ++j)
          if ((a >> 6) == j) um[j] &= ~(1ull << (a & 63));
        if (shared_jobs<G>(sp)) {
          batch_expand_shared<G, Acc::LDS>(sm, np, sp, E, g, TV, B, nid, leaf, sp.net, yleaf, um, nun - 1, 1, key,
                                           sim + 1, &st, prepicked, [&]() {
                                             if (replay_parallel(true, B, depth))
                                               verify_preload<G, Acc>(sm, sp, TV, T, nact, depth);
                                           });
          st.lap(71);
        } else {
          if (wave_id() == 0) {
            // every pick at once (pick_all), then published together
            pick_all<G>(um, nun - 1, 1, B - 1, key, sim + 1, sm.u.f.acts, &st);
            wave_lds_sync();
            if (lane_id_local() == 0) __hip_atomic_store(&sm.t.npick, B, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            st.lap(71);
          }
          batch_expand<G, Acc::LDS>(sm, np, sp, TV, B, nid, yleaf, &st);
        }
        __syncthreads();
        st.lap(5);
        if (eager_rows) rows += B;
        if (replay_parallel(shared_jobs<G>(sp), B, depth)) {
          const int m = verify_batch<G, Acc>(sm, sp, E, g, TV, T, nact, leaf, depth, B, nid, &st, shared_jobs<G>(sp));
          nodes += m;
          sim += m;
          st.lap(63);
          if (tid_local() == 0) { st.wave_add(31, 1); st.wave_add(28, (unsigned long long)m); }
          continue;
        }
        if (wave_id() == 0) {
          const int lane = lane_id_local();
          if (lane == 0) { sm.t.newest = -1; sm.t.ycache = leaf; }
          wave_lds_sync();
          int m = 0;
          const bool alt = sp.variant == 0;
          {
            for (int i = 0; i < B; ++i) {
              const int ai = sm.u.f.acts[i];
              if (i > 0) {
                const int a2 = select_leaf<G>(sm.t, T, sp, key, sim + i, &st);
                st.wave_add(92, 1);
                st.wave_add(95, (unsigned long long)sm.t.depth);
                if (a2 != ai || sm.t.leaf != leaf) {           // prediction ends: a2 is sim + i's select
                  if (lane == 0) sm.t.action = a2;
                  break;
                }
              }
              const int n2 = nid + i;
              if (lane == 0) { T.init(n2); nact[n2] = ai; }
              if (lane == (ai & 63)) T.set_child(leaf, ai, n2);
              // the next select reads leaf's child row: from LDS (rowc) on LDS
              // trees; otherwise let the HBM store land first
              if constexpr (!Acc::LDS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              backup<G>(T, depth, n2, sm.u.f.bv[i], alt);
              ++m;
            }
          }
          if (lane == 0) sm.t.bcast = m;
          st.wave_add(93, 1);
          st.wave_add(94, (unsigned long long)m);
        }
        __syncthreads();
        const int m = sm.t.bcast;
        nodes += m;
        sim += m;
        pending = m < B;
        st.lap(63);
        if (tid_local() == 0) { st.wave_add(31, 1); st.wave_add(28, (unsigned long long)m); }
        continue;
      }
      // ---- one expansion ----
      // (nid may be the id of a dropped batch child: clear its lazy mark, the
      // eager priors below are this node's)
      if (tid_local() == 0) {
        T.init(nid);
        sm.t.newest = nid;
        if constexpr (G::TREE_CAP > 0)
          if (nid < G::TREE_CAP) sm.t.rawp[nid >> 5] &= ~(1u << (nid & 31));
      }
      const unsigned long long t_x = st.now();
      expand_heads<G>(sm.u.f, yleaf, yc == leaf, np.etab + (size_t)a * 9 * G::C, np.head_w);
      if (tid_local() == 0) st.wave_add(56, st.now() - t_x);
      ++rows;
      __syncthreads();
      if (tid_local() == 0 && decltype(sm.u.f)::CACHE) sm.t.ycache = leaf;   // read by all before the barrier
      heads = sm.u.f.xh;
    } else {
      if (tid_local() == 0) { T.init(nid); sm.t.newest = nid; }
      latent_conv<G, G::C, G::C, 3>(sm, np.w_dyn, np.b_dyn, pool + (size_t)leaf * node_floats, G::CS,
                                    np.emb + (size_t)a * G::C, pool + (size_t)nid * node_floats, G::CS, G::CS,
                                    np.head_w, &st);
      heads = sm.heads();
    }
    nodes += 1;
    st.lap(2);
    // wave 1: policy logits -> the new node's priors (published in LDS for a
    // select that reaches it); wave 0, meanwhile: value/reward heads, backup
    // and (next iteration) the next select.  Wave 0 issues no HBM stores, so
    // its tree loads never wait for store acks.  The select barrier joins them.
    if (wave_id() == 1) {
      const unsigned long long t1 = st.now();
      int* crow = TV.child + (size_t)nid * G::A;        // the new node: no children yet
      for (int i = lane_id_local(); i < G::A; i += 64) crow[i] = -1;   // (before its priors are published)
      float x[G::AP];
      if (factored) logits_regs<G, 1>(heads, true, sm.t.hsc, x);
      else logits_regs<G, Smem<G>::HEAD_PARTS>(heads, true, sm.t.hsc, x);
      const unsigned long long t2 = st.now();
      child_priors<G>(sm.t, x, TV.prior + (size_t)nid * G::A, nid, sp.variant);
      st.wave_add(57, t2 - t1);
      st.wave_add(58, st.now() - t2);
    }
    if (wave_id() == 0) {
      float r, v;
      if (factored) heads_value<G, 1>(heads, true, sm.t.hsc, r, v);
      else heads_value<G, Smem<G>::HEAD_PARTS>(heads, true, sm.t.hsc, r, v);
      if (lane_id_local() == (a & 63)) T.set_child(leaf, a, nid);
      if (lane_id_local() == 0) nact[nid] = a;
      backup<G>(T, depth, nid, (double)r + sp.discount * (double)v, sp.variant == 0);
    }
    st.lap(3);
    ++sim;
  }
  __syncthreads();
  st.flush();
  tree_flush<G>(T, nodes);
  if (tid_local() == 0) {
    E.nodes[g] = nodes;
    // direct dynamics: one conv per expansion
    atomicAdd(&E.counters[3], (unsigned long long)(factored ? convs : nodes - 1));
    atomicAdd(&E.counters[5], (unsigned long long)(factored ? rows : nodes - 1));
  }
  __syncthreads();
}

template <class G, class PlaneFn>
__device__ __forceinline__ void run_search(Smem<G>& sm, const NetParams& np, const SearchParams& sp,
                                  const EngineArrays& E, int g, PlaneFn planes, const double* noise,
                                  uint64_t key, unsigned long long* ts = nullptr, double* noise_out = nullptr) {
  const TreeView TV = TreeViewOf<G>::make(E, g);
  if (tid_local() == 0) sm.t.ngrab = 0;             // draw_dirichlet's counter (build_mask's barrier orders it)
  build_mask<G>(sm.t, sp.pass_epsilon, [&](int a) { return planes(3, a); });
  float* pool = pool_of<G>(E, g);
  const size_t node_floats = (size_t)G::C * G::CS;
  // root latent: node 0's slot (direct; node 1's slot is strip-conv scratch) or
  // the scratch slot (factored: node 0's slot receives its conv Y)
  if (sp.factored && shared_jobs<G>(sp))
    representation<G>(sm, np, planes, pool + (size_t)(E.S + 1) * node_floats, G::CS, pool, ts ? ts + 3 : nullptr,
                      [&](int k) { rep_shared<G>(sm, np, E, g, sp.net, k); return true; });
  else if (sp.factored)
    representation<G>(sm, np, planes, pool + (size_t)(E.S + 1) * node_floats, G::CS, pool, ts ? ts + 3 : nullptr);
  else
    representation<G>(sm, np, planes, pool, G::CS, pool + node_floats, ts ? ts + 3 : nullptr);
#ifdef MZGO_STAMPS
  if (ts) ts[0] = __builtin_amdgcn_s_memtime();
#endif
  if (noise) {
    if (wave_id() == 0) root_priors<G>(sm.t, TV, sp, noise, key, nullptr, noise_out);
  } else {
    static_assert(G::AP < G::WAVES, "a wave per 64 Gamma draws besides wave 0");
    draw_dirichlet<G>(sm.t, key, sp.dirichlet_alpha, &sm.t.ngrab);
    if (wave_id() == 0) root_priors<G>(sm.t, TV, sp, noise, key, &sm.t.ngrab, noise_out);
  }
  __syncthreads();
#ifdef MZGO_STAMPS
  if (ts) ts[1] = __builtin_amdgcn_s_memtime();
#endif
  if constexpr (G::TREE_CAP > 0) {
    if (sp.num_simulations + 2 <= G::TREE_CAP) {
      sim_loop<G, TreeAcc<G, true>>(sm, np, sp, E, g, TV, key);
      return;
    }
  }
  sim_loop<G, TreeAcc<G, false>>(sm, np, sp, E, g, TV, key);
}

// root-child visit counts and root value of the finished search
template <class G>
__device__ __forceinline__ void search_outputs(const EngineArrays& E, int g, int* out_visits, double* out_value) {
  const TreeView T = TreeViewOf<G>::make(E, g);
  for (int a = tid_local(); a < G::A; a += G::THREADS) {
    const int c = T.child[a];
    if (out_visits) out_visits[(size_t)g * G::A + a] = c >= 0 ? T.visits[c] : 0;
  }
  if (tid_local() == 0 && out_value) {
    const int n = T.visits[0];
    out_value[g] = n > 0 ? T.wsum[0] / (double)n : 0.0;
  }
}

// Form the priors of every lazily expanded node no select reached
// (TreeLds::rawp): the search API exports whole trees (mzgo_tree_export),
// self-play does not and skips this.  Each wave takes parents p = wave,
// wave + WAVES, ... and every raw child c = child[p][a]: its policy sums
// from p's Y and E[a] (policy_sums_wave), then settle_lazy.  All threads;
// the batch buffers serve as per-wave scratch.
template <class G>
__device__ __forceinline__ void settle_all_priors(Smem<G>& sm, const NetParams& np, const EngineArrays& E, int g,
                                                  int nodes, int variant) {
  if constexpr (decltype(sm.u.f)::BATCH && G::TREE_CAP > 0) {
    const TreeView TV = TreeViewOf<G>::make(E, g);
    const float* pool = pool_of<G>(E, g);
    const int wave = __builtin_amdgcn_readfirstlane(wave_id());
    const int lane = lane_id_local();
    auto& W = sm.u.f.wv[wave];
    static_assert(sizeof(W.xw) >= sizeof(float) * G::CELLS, "a wave's head rows hold one node's policy sums");
    const int lim = nodes < G::TREE_CAP ? nodes : G::TREE_CAP;
    if (wave == 0 && lane == 0) sm.t.lognode = -1;
    for (int p = wave; p < lim; p += G::WAVES) {
      if (sm.t.is_raw(p)) continue;                  // (no children)
      for (int a0 = 0; a0 < G::A; a0 += 64) {
        const int a = a0 + lane;
        const int c = a < G::A ? TV.child[(size_t)p * G::A + a] : -1;
        for (uint64_t m = __ballot(c > 0 && c < lim && sm.t.is_raw(c)); m; m &= m - 1) {
          const int l = __builtin_ctzll(m);
          const int cc = __builtin_amdgcn_readlane(c, l), ca = a0 + l;
          policy_sums_wave<G>(W.xw, pool + (size_t)p * G::C * G::CS, np.etab + (size_t)ca * 9 * G::C, np.head_w);
          wave_lds_sync();
          float x[G::AP], q[G::AP];
          policy_logits<G>(W.xw, sm.t.hsc, x);
          child_prior_regs<G>(sm.t, x, q, variant, W.fb, W.db);
#pragma unroll
          for (int j = 0; j < G::AP; ++j)
            if (lane + 64 * j < G::A) {
              TV.prior[(size_t)cc * G::A + lane + 64 * j] = q[j];
              TV.child[(size_t)cc * G::A + lane + 64 * j] = -1;
            }
          wave_lds_sync();
        }
      }
    }
    __syncthreads();
    for (int i = tid_local(); i < (G::TREE_CAP + 31) / 32; i += G::THREADS) sm.t.rawp[i] = 0u;
  }
  __syncthreads();
}

template <int N, int C>
__global__ void __launch_bounds__((Geo<N, C>::THREADS)) __attribute__((amdgpu_waves_per_eu(Geo<N, C>::WPE, Geo<N, C>::WPE))) k_search(NetParams np_arg, SearchParams sp, EngineArrays E_arg,
                                                      const float* __restrict__ root_obs,
                                                      const double* __restrict__ noise, int game_base,
                                                      int move_index, int* out_visits, double* out_value) {
  typedef Geo<N, C> G;
  __shared__ Smem<G> sm;
  static_assert(sizeof(Smem<G>) <= 160 * 1024, "one workgroup per CU: the whole LDS at most");
  if constexpr (G::WINO) wino_raw_zero<G>(sm.raw);        // zero halo of the conv input planes
  // (as k_selfplay_move: no address arithmetic hoisted into registers kept
  // live across the whole search -- it spilled, 68 B/lane at 19x19)
  const EngineArrays E = launder_arrays(E_arg);
  const NetParams np = launder_params(np_arg);
  const int g = blockIdx.x;
  const float* o = root_obs + (size_t)g * 6 * G::CELLS;
  const uint64_t key = stream_key(sp.seed, (uint32_t)(game_base + g), (uint32_t)move_index);
  run_search<G>(sm, np, sp, E, g, [&](int c, int j) { return o[c * G::CELLS + j]; },
                noise ? noise + (size_t)g * G::A : nullptr, key);
  settle_all_priors<G>(sm, np, E, g, E.nodes[g], sp.variant);
  search_outputs<G>(E, g, out_visits, out_value);
}

// ---------------------------------------------------------------------------
// Boards
// ---------------------------------------------------------------------------
template <class G>
__device__ __forceinline__ void load_board(Smem<G>& sm, const EngineArrays& E, int g, BoardMeta& m) {
  for (int c = tid_local(); c < G::CELLS; c += G::THREADS) {
    sm.stone[c] = E.stones[(size_t)g * G::CELLS + c];
    sm.invd[c] = E.invd[(size_t)g * G::CELLS + c];
  }
  const int* mm = E.meta + g * 4;
  m.turn = mm[0]; m.passed = mm[1]; m.done = mm[2]; m.moves = mm[3];
  __syncthreads();
}

template <class G>
__device__ __forceinline__ void store_board(Smem<G>& sm, const EngineArrays& E, int g, const BoardMeta& m) {
  for (int c = tid_local(); c < G::CELLS; c += G::THREADS) {
    E.stones[(size_t)g * G::CELLS + c] = sm.stone[c];
    E.invd[(size_t)g * G::CELLS + c] = sm.invd[c];
  }
  if (tid_local() == 0) {
    int* mm = E.meta + g * 4;
    mm[0] = m.turn; mm[1] = m.passed; mm[2] = m.done; mm[3] = m.moves;
  }
}

template <class G>
__device__ __forceinline__ float board_plane(const Smem<G>& sm, const BoardMeta& m, int c, int j) {
  switch (c) {
    case 0: return sm.stone[j] == 1 ? 1.f : 0.f;
    case 1: return sm.stone[j] == 2 ? 1.f : 0.f;
    case 2: return (float)m.turn;
    case 3: return (float)sm.invd[j];
    case 4: return (float)m.passed;
    default: return (float)m.done;
  }
}

template <int N, int C>
__global__ void __launch_bounds__((Geo<N, C>::THREADS)) __attribute__((amdgpu_waves_per_eu(Geo<N, C>::WPE, Geo<N, C>::WPE))) k_board_reset(EngineArrays E) {
  typedef Geo<N, C> G;
  const int g = blockIdx.x;
  for (int c = tid_local(); c < G::CELLS; c += G::THREADS) {
    E.stones[(size_t)g * G::CELLS + c] = 0;
    E.invd[(size_t)g * G::CELLS + c] = 0;
  }
  if (tid_local() < 4) E.meta[g * 4 + tid_local()] = 0;
  if (tid_local() == 0) { E.status[g] = 0; E.game_len[g] = 0; E.final_reward[g] = 0.0; }
}

// Step every slot with actions[g] >= 0 (gogame.next_state); status[g] gets a
// BOARD_* code; winner[g] = GoEnv.winner() after the step (0 unless ended).
template <int N, int C>
__global__ void __launch_bounds__((Geo<N, C>::THREADS)) __attribute__((amdgpu_waves_per_eu(Geo<N, C>::WPE, Geo<N, C>::WPE))) k_board_step(EngineArrays E, const int* __restrict__ actions,
                                                          int* status, double* winner, double komi) {
  typedef Geo<N, C> G;
  __shared__ Smem<G> sm;
  static_assert(sizeof(Smem<G>) <= 160 * 1024, "one workgroup per CU: the whole LDS at most");
  const int g = blockIdx.x;
  const int a = actions[g];
  if (a < 0) return;
  BoardMeta m;
  load_board<G>(sm, E, g, m);
  BoardLds<G> b = board_lds<G>(sm);
  const int st = board_step<G>(b, m, a);
  __syncthreads();
  if (st == BOARD_OK) store_board<G>(sm, E, g, m);
  double w = 0.0;
  if (st == BOARD_OK && m.done) w = board_winning<G>(b, komi);
  if (tid_local() == 0) {
    if (status) status[g] = st;
    if (winner) winner[g] = w;
  }
}

// f64 observation planes [G][6][CELLS] of the current boards (GoEnv state)
template <int N, int C>
__global__ void __launch_bounds__((Geo<N, C>::THREADS)) __attribute__((amdgpu_waves_per_eu(Geo<N, C>::WPE, Geo<N, C>::WPE))) k_board_planes(EngineArrays E, double* planes) {
  typedef Geo<N, C> G;
  const int g = blockIdx.x;
  const int* mm = E.meta + g * 4;
  double* p = planes + (size_t)g * 6 * G::CELLS;
  for (int j = tid_local(); j < G::CELLS; j += G::THREADS) {
    const int s = E.stones[(size_t)g * G::CELLS + j];
    p[j] = s == 1; p[G::CELLS + j] = s == 2; p[2 * G::CELLS + j] = mm[0];
    p[3 * G::CELLS + j] = E.invd[(size_t)g * G::CELLS + j];
    p[4 * G::CELLS + j] = mm[1]; p[5 * G::CELLS + j] = mm[2];
  }
}

// ---------------------------------------------------------------------------
// Action choice (MuZeroAgent.select_action, self_play.py:357-402).  Wave 0.
// Writes the policy target to pol[A]; returns the action.
// ---------------------------------------------------------------------------
// main.py's move rule (self-play :660-673 and the arena evaluator :552-565):
// visit_counts = child visit counts where valid_mask > 0; argmax (first max)
// with policy = counts / sum, else random.choice(valid actions) with a one-hot
// policy.  Temperature plays no part.  Wave 0.
template <class G>
__device__ __forceinline__ int choose_action_main(TreeLds<G>& t, const TreeView& T, uint64_t key, double* pol) {
  const int lane = lane_id_local();
  double vc[G::AP];
  double bv = -1.0, tot = 0.0;
  int ba = 0x7fffffff, best_c = 0;
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    vc[j] = 0.0;
    if (a < G::A && mask_of<G>(t, a) > 0) { const int c = T.child[a]; vc[j] = c >= 0 ? (double)T.visits[c] : 0.0; }
    tot += vc[j];
    if (a < G::A && (vc[j] > bv || (vc[j] == bv && a < ba))) { bv = vc[j]; ba = a; }
  }
  tot = wave_sum(tot);                          // integer counts: exact in any order
  wave_argmax(bv, ba, best_c);
  int action = ba;
  if (!(tot > 0)) {                             // random.choice(valid actions)
    uint64_t vb[G::AP];
    int nvalid = 0;
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const int a = lane + 64 * j;
      vb[j] = __ballot(a < G::A && mask_of<G>(t, a) > 0);
      nvalid += __popcll(vb[j]);
    }
    uint32_t k = randbelow(draw(key, TAG_ACTION, 0), (uint32_t)nvalid);
    action = -1;
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const uint32_t c = __popcll(vb[j]);
      if (action < 0 && k < c) {
        uint64_t mm = vb[j];
        for (uint32_t i = 0; i < k; ++i) mm &= mm - 1;
        action = 64 * j + __ffsll((long long)mm) - 1;
      } else if (action < 0) {
        k -= c;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    if (a < G::A) pol[a] = tot > 0 ? vc[j] / tot : (a == action ? 1.0 : 0.0);
  }
  return action;
}

template <class G>
__device__ __forceinline__ int choose_action(TreeLds<G>& t, const TreeView& T, int compat, double temperature,
                                    uint64_t key, double* pol) {
  const int lane = lane_id_local();
  // visit_counts * valid_mask (zeros under compat "reference", §0.6)
  for (int a = lane; a < G::A; a += 64) {
    double vc = 0.0;
    if (compat == 1) { const int c = T.child[a]; vc = c >= 0 ? (double)T.visits[c] : 0.0; }
    t.dbuf[a] = vc * mask_of<G>(t, a);
  }
  wave_lds_sync();
  const double vsum = np_pairwise_sum<double, G::A>(t.dbuf);
  double vcm[G::AP];
#pragma unroll
  for (int j = 0; j < G::AP; ++j) { const int a = lane + 64 * j; vcm[j] = a < G::A ? t.dbuf[a] : 0.0; }
  wave_lds_sync();
  for (int a = lane; a < G::A; a += 64) t.dbuf[a] = mask_of<G>(t, a);
  wave_lds_sync();
  const double msum = np_pairwise_sum<double, G::A>(t.dbuf);
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    if (a < G::A) pol[a] = vsum > 0 ? vcm[j] / vsum : mask_of<G>(t, a) / msum;
  }
  const uint64_t h = draw(key, TAG_ACTION, 0);
  int action = 0;
  if (temperature == 0.0) {
    if (vsum > 0) {                                    // argmax, first max wins
      double bv = -1.0; int ba = 0x7fffffff;
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane + 64 * j;
        if (a < G::A && (vcm[j] > bv || (vcm[j] == bv && a < ba))) { bv = vcm[j]; ba = a; }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(bv, o); const int oa = __shfl_xor(ba, o);
        if (ov > bv || (ov == bv && oa < ba)) { bv = ov; ba = oa; }
      }
      action = ba;
    } else {                                           // random.choice(valid actions)
      uint64_t vb[G::AP];
      int nvalid = 0;
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane + 64 * j;
        vb[j] = __ballot(a < G::A && mask_of<G>(t, a) > 0);
        nvalid += __popcll(vb[j]);
      }
      uint32_t k = randbelow(h, (uint32_t)nvalid);
      action = -1;
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const uint32_t c = __popcll(vb[j]);
        if (action < 0 && k < c) {
          uint64_t mm = vb[j];
          for (uint32_t i = 0; i < k; ++i) mm &= mm - 1;
          action = 64 * j + __ffsll((long long)mm) - 1;
        } else if (action < 0) {
          k -= c;
        }
      }
    }
  } else {
    // probabilities = (vc**(1/T) * mask) / sum, or mask / sum(mask); then
    // np.random.choice's inverse CDF on a cumulative sum
    const double e = 1.0 / temperature;
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const int a = lane + 64 * j;
      if (a < G::A) t.dbuf[a] = (e == 1.0 ? vcm[j] : pow(vcm[j], e)) * mask_of<G>(t, a);
    }
    wave_lds_sync();
    const double ts = np_pairwise_sum<double, G::A>(t.dbuf);
    wave_lds_sync();
    for (int a = lane; a < G::A; a += 64) t.dbuf[a] = ts > 0 ? t.dbuf[a] / ts : mask_of<G>(t, a) / msum;
    wave_lds_sync();
    if (lane == 0) {
      double cdf = 0.0;
      for (int a = 0; a < G::A; ++a) cdf += t.dbuf[a];
      const double total = cdf;
      const double u = u01(h);
      double run = 0.0;
      int idx = 0;
      for (int a = 0; a < G::A; ++a) {
        run += t.dbuf[a];
        if (run / total <= u) idx = a + 1;
      }
      t.bcast = idx;
    }
    wave_lds_sync();
    action = t.bcast;
  }
  return action;
}

// ---------------------------------------------------------------------------
// One self-play move for every unfinished slot (run_self_play_game's loop
// body, self_play.py:465-507): record the observation, search, choose, step
// the board, record the result; finish the game on double pass or N*N moves.
// ---------------------------------------------------------------------------
struct PlayParams {
  double temperature;     // 1.0
  int temperature_moves;  // 15
  double komi;            // 0
  int game_base;          // global id of slot 0 (multi-GPU sharding)
  int epoch;              // game generation (slot restarts), part of the RNG key
  const double* noise;    // test hook: injected Dirichlet samples [G][M][A], or null
  double* noise_out;      // test hook: every root's normalised Dirichlet sample [G][M][A], or null
  int arena;              // 0: one network; 1: main.py's evaluator -- game i's first
                          // mover is network (i % 2), then the networks alternate
  int moves;              // moves per game in this launch (each game stops at its end)
};

template <int N, int C>
__global__ void __launch_bounds__((Geo<N, C>::THREADS)) __attribute__((amdgpu_waves_per_eu(Geo<N, C>::WPE, Geo<N, C>::WPE))) k_selfplay_move(NetParams np_a_arg, NetParams np_b_arg,
                                                             SearchParams sp, PlayParams pp, EngineArrays E_arg) {
  typedef Geo<N, C> G;
  __shared__ Smem<G> sm;
  static_assert(sizeof(Smem<G>) <= 160 * 1024, "one workgroup per CU: the whole LDS at most");
  // blocks past the games are helper workgroups (batch_expand_shared): helper h
  // serves game h % games.  Under round-robin dispatch that is the game's XCD
  // when games % 8 == 0 (every bench and test shape: 64, 256); otherwise a
  // helper may sit on another XCD -- a speed matter only, the job hand-offs
  // are agent-scope release / acquire and placement-independent.
  const int games = gridDim.x - sp.helpers;
  if ((int)blockIdx.x >= games) {
    if constexpr (Smem<G>::GLOBAL_Y && G::WINO) {
      wino_raw_zero<G>(sm.raw);                          // the conv strips' zero halo
      int t = (blockIdx.x - games) % games;
      for (;;) {
        helper_loop<G>(sm, np_a_arg, np_b_arg, sp, E_arg, t);
        if (!sp.tail) break;
        t = join_running_game<G>(sm, E_arg, games, t);   // its game ended: the epoch tail
        if (t < 0) break;
      }
    }
    return;
  }
  const int g = blockIdx.x;
  const EngineArrays& E = E_arg;
  // (every game workgroup counts itself resident: mzgo_stream_wait_started)
  if (tid_local() == 0) atomicAdd(&E_arg.counters[6], 1ull);
  auto release_helpers = [&]() {
    if ((sp.helpers > 0 || sp.tail) && tid_local() == 0)
      __hip_atomic_store(job_of<G>(E_arg, g).seq(), kJobExit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // an ended game's workgroup serves running games: their parent convs (9x9)
  // or all their jobs as one more helper (19x19)
  auto tail_phase = [&]() {
    if constexpr (Smem<G>::GLOBAL_Y && G::WINO) {
      if (sp.tail) {
        __syncthreads();
        for (int t = g; (t = join_running_game<G>(sm, E_arg, games, t)) >= 0;)
          helper_loop<G>(sm, np_a_arg, np_b_arg, sp, E_arg, t);
      }
    }
    if constexpr (TailConvs<G>::value)
      if (sp.tail) {
        __syncthreads();
#ifdef MZGO_STAMPS
        const unsigned long long th = __builtin_amdgcn_s_memtime();
#endif
        tail_help<G>(sm, np_a_arg, np_b_arg, E_arg, g, games);
#ifdef MZGO_STAMPS
        // slot 47: the workgroup's cycles in the tail phase (serving + waiting)
        if (tid_local() == 0 && E_arg.stamps) E_arg.stamps[(size_t)blockIdx.x * kStampPhases + 47] +=
            __builtin_amdgcn_s_memtime() - th;
#endif
      }
  };
  if (E.status[g] != 0) { release_helpers(); tail_phase(); return; }
  if ((sp.helpers > 0 || sp.tail) && tid_local() == 0)
    __hip_atomic_store(job_of<G>(E_arg, g).started(), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if constexpr (G::WINO) wino_raw_zero<G>(sm.raw);        // zero halo of the conv input planes
  BoardMeta m;
  load_board<G>(sm, E, g, m);
  // pp.moves moves of this game in one launch (the board stays in LDS between
  // them): a game's moves run back to back on its CU instead of every move of
  // every game waiting for the slowest game's move at a launch boundary
  for (int step = 0; step < pp.moves; ++step) {
#ifdef MZGO_STAMPS
  unsigned long long tm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  tm[0] = __builtin_amdgcn_s_memtime();
#else
  unsigned long long* tm = nullptr;
#endif
  const int mv = m.moves;
  // this move's view of the arguments (launder_global: no address arithmetic
  // of the move is hoisted above this point)
  const EngineArrays E = launder_arrays(E_arg);
  const NetParams np_a = launder_params(np_a_arg), np_b = launder_params(np_b_arg);
  // arena (main.py:535-549): turn 0 = "current" (np_a), 1 = "best" (np_b); game
  // i starts with turn i % 2 (evaluate, :597-599)
  // (field by field: a reference chosen between the two by-value kernel
  // arguments would copy both to scratch)
  const NetParams np = select_params(pp.arena && (((pp.game_base + g) + mv) & 1), np_b, np_a);
  const size_t rec = (size_t)g * E.max_moves + mv;
  for (int c = tid_local(); c < G::CELLS; c += G::THREADS) {
    E.rec_stones[rec * G::CELLS + c] = sm.stone[c];
    E.rec_invd[rec * G::CELLS + c] = sm.invd[c];
  }
  if (tid_local() == 0) E.rec_flags[rec] = (uint8_t)(m.turn | (m.passed << 1) | (m.done << 2));

  const uint32_t gid = (uint32_t)(pp.game_base + g) ^ ((uint32_t)pp.epoch << 24);
  const uint64_t key = stream_key(sp.seed, gid, (uint32_t)mv);
  const BoardMeta m0 = m;
  const double* noise = pp.noise ? pp.noise + ((size_t)g * E.max_moves + mv) * G::A : nullptr;
  double* noise_out = pp.noise_out ? pp.noise_out + ((size_t)g * E.max_moves + mv) * G::A : nullptr;
#ifdef MZGO_STAMPS
  tm[1] = __builtin_amdgcn_s_memtime();
#endif
  SearchParams spm = launder_search(sp);
  spm.net = (pp.arena && (((pp.game_base + g) + mv) & 1)) ? 1 : 0;
  run_search<G>(sm, np, spm, E, g, [&](int c, int j) { return board_plane<G>(sm, m0, c, j); }, noise, key,
                tm ? tm + 2 : nullptr, noise_out);
#ifdef MZGO_STAMPS
  tm[4] = __builtin_amdgcn_s_memtime();
#endif

  const TreeView T = TreeViewOf<G>::make(E, g);
  if (wave_id() == 0) {
    const double temp = mv < pp.temperature_moves ? pp.temperature : 0.0;
    const int a = sp.variant == 1 ? choose_action_main<G>(sm.t, T, key, E.rec_policy + rec * G::A)
                                  : choose_action<G>(sm.t, T, sp.compat, temp, key, E.rec_policy + rec * G::A);
    if (lane_id_local() == 0) {
      sm.bc[0] = a;
      E.rec_action[rec] = a;
      const int n = T.visits[0];
      E.rec_value[rec] = n > 0 ? T.wsum[0] / (double)n : 0.0;
    }
  }
  __syncthreads();
  const int action = sm.bc[0];
  BoardLds<G> b = board_lds<G>(sm);
  const int st = board_step<G>(b, m, action);
  __syncthreads();
  double w = 0.0;
  if (st == BOARD_OK && m.done) w = board_winning<G>(b, pp.komi);
  store_board<G>(sm, E, g, m);
#ifdef MZGO_STAMPS
  // move phases (slots 83-87): board load + record, representation, root
  // priors, the simulations, action choice + board step
  if (tid_local() == 0 && E.stamps) {
    const unsigned long long t5 = __builtin_amdgcn_s_memtime();
    unsigned long long* sl = E.stamps + (size_t)blockIdx.x * kStampPhases;
    sl[83] += tm[1] - tm[0];
    sl[84] += tm[2] - tm[1];
    sl[85] += tm[3] - tm[2];
    sl[86] += tm[4] - tm[3];
    sl[87] += t5 - tm[4];
    sl[88] += tm[5] - tm[1];                     // representation: board planes + conv1
    sl[89] += tm[6] - tm[5];                     //   conv2
    sl[90] += tm[2] - tm[6];                     //   conv3 + heads
  }
#endif
  const bool over = st != BOARD_OK || m.done || m.moves >= E.max_moves;
  if (tid_local() == 0) {
    E.rec_reward[rec] = w;
    atomicAdd(&E.counters[0], (unsigned long long)sp.num_simulations);
    atomicAdd(&E.counters[1], 1ull);
    if (st != BOARD_OK) {
      E.status[g] = 16 + st;
    } else if (m.done || m.moves >= E.max_moves) {
      E.status[g] = 1;
      E.game_len[g] = m.moves;
      E.final_reward[g] = m.done ? w : 0.0;      // env.winner() is 0 unless ended
      atomicAdd(&E.counters[2], 1ull);
    }
  }
  if (over) break;
  __syncthreads();                               // this move's LDS reads before the next move's writes
  }
  release_helpers();
  tail_phase();
}

// ---------------------------------------------------------------------------
// The move-parallel epoch, first launch: every game's moves without their
// searches (record, legal mask, action, board step, result).  A game's
// moves are a serial chain of board steps, each a few label-propagation
// rounds with a barrier apiece, so the step's latency is
// the launch's: a workgroup of BoardsGeo::THREADS (one cell per lane, 2 waves
// at 9x9) with a few KB of LDS instead of k_selfplay_move's 12 waves and 159
// KB.  Same operations as k_selfplay_move's move (build_mask, choose_action,
// board_step, board_winning with this workgroup as the team), so the records
// are the same.
// ---------------------------------------------------------------------------
template <class G>
struct BoardsGeo {
  static constexpr int THREADS = (G::CELLS + 63) / 64 * 64 < 512 ? (G::CELLS + 63) / 64 * 64 : 512;
};
template <class G>
struct BoardsTeam {
  static constexpr int SIZE = BoardsGeo<G>::THREADS;
  __device__ static int id() { return tid_local(); }
  __device__ static void sync() { __syncthreads(); }
  __device__ static bool any(int v) { return __syncthreads_or(v) != 0; }
  __device__ static bool leader() { return tid_local() == 0; }
};
template <class G>
struct BoardsSmem {
  TreeLds<G> t;                                          // choose_action's mask and scratch
  int label[G::CELLS], libs[G::CELLS], gsize[G::CELLS];
  int8_t stone[G::CELLS];
  uint8_t invd[G::CELLS];
  int killed[4];
  int misc[8];
  int bc[8];
};

template <int N, int C>
__global__ void __launch_bounds__((BoardsGeo<Geo<N, C>>::THREADS)) k_selfplay_boards(SearchParams sp, PlayParams pp,
                                                                                    EngineArrays E) {
  typedef Geo<N, C> G;
  typedef BoardsTeam<G> T;
  constexpr int BT = BoardsGeo<G>::THREADS;
  __shared__ BoardsSmem<G> sm;
  const int g = blockIdx.x;
  const int tid = tid_local();
  if (tid == 0) {
    atomicAdd(&E.counters[6], 1ull);
    E.mpq[2 * g + 1] = 0;
  }
  if (E.status[g] != 0) return;
  for (int c = tid; c < G::CELLS; c += BT) {
    sm.stone[c] = E.stones[(size_t)g * G::CELLS + c];
    sm.invd[c] = E.invd[(size_t)g * G::CELLS + c];
  }
  BoardMeta m;
  {
    const int* mm = E.meta + g * 4;
    m.turn = mm[0]; m.passed = mm[1]; m.done = mm[2]; m.moves = mm[3];
  }
  __syncthreads();
  BoardLds<G> b;
  b.stone = sm.stone; b.invd = sm.invd;
  b.label = sm.label; b.libs = sm.libs; b.gsize = sm.gsize;
  b.killed = sm.killed; b.misc = sm.misc;
  const int mv_first = m.moves;
  int played = 0;
  const TreeView TV = TreeViewOf<G>::make(E, g);         // (compat "reference" reads no tree)
  for (int step = 0; step < pp.moves; ++step) {
    const int mv = m.moves;
    const size_t rec = (size_t)g * E.max_moves + mv;
    for (int c = tid; c < G::CELLS; c += BT) {
      E.rec_stones[rec * G::CELLS + c] = sm.stone[c];
      E.rec_invd[rec * G::CELLS + c] = sm.invd[c];
    }
    if (tid == 0) E.rec_flags[rec] = (uint8_t)(m.turn | (m.passed << 1) | (m.done << 2));
    ++played;
    const uint32_t gid = (uint32_t)(pp.game_base + g) ^ ((uint32_t)pp.epoch << 24);
    const uint64_t key = stream_key(sp.seed, gid, (uint32_t)mv);
    // build_mask (self_play.py:152, :363) with this workgroup's stride
    {
      int any = 0;
      for (int a = tid; a < G::A; a += BT) {
        const uint8_t v = a < G::CELLS ? (sm.invd[a] == 0 ? 1 : 0) : 1;
        sm.t.valid[a] = v;
        any |= (a < G::CELLS) && v;
      }
      any = __syncthreads_or(any);
      if (tid == 0) sm.t.pass_prior = any ? sp.pass_epsilon : 1.0;
      __syncthreads();
    }
    if (wave_id() == 0) {
      const double temp = mv < pp.temperature_moves ? pp.temperature : 0.0;
      const int a = choose_action<G>(sm.t, TV, sp.compat, temp, key, E.rec_policy + rec * G::A);
      if (lane_id_local() == 0) {
        sm.bc[0] = a;
        E.rec_action[rec] = a;
      }
    }
    __syncthreads();
    const int action = sm.bc[0];
    const int st = board_step<G, T>(b, m, action);
    __syncthreads();
    double w = 0.0;
    if (st == BOARD_OK && m.done) w = board_winning<G, T>(b, pp.komi);
    for (int c = tid; c < G::CELLS; c += BT) {
      E.stones[(size_t)g * G::CELLS + c] = sm.stone[c];
      E.invd[(size_t)g * G::CELLS + c] = sm.invd[c];
    }
    const bool over = st != BOARD_OK || m.done || m.moves >= E.max_moves;
    if (tid == 0) {
      int* mm = E.meta + g * 4;
      mm[0] = m.turn; mm[1] = m.passed; mm[2] = m.done; mm[3] = m.moves;
      E.rec_reward[rec] = w;
      atomicAdd(&E.counters[0], (unsigned long long)sp.num_simulations);
      atomicAdd(&E.counters[1], 1ull);
      if (st != BOARD_OK) {
        E.status[g] = 16 + st;
      } else if (m.done || m.moves >= E.max_moves) {
        E.status[g] = 1;
        E.game_len[g] = m.moves;
        E.final_reward[g] = m.done ? w : 0.0;
        atomicAdd(&E.counters[2], 1ull);
      }
    }
    if (over) break;
    __syncthreads();                               // this move's LDS reads before the next move's writes
  }
  if (tid == 0) {
    E.mpq[2 * g] = mv_first;
    E.mpq[2 * g + 1] = played;
  }
}

// ---------------------------------------------------------------------------
// The move-parallel epoch, second launch (compat "reference", SURVEY.md §0.6:
// the action is a uniform draw over the legal moves and the policy target is
// mask / sum, so a game's board sequence never reads its searches and every
// (game, move) search is independent once the boards are played).  A
// persistent grid of one workgroup per CU claims (game, move) items from one
// queue -- the moves of every game, latest first -- and runs each search in
// its own tree slot (blockIdx.x) from the recorded observation; the search's
// root value is the record's.  The same searches, keys and noise as the
// game-per-workgroup launch, so the records are identical; the epoch's tail
// (a game's whole remaining move sequence on one CU while the others idle)
// shrinks to one search.
// ---------------------------------------------------------------------------
template <int N, int C>
__global__ void __launch_bounds__((Geo<N, C>::THREADS)) __attribute__((amdgpu_waves_per_eu(Geo<N, C>::WPE, Geo<N, C>::WPE))) k_search_queue(NetParams np_arg, SearchParams sp, PlayParams pp,
                                                            EngineArrays E_arg, int games) {
  typedef Geo<N, C> G;
  __shared__ Smem<G> sm;
  static_assert(sizeof(Smem<G>) <= 160 * 1024, "one workgroup per CU: the whole LDS at most");
  if constexpr (G::WINO) wino_raw_zero<G>(sm.raw);        // zero halo of the conv input planes
  // sp.helpers > 0 (19x19, MZGO_QUEUE_HELPERS): the first gridDim.x /
  // (1 + helpers per leader) workgroups claim searches, the others serve a
  // leader's batch expansions and parent convs as jobs (helper_loop) for the
  // whole launch, as a game's helpers do in the game-per-workgroup launch
  const int leaders = (int)gridDim.x - sp.helpers;
  if ((int)blockIdx.x >= leaders) {
    if constexpr (Smem<G>::GLOBAL_Y && G::WINO)
      helper_loop<G>(sm, np_arg, np_arg, sp, E_arg, ((int)blockIdx.x - leaders) % leaders);
    return;
  }
  const int slot = blockIdx.x;
  const int items = games * pp.moves;
  for (;;) {
    if (tid_local() == 0) sm.bc[0] = (int)atomicAdd((unsigned*)&E_arg.mpq[2 * games], 1u);
    __syncthreads();
    const int k = sm.bc[0];
    __syncthreads();                               // (sm.bc is the search's scratch too)
    if (k >= items) break;
    const int j = k / games, g = k % games;
    const int mv0 = __builtin_amdgcn_readfirstlane(E_arg.mpq[2 * g]);
    const int nmv = __builtin_amdgcn_readfirstlane(E_arg.mpq[2 * g + 1]);
    if (j >= nmv) continue;
    const int mv = mv0 + nmv - 1 - j;
    const EngineArrays E = launder_arrays(E_arg);
    const NetParams np = launder_params(np_arg);
    const size_t rec = (size_t)g * E.max_moves + mv;
    for (int c = tid_local(); c < G::CELLS; c += G::THREADS) {
      sm.stone[c] = E.rec_stones[rec * G::CELLS + c];
      sm.invd[c] = E.rec_invd[rec * G::CELLS + c];
    }
    const int fl = E.rec_flags[rec];
    BoardMeta m0;
    m0.turn = fl & 1; m0.passed = (fl >> 1) & 1; m0.done = (fl >> 2) & 1; m0.moves = mv;
    __syncthreads();
    const uint32_t gid = (uint32_t)(pp.game_base + g) ^ ((uint32_t)pp.epoch << 24);
    const uint64_t key = stream_key(sp.seed, gid, (uint32_t)mv);
    const double* noise = pp.noise ? pp.noise + rec * G::A : nullptr;
    double* noise_out = pp.noise_out ? pp.noise_out + rec * G::A : nullptr;
    SearchParams spm = launder_search(sp);
    spm.net = 0;
    run_search<G>(sm, np, spm, E, slot, [&](int c, int jj) { return board_plane<G>(sm, m0, c, jj); }, noise, key,
                  nullptr, noise_out);
    if (tid_local() == 0) {
      const TreeView T = TreeViewOf<G>::make(E, slot);
      const int n = T.visits[0];
      E.rec_value[rec] = n > 0 ? T.wsum[0] / (double)n : 0.0;
    }
    __syncthreads();                               // this search's LDS reads before the next board
  }
  if (sp.helpers > 0 && tid_local() == 0)
    __hip_atomic_store(job_of<G>(E_arg, slot).seq(), kJobExit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace mzgo

// mzgo_search.hpp -- the MCTS of self_play.py as wave64 device code.
//
// One game's tree lives in HBM as structure-of-arrays node pools; wave 0 of
// the game's workgroup walks it.  A lane owns actions a = lane + 64*j.
//
//   select_leaf       self_play.py:239-335  (unexpanded-first, min-max-Q PUCT)
//   expand + backup   self_play.py:198-230, :337-343
//   root_priors       self_play.py:151-182  (mask, normalise, Dirichlet, re-mask)
//   choose_action     self_play.py:357-402  (compat "reference" and "fixed")
//
// Numerics follow numpy's dtype chain: root priors float64,
// child priors float32 (softmax * root mask / numpy-ordered f32 sum), Q, U
// and scores float64, backup value float64 = reward + 0.99 * value.
#pragma once
#include "mzgo_common.hpp"
#include <type_traits>

namespace mzgo {

struct SearchParams {
  double c_puct;            // 2.5 (self_play.py:143)
  double discount;          // 0.99 (self_play.py:25)
  double dirichlet_alpha;   // 0.15
  double dirichlet_epsilon; // 0.02
  double pass_epsilon;      // 0.01
  int num_simulations;      // S
  int compat;               // 0: reference (zero visit counts), 1: fixed
  int variant;              // 0: self_play.py MCTS, 1: main.py MCTS (main.py:246-368)
  int factored;             // 1: factored dynamics expansion (mzgo_expand.hpp), 0: a conv per simulation
  uint64_t seed;
  int helpers;              // helper workgroups sharing the batch expansions (GLOBAL_Y boards; 0: none)
  int net;                  // k_selfplay_move: the network of this move (arena: 1 = np_b), for the helpers
  int tail;                 // 9x9 whole-game launches: a workgroup whose game has ended helps running
                            // games with their parent convs (tail_help; 0: off)
  int lazy_rows;            // Y-streaming boards (19x19) without helpers: batched children keep the
                            // lazy policy head (kLazyRow, as the shared batches do); 0: eager rows
                            // (mzgo_search, whose trees are exported whole)
};

// One game's tree (global memory).  Node 0 is the root; node ids grow by one
// per expansion, so a search of S simulations uses at most S + 1 nodes.
struct TreeView {
  float* prior;       // [S+1][A] child priors of non-root nodes (f32)
  int* child;         // [S+1][A] child node id, -1 = unexpanded
  int* visits;        // [S+1]
  double* wsum;       // [S+1]  value_sum
  double* root_prior; // [A]    root child priors (f64)
  int* path;          // [S+2]
};

// child-row entry 0 of a node whose prior row still holds its policy logits
// (the tower engine's HBM trees, k_texpand; select_leaf settles it)
constexpr int kRawRow = -2;
// child-row entry 0 of a batched child whose policy head was never computed
// (the main engine's HBM trees: expand_child<LAZYH>, lazy policy head); its
// prior row holds nothing until a select first reaches it
constexpr int kLazyRow = -3;
// select_leaf's result when its walk reached such a node (t.leaf) whose
// policy sums are not in t.logits yet: the caller forms them (policy_sums_wg
// from t.lpar's Y and E[t.lact]) and resumes the walk at t.leaf
constexpr int kNeedLogits = -4;

// Per-game LDS block used by the tree phases.
template <class G>
struct TreeLds {
  float logits[G::A];
  float fbuf[G::A];
  double dbuf[G::A];
  uint8_t valid[G::A];     // valid_board (INVD == 0) for a < CELLS, 1 for pass
  double pass_prior;       // 0.01 or 1.0
  float reward, value;
  int leaf, action, nid, depth, nodes, bcast;
  int yready;              // select's leaf already has a child (its conv Y exists: factored mode)
  int npick;               // batch actions published so far (pick_sequence -> batch_expand)
  int ngrab;               // batch children claimed by the expanding waves so far
  int nunexp;              // select's leaf: number of unexpanded eligible children
  uint64_t umask[G::AP];   //   and their bitmask (a = 64 j + bit), the chosen one included
  int ycache;              // node whose Y the LDS copy holds (factored mode), -1: none
  int lognode;             // node whose policy sums (no bias) logits[0..CELLS) holds (lazy head), -1: none
  int lpar, lact;          // kNeedLogits: the parent and action of node t.leaf
  float hsc[56];                   // staged HeadScalars (HS_* offsets, HS_COUNT of them)
  // LDS-resident tree state (boards with G::TREE_CAP > 0 and S + 2 <= TREE_CAP)
  int svis[G::TREE_CAP > 0 ? G::TREE_CAP : 1];
  double sws[G::TREE_CAP > 0 ? G::TREE_CAP : 1];
  int spath[G::TREE_CAP > 0 ? G::TREE_CAP : 1];
  int rchild[G::TREE_CAP > 0 ? G::A : 1];
  double rprior[G::TREE_CAP > 0 ? G::A : 1];
  // visit counts / value sums of the root's children, indexed by action (a
  // mirror of svis / sws of node rchild[a]: the root's PUCT reads them in the
  // same round trip as its priors, without a dependent gather)
  int rvis[G::TREE_CAP > 0 ? G::A : 1];
  double rws[G::TREE_CAP > 0 ? G::A : 1];
  int ract;                // root action on the current simulation's path
  // LDS copy of one non-root node's prior row and child row (the leaf of a
  // speculative batch, whose child row the batch's replay keeps updating)
  int rowc_node;           // -1: none
  int rowc_child[G::TREE_CAP > 0 ? G::A : 1];
  float rowc_prior[G::TREE_CAP > 0 ? G::A : 1];
  // priors of the newest node, written by wave 1 while wave 0 backs up and
  // selects the next leaf; select waits on newp_node only if it reaches it
  float newp[G::A];
  int newest;              // id of the newest node (-1: none)
  int newp_node;           // node whose priors newp holds (atomic, workgroup scope)
  // batched children whose policy head was never computed (LDS trees, lazy
  // policy head: their prior rows are formed when a select first reaches the
  // node -- most children never are; see batch_expand)
  uint32_t rawp[G::TREE_CAP > 0 ? (G::TREE_CAP + 31) / 32 : 1];
  __device__ __forceinline__ bool is_raw(int n) const {
    if constexpr (G::TREE_CAP > 0) return n < G::TREE_CAP && ((rawp[n >> 5] >> (n & 31)) & 1u);
    else return false;
  }
};

// Tree accessor: node stats, path and the root's child row / priors either in
// LDS (L: small boards, S + 2 <= TREE_CAP; copied back to HBM by tree_flush)
// or in HBM.  Child rows / priors of non-root nodes always live in HBM.  The
// choice is a template parameter so every access compiles to ds_* or
// global_* (a runtime pointer choice would make them flat_* accesses).
template <class G, bool L>
struct TreeAcc {
  static_assert(!L || G::TREE_CAP > 0, "LDS tree needs TREE_CAP");
  static constexpr bool LDS = L;
  TreeView T;
  TreeLds<G>& t;
  __device__ __forceinline__ TreeAcc(const TreeView& tv, TreeLds<G>& tl) : T(tv), t(tl) {}
  __device__ __forceinline__ int vis(int n) const { if constexpr (L) return t.svis[n]; else return T.visits[n]; }
  __device__ __forceinline__ double ws(int n) const { if constexpr (L) return t.sws[n]; else return T.wsum[n]; }
  __device__ __forceinline__ void add(int n, double dv) {
    if constexpr (L) { t.svis[n] += 1; t.sws[n] = t.sws[n] + dv; }
    else { T.visits[n] += 1; T.wsum[n] = T.wsum[n] + dv; }
  }
  __device__ __forceinline__ void init(int n) {
    if constexpr (L) { t.svis[n] = 0; t.sws[n] = 0.0; } else { T.visits[n] = 0; T.wsum[n] = 0.0; }
  }
  __device__ __forceinline__ void set(int n, int vis, double ws) {
    if constexpr (L) { t.svis[n] = vis; t.sws[n] = ws; } else { T.visits[n] = vis; T.wsum[n] = ws; }
  }
  __device__ __forceinline__ int path(int i) const { if constexpr (L) return t.spath[i]; else return T.path[i]; }
  __device__ __forceinline__ void set_path(int i, int n) { if constexpr (L) t.spath[i] = n; else T.path[i] = n; }
  __device__ __forceinline__ int child(int n, int a) const {
    if constexpr (L) { if (n == 0) return t.rchild[a]; }
    return T.child[(size_t)n * G::A + a];
  }
  __device__ __forceinline__ void set_child(int n, int a, int c) {
    T.child[(size_t)n * G::A + a] = c;
    if constexpr (L) {
      if (n == 0) { t.rchild[a] = c; t.rvis[a] = 0; t.rws[a] = 0.0; }
      else if (n == t.rowc_node) t.rowc_child[a] = c;
    }
  }
  // the root-child mirror: stats of the root's child a (LDS trees)
  __device__ __forceinline__ void add_root_child(int a, double dv) {
    if constexpr (L) { t.rvis[a] += 1; t.rws[a] = t.rws[a] + dv; }
  }
  __device__ __forceinline__ double root_prior(int a) const {
    if constexpr (L) return t.rprior[a]; else return T.root_prior[a];
  }
};

template <class G>
__device__ __forceinline__ double mask_of(const TreeLds<G>& t, int a) {
  return a < G::CELLS ? (t.valid[a] ? 1.0 : 0.0) : t.pass_prior;
}

// valid_mask from the INVD plane (self_play.py:152-158); call with all threads
template <class G, class InvdFn>
__device__ __forceinline__ void build_mask(TreeLds<G>& t, double pass_epsilon, InvdFn invd) {
  int any = 0;
  for (int a = tid_local(); a < G::A; a += G::THREADS) {
    uint8_t v = a < G::CELLS ? (invd(a) == 0 ? 1 : 0) : 1;
    t.valid[a] = v;
    any |= (a < G::CELLS) && v;
  }
  any = __syncthreads_or(any);
  if (tid_local() == 0) t.pass_prior = any ? pass_epsilon : 1.0;
  __syncthreads();
}

// softmax of a lane's logits x[j] (a = lane + 64*j; entries a >= A ignored)
// -> p[j], torch CPU order: exp(x - max) * (1/sum), the per-lane partial sums
// taken in ascending j, then the wave butterfly.  Wave-level, registers only.
template <class G>
__device__ __forceinline__ void softmax_regs(const float (&x)[G::AP], float (&p)[G::AP]) {
  const int lane = lane_id_local();
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < G::AP; ++j)
    if (lane + 64 * j < G::A) m = fmax_(m, x[j]);
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    p[j] = lane + 64 * j < G::A ? expf(x[j] - m) : 0.f;
    s += p[j];
  }
  s = wave_sum(s);
  const float inv = 1.0f / s;
#pragma unroll
  for (int j = 0; j < G::AP; ++j) p[j] = p[j] * inv;
}

// softmax over t.logits -> t.fbuf.  Wave 0 only.
template <class G>
__device__ __forceinline__ void softmax_wave(TreeLds<G>& t) {
  const int lane = lane_id_local();
  float x[G::AP], p[G::AP];
#pragma unroll
  for (int j = 0; j < G::AP; ++j) x[j] = lane + 64 * j < G::A ? t.logits[lane + 64 * j] : 0.f;
  softmax_regs<G>(x, p);
#pragma unroll
  for (int j = 0; j < G::AP; ++j)
    if (lane + 64 * j < G::A) t.fbuf[lane + 64 * j] = p[j];
}

// Reward / value / logits from the fused head partials (self_play.py:91-94,
// :105-112).  hp: [2][3][CS]; heads h0 (reward if has_reward), then value,
// then policy.  hw: small head parameters (see HeadScalars).  Wave 0 only.
struct HeadScalars {
  const float* reward_b;    // [1]  reward_conv.bias
  const float* fc1_w;       // [16] fc_reward_hidden.weight
  const float* fc1_b;       // [16]
  const float* fc2_w;       // [16] fc_reward_output.weight
  const float* fc2_b;       // [1]
  const float* value_b;     // [1]  value_conv.bias
  const float* vfc_w;       // [1]  value_fc.weight
  const float* vfc_b;       // [1]
  const float* policy_b;    // [1]  policy_conv.bias
  const float* pass_logit;  // [1]
};

// HeadScalars staged in LDS (one load round per kernel instead of one per
// simulation): offsets into TreeLds::hsc.
enum : int { HS_RB = 0, HS_FC1W = 1, HS_FC1B = 17, HS_FC2W = 33, HS_FC2B = 49, HS_VB = 50, HS_VFCW = 51,
             HS_VFCB = 52, HS_PB = 53, HS_PASS = 54, HS_COUNT = 55 };
static_assert(HS_COUNT <= 56, "TreeLds::hsc holds the staged head scalars");

// All threads; visible after the caller's next barrier.
__device__ __forceinline__ void stage_head_scalars(const HeadScalars& hs, float* dst) {
  const int i = tid_local();
  if (i >= HS_COUNT) return;
  const float* src;
  if (i == HS_RB) src = hs.reward_b;
  else if (i < HS_FC1B) src = hs.fc1_w + (i - HS_FC1W);
  else if (i < HS_FC2W) src = hs.fc1_b + (i - HS_FC1B);
  else if (i < HS_FC2B) src = hs.fc2_w + (i - HS_FC2W);
  else if (i == HS_FC2B) src = hs.fc2_b;
  else if (i == HS_VB) src = hs.value_b;
  else if (i == HS_VFCW) src = hs.vfc_w;
  else if (i == HS_VFCB) src = hs.vfc_b;
  else if (i == HS_PB) src = hs.policy_b;
  else src = hs.pass_logit;
  dst[i] = *src;
}

// hp: [NPART][3][CS] partial sums over cout groups, added in a fixed order
template <class G, int NPART>
__device__ __forceinline__ float head_at(const float* hp, int h, int c) {
  float s = hp[h * G::CS + c];
#pragma unroll
  for (int p = 1; p < NPART; ++p) s += hp[(p * 3 + h) * G::CS + c];
  return s;
}

// value (and reward) heads; returns them on every lane.  One wave.
template <class G, int NPART>
__device__ __forceinline__ void heads_value(const float* hp, bool has_reward, const float* hsc, float& reward,
                                            float& value) {
  const int lane = lane_id_local();
  const int hv = has_reward ? 1 : 0;
  const float vb = hsc[HS_VB];
  float vs = 0.f, rs = 0.f;
  const float rb = has_reward ? hsc[HS_RB] : 0.f;
  constexpr int CP = (G::CELLS + 63) / 64;
#pragma unroll
  for (int j = 0; j < CP; ++j) {                  // cells c = lane + 64 j, ascending per lane
    const int c = lane + 64 * j;
    if (c < G::CELLS) {
      vs += head_at<G, NPART>(hp, hv, c) + vb;
      if (has_reward) rs += head_at<G, NPART>(hp, 0, c) + rb;
    }
  }
  vs = wave_sum(vs);
  const float vmean = vs / (float)G::CELLS;
  value = vmean * hsc[HS_VFCW] + hsc[HS_VFCB];
  reward = 0.f;
  if (has_reward) {
    rs = wave_sum(rs);
    const float rmean = rs / (float)G::CELLS;
    float h = 0.f;
    if (lane < 16) {
      h = rmean * hsc[HS_FC1W + lane] + hsc[HS_FC1B + lane];
      h = h > 0.f ? h : 0.f;
      h = h * hsc[HS_FC2W + lane];
    }
    h = wave_sum(h);
    reward = h + hsc[HS_FC2B];
  }
}

// value and reward heads (self_play.py:91-94, :105-110) from the totals over
// cells and channels of their 1x1 convs without biases (expand_wave):
// mean = total / CELLS + bias.  Every lane.
template <class G>
__device__ __forceinline__ void heads_from_totals(float rsum, float vsum, const float* hsc, float& reward,
                                                  float& value) {
  const float vmean = vsum / (float)G::CELLS + hsc[HS_VB];
  value = vmean * hsc[HS_VFCW] + hsc[HS_VFCB];
  const float rmean = rsum / (float)G::CELLS + hsc[HS_RB];
  const int lane = lane_id_local();
  float h = 0.f;
  if (lane < 16) {
    h = rmean * hsc[HS_FC1W + lane] + hsc[HS_FC1B + lane];
    h = h > 0.f ? h : 0.f;
    h = h * hsc[HS_FC2W + lane];
  }
  h = wave_sum(h);
  reward = h + hsc[HS_FC2B];
}

// policy logits of a lane's actions a = lane + 64 j (cells, then the learned
// pass logit), in registers.  One wave.
template <class G, int NPART>
__device__ __forceinline__ void logits_regs(const float* hp, bool has_reward, const float* hsc, float (&x)[G::AP]) {
  const int lane = lane_id_local();
  const int hpol = has_reward ? 2 : 1;
  const float pb = hsc[HS_PB];
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    x[j] = a < G::CELLS ? head_at<G, NPART>(hp, hpol, a) + pb : hsc[HS_PASS];
  }
}

// policy logits from one row of policy 1x1-conv sums (no bias) per cell: a
// lane's actions a = lane + 64 j (cells, then the learned pass logit).  One
// wave.
template <class G>
__device__ __forceinline__ void policy_logits(const float* row, const float* hsc, float (&x)[G::AP]) {
  const int lane = lane_id_local();
  const float pb = hsc[HS_PB];
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    x[j] = a < G::CELLS ? row[a] + pb : hsc[HS_PASS];
  }
}

// policy logits -> logits[A] (LDS).  One wave.
template <class G, int NPART>
__device__ __forceinline__ void heads_logits(const float* hp, bool has_reward, const float* hsc, float* logits) {
  const int lane = lane_id_local();
  float x[G::AP];
  logits_regs<G, NPART>(hp, has_reward, hsc, x);
#pragma unroll
  for (int j = 0; j < G::AP; ++j)
    if (lane + 64 * j < G::A) logits[lane + 64 * j] = x[j];
}

template <class G, int NPART>
__device__ __forceinline__ void finalize_heads(const float* hp, bool has_reward, const float* hsc,
                                      float* logits, float* reward, float* value) {
  float r, v;
  heads_value<G, NPART>(hp, has_reward, hsc, r, v);
  heads_logits<G, NPART>(hp, has_reward, hsc, logits);
  if (lane_id_local() == 0) { *value = v; *reward = r; }
}

// Child priors of a new node (self_play.py:204-224) from its logits x (a =
// lane + 64 j): p = softmax * root mask, normalised by numpy's f32 pairwise
// sum; entries with mask 0 are 0.  Written to dst (HBM row) and, for a node
// >= 0, published in t.newp for a select running concurrently on another
// wave.  One wave; values stay in registers except for the ordered sum.
// fbuf / dbuf: this wave's LDS scratch for the ordered sums (A entries each).
template <class G>
__device__ __forceinline__ void child_prior_regs(const TreeLds<G>& t, const float (&x)[G::AP], float (&q)[G::AP],
                                                 int variant, float* fbuf, double* dbuf) {
  const int lane = lane_id_local();
  float p[G::AP];
  double m[G::AP];
  softmax_regs<G>(x, p);
#pragma unroll
  for (int j = 0; j < G::AP; ++j) m[j] = lane + 64 * j < G::A ? mask_of<G>(t, lane + 64 * j) : 0.0;
  if (variant == 1) {
    // main.py:299-309: softmax[a] where valid_mask[a] > 0, not renormalised
#pragma unroll
    for (int j = 0; j < G::AP; ++j) q[j] = m[j] > 0 ? p[j] : 0.f;
  } else {
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      p[j] = mul_f32_by_f64(p[j], m[j]);
      if (lane + 64 * j < G::A) fbuf[lane + 64 * j] = p[j];
    }
    const float s = np_pairwise_sum<float, G::A>(fbuf);
    if (s > 0.f) {
#pragma unroll
      for (int j = 0; j < G::AP; ++j) q[j] = m[j] > 0 ? p[j] / s : 0.f;
    } else {
      // fallback of :215 (uniform over the mask; the reference's f64 here is
      // stored as f32 -- unreachable unless every valid softmax entry underflows)
      wave_lds_sync();
#pragma unroll
      for (int j = 0; j < G::AP; ++j)
        if (lane + 64 * j < G::A) dbuf[lane + 64 * j] = m[j];
      const double ms = np_pairwise_sum<double, G::A>(dbuf);
#pragma unroll
      for (int j = 0; j < G::AP; ++j) q[j] = (float)(m[j] / ms);
    }
  }
}

template <class G>
__device__ __forceinline__ void child_priors(TreeLds<G>& t, const float (&x)[G::AP], float* __restrict__ dst,
                                             int node = -1, int variant = 0, float* fbuf = nullptr,
                                             double* dbuf = nullptr) {
  const int lane = lane_id_local();
  if (!fbuf) { fbuf = t.fbuf; dbuf = t.dbuf; }
  float q[G::AP];
  child_prior_regs<G>(t, x, q, variant, fbuf, dbuf);
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    if (a < G::A) {
      dst[a] = q[j];
      if (node >= 0) t.newp[a] = q[j];
    }
  }
  // publish newp for a select running concurrently on another wave
  if (node >= 0 && lane == 0)
    __hip_atomic_store(&t.newp_node, node, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// A lazily expanded node's child priors from its policy sums in t.logits
// (policy_sums_wg): logits = sums + policy bias, pass logit last, then
// child_priors' operations -> its prior row (in place), -1s into its child
// row; q gets them too.  One wave; fbuf / dbuf: its LDS scratch.
template <class G>
__device__ __forceinline__ void settle_lazy(TreeLds<G>& t, float* row, int* crow, int variant, float* fbuf,
                                            double* dbuf, float (&q)[G::AP]) {
  const int lane = lane_id_local();
  float x[G::AP];
  policy_logits<G>(t.logits, t.hsc, x);
  child_prior_regs<G>(t, x, q, variant, fbuf, dbuf);
#pragma unroll
  for (int j = 0; j < G::AP; ++j)
    if (lane + 64 * j < G::A) { row[lane + 64 * j] = q[j]; crow[lane + 64 * j] = -1; }
}

// The root's Gamma draws a = lane + 64 (w - 1) on waves w = 1..AP (one per
// lane, in parallel, while wave 0 forms the softmax): dbuf[a], then *done += 1
// per wave.  Call from every wave.
template <class G>
__device__ __forceinline__ void draw_dirichlet(TreeLds<G>& t, uint64_t key, double alpha, int* done);

// Gamma(alpha) by Marsaglia-Tsang with the alpha+1 boost, from the counter
// stream (a << 16 | k).  Bounded: at most 64 proposals.
__device__ __forceinline__ double gamma_draw(uint64_t key, int a, double alpha) {
  uint32_t k = 0;
  auto U = [&]() { return u01(draw(key, TAG_DIRICHLET, ((uint64_t)a << 16) | (k++))); };
  const double boost = pow(1.0 - U(), 1.0 / alpha);  // U in (0,1]
  const double d = alpha + 1.0 - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  for (int it = 0; it < 64; ++it) {
    const double u1 = 1.0 - U(), u2 = U();
    const double x = sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
    double v = 1.0 + c * x;
    if (v <= 0.0) continue;
    v = v * v * v;
    const double u = 1.0 - U();
    if (log(u) < 0.5 * x * x + d - d * v + d * log(v)) return d * v * boost;
  }
  return d * boost;
}

template <class G>
__device__ __forceinline__ void draw_dirichlet(TreeLds<G>& t, uint64_t key, double alpha, int* done) {
  const int w = __builtin_amdgcn_readfirstlane(wave_id());
  if (w < 1 || w > G::AP) return;
  const int a = lane_id_local() + 64 * (w - 1);
  if (a < G::A) t.dbuf[a] = gamma_draw(key, a, alpha);
  wave_lds_sync();
  if (lane_id_local() == 0) __hip_atomic_fetch_add(done, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Root priors (self_play.py:151-182) into T.root_prior.  noise: injected
// Dirichlet sample [A] (nullable: sample from the counter stream); noise_out
// (test hook, nullable): the normalised sample used [A].  Wave 0.
template <class G>
__device__ __forceinline__ void root_priors(TreeLds<G>& t, const TreeView& T, const SearchParams& sp,
                                   const double* noise, uint64_t key, int* drawn = nullptr,
                                   double* noise_out = nullptr) {
  const int lane = lane_id_local();
  softmax_wave<G>(t);
  for (int a = lane; a < G::A; a += 64) t.fbuf[a] = mul_f32_by_f64(t.fbuf[a], mask_of<G>(t, a));
  const float s = np_pairwise_sum<float, G::A>(t.fbuf);
  // Dirichlet sample d[a] -> dbuf (f64)
  if (noise) {
    for (int a = lane; a < G::A; a += 64) t.dbuf[a] = noise[a];
  } else {
    if (drawn) {
      // the Gamma draws were made by other waves meanwhile (draw_dirichlet)
      while (__hip_atomic_load(drawn, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < G::AP)
        __builtin_amdgcn_s_sleep(2);
    } else {
      for (int a = lane; a < G::A; a += 64) t.dbuf[a] = gamma_draw(key, a, sp.dirichlet_alpha);
    }
    const double gs = np_pairwise_sum<double, G::A>(t.dbuf);
    for (int a = lane; a < G::A; a += 64) t.dbuf[a] = gs > 0 ? t.dbuf[a] / gs : 1.0 / G::A;
  }
  if (noise_out)
    for (int a = lane; a < G::A; a += 64) noise_out[a] = t.dbuf[a];
  const double eps = sp.dirichlet_epsilon;
  const float keep32 = (float)(1.0 - eps);   // Python float * f32 array -> f32 (NEP 50)
  if (sp.variant == 1) {
    // main.py:266-287: normalise only if the sum is positive, mix the noise,
    // keep p[a] where valid_mask[a] > 0 -- no re-mask, no renormalisation
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const int a = lane + 64 * j;
      if (a < G::A) {
        const float p = s > 0.f ? t.fbuf[a] / s : t.fbuf[a];
        const double q = (double)(keep32 * p) + eps * t.dbuf[a];
        const double pr = mask_of<G>(t, a) > 0 ? q : 0.0;
        T.root_prior[a] = pr;
        if (G::TREE_CAP > 0) t.rprior[a] = pr;
      }
    }
    return;
  }
  double q[G::AP];
  if (s > 0.f) {
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const int a = lane + 64 * j;
      if (a < G::A) {
        const float p = t.fbuf[a] / s;
        q[j] = (double)(keep32 * p) + eps * t.dbuf[a];
      }
    }
  } else {
    // uniform-over-mask fallback (:164) is float64, so the noise mix is too
    for (int a = lane; a < G::A; a += 64) t.fbuf[a] = 0.f;
    double tmp[G::AP];
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const int a = lane + 64 * j;
      tmp[j] = a < G::A ? mask_of<G>(t, a) : 0.0;
    }
    // sum of the mask in numpy order (reuse root_prior as scratch)
#pragma unroll
    for (int j = 0; j < G::AP; ++j) { const int a = lane + 64 * j; if (a < G::A) T.root_prior[a] = tmp[j]; }
    __threadfence_block();
    const double ms = np_pairwise_sum<double, G::A>(T.root_prior);
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const int a = lane + 64 * j;
      if (a < G::A) q[j] = (1.0 - eps) * (tmp[j] / ms) + eps * t.dbuf[a];
    }
  }
  // policy *= valid_mask; normalise by numpy's f64 sum (:169-174)
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    if (a < G::A) { q[j] = q[j] * mask_of<G>(t, a); t.dbuf[a] = q[j]; }
  }
  const double s2 = np_pairwise_sum<double, G::A>(t.dbuf);
  double ms = 0.0;
  if (!(s2 > 0.0)) {
    for (int a = lane; a < G::A; a += 64) t.dbuf[a] = mask_of<G>(t, a);
    ms = np_pairwise_sum<double, G::A>(t.dbuf);
  }
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const int a = lane + 64 * j;
    if (a < G::A) {
      const double m = mask_of<G>(t, a);
      const double p = s2 > 0.0 ? q[j] / s2 : m / ms;
      T.root_prior[a] = m > 0 ? p : 0.0;
      if (G::TREE_CAP > 0) t.rprior[a] = m > 0 ? p : 0.0;   // LDS mirror (used if the tree is in LDS)
    }
  }
}

// The choices of simulations sim0, sim0 + 1, ... (count of them) that each
// take an unexpanded eligible child of the same node: simulation sim0 + i
// picks the r_i-th (ascending) of the n - i still unexpanded ones (bitmask m),
// r_i = randbelow(draw(key, TAG_SELECT, sim0 + i), n - i) -- select_leaf's
// random.choice (self_play.py:283-287) replayed.  The draws are made in
// parallel (lane i = lane + 64 q); then, pick by pick, the remaining element
// of rank r_i is found in the remaining set's bitmask with scalar popcounts
// and removed.  out[i0 + i] (LDS) gets the actions; *progress (LDS, if given)
// is published after the first `head` picks and every 12 after.  Wave-level.
template <class G>
struct PickSeq {
  uint32_t r[G::AP];       // lane i = lane + 64 q: simulation i's rank among the remaining
  uint64_t rem[G::AP];     // the remaining elements (wave-uniform: scalar registers)
  __device__ __forceinline__ PickSeq() {}
  __device__ __forceinline__ PickSeq(const uint64_t (&m)[G::AP], int n, int count, uint64_t key, int sim0) {
    const int lane = lane_id_local();
#pragma unroll
    for (int q = 0; q < G::AP; ++q) {
      const int i = lane + 64 * q;
      r[q] = i < count ? randbelow(draw(key, TAG_SELECT, (uint64_t)(sim0 + i)), (uint32_t)(n - i)) : 0u;
    }
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)m[j]);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(m[j] >> 32));
      rem[j] = ((uint64_t)hi << 32) | lo;
    }
  }
  // pick i (in order i = 0, 1, ...): the remaining element of rank r_i: the
  // word from the words' prefix popcounts (scalar, no branches), the bit by a
  // ballot of the lanes' mbcnt ranks inside it
  __device__ __forceinline__ int pick(int i) {
    uint32_t k = 0;
#pragma unroll
    for (int q = 0; q < G::AP; ++q)
      if ((i >> 6) == q) k = (uint32_t)__builtin_amdgcn_readlane((int)r[q], i & 63);
    uint32_t pre = 0, w = 0, base = 0;
#pragma unroll
    for (int j = 0; j < G::AP - 1; ++j) {
      pre += (uint32_t)__builtin_popcountll(rem[j]);
      const bool past = k >= pre;                    // rank k lies beyond word j
      w += past ? 1u : 0u;
      base = past ? pre : base;
    }
    k -= base;
    uint64_t x = rem[0];
#pragma unroll
    for (int j = 1; j < G::AP; ++j) x = w == (uint32_t)j ? rem[j] : x;
    // the k-th set bit of x: the lane holding a set bit with k set bits below it
    const uint32_t lane = (uint32_t)lane_id_local();
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(x >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)x, 0u));
    const uint32_t pos = (uint32_t)__builtin_ctzll(__ballot(((x >> lane) & 1ull) && below == k));
#pragma unroll
    for (int j = 0; j < G::AP; ++j) rem[j] &= w == (uint32_t)j ? ~(1ull << pos) : ~0ull;
    return (int)(64 * w + pos);
  }

};

// gout (HBM, optional): every action also goes to gout[i0 + i] as gtag << 32
// | action (an agent-scope relaxed store, never waited for), for other
// workgroups (batch_expand_shared: the tag tells them the entry is current).
template <class G>
__device__ __forceinline__ void pick_sequence(const uint64_t (&m)[G::AP], int n, int i0, int count, uint64_t key,
                                              int sim0, int* out, int* progress = nullptr, int head = 1,
                                              Stamp* st = nullptr, unsigned long long* gout = nullptr,
                                              unsigned gtag = 0) {
  const int lane = lane_id_local();
  const unsigned long long t0 = st ? st->now() : 0;
  PickSeq<G> ps(m, n, count, key, sim0);
  const unsigned long long t1 = st ? st->now() : 0;
  if (st) st->wave_add(66, t1 - t0);
  int next_pub = head < count ? head : count;
  for (int i = 0; i < count; ++i) {
    const int a = ps.pick(i);
    if (lane == 0) {
      out[i0 + i] = a;
      if (gout)
        __hip_atomic_store(gout + i0 + i, (unsigned long long)gtag << 32 | (unsigned)a, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
    if (progress && i + 1 == next_pub) {
      wave_lds_sync();
      if (lane == 0) __hip_atomic_store(progress, i0 + i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      next_pub = next_pub + 12 < count ? next_pub + 12 : count;
    }
  }
  if (st) st->wave_add(67, st->now() - t1);
}

// pick_sequence's choices, all at once.  Pick i takes the element of rank r_i
// among the n - i still remaining; in ranks of the original n elements that
// is p_i = r_i lifted past every earlier pick: with q_i = r_i to start, for i
// = count-2 down to 0, q_j += (q_j >= r_i) for every j > i leaves q_j = p_j
// (step i maps ranks in the set without p_0..p_i to ranks in the set without
// p_0..p_(i-1); r_i itself is p_i in those coordinates, and no step touches
// q_i before step i -- the Lehmer code decoded backwards).  Lane j owns q_j:
// count steps of a compare-and-add instead of count dependent scalar
// searches.  p -> action through an LDS rank table built in out[i0 ..] (n <=
// A - i0 entries), read back before the actions overwrite it.
template <class G, int NG>
__device__ __forceinline__ void lehmer_lift(uint32_t (&v)[G::AP], const uint32_t (&r)[G::AP], int count) {
  const int lane = lane_id_local();
#pragma unroll
  for (int gi = NG - 1; gi >= 0; --gi) {
    const int top = min(count - 2, 64 * gi + 63);
    for (int i = top; i >= 64 * gi; --i) {
      const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)r[gi], i - 64 * gi);
      v[gi] += (lane > i - 64 * gi && v[gi] >= s) ? 1u : 0u;
#pragma unroll
      for (int q = gi + 1; q < NG; ++q) v[q] += v[q] >= s ? 1u : 0u;
    }
  }
}

template <class G>
__device__ __forceinline__ void pick_all(const uint64_t (&m)[G::AP], int n, int i0, int count, uint64_t key,
                                         int sim0, int* out, Stamp* st = nullptr,
                                         unsigned long long* gout = nullptr, unsigned gtag = 0) {
  if (count <= 0) return;
  const int lane = lane_id_local();
  const unsigned long long t0 = st ? st->now() : 0;
  PickSeq<G> ps(m, n, count, key, sim0);
  uint32_t v[G::AP];
#pragma unroll
  for (int q = 0; q < G::AP; ++q) v[q] = ps.r[q];
  const int ng = (count + 63) >> 6;
  switch (ng) {                                     // (only the groups holding picks)
#define MZGO_LIFT(K) case K: if constexpr (K <= G::AP) lehmer_lift<G, K>(v, ps.r, count); break;
    MZGO_LIFT(1) MZGO_LIFT(2) MZGO_LIFT(3) MZGO_LIFT(4) MZGO_LIFT(5) MZGO_LIFT(6)
#undef MZGO_LIFT
    default: break;
  }
  static_assert(G::AP <= 6, "lehmer_lift dispatch covers up to 6 lane groups");
  // rank table: the k-th remaining element (ascending) at tab[k]
  int* tab = out + i0;
  uint32_t pre = 0;
#pragma unroll
  for (int w = 0; w < G::AP; ++w) {
    const uint32_t lo = (uint32_t)ps.rem[w], hi = (uint32_t)(ps.rem[w] >> 32);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
    if ((ps.rem[w] >> lane) & 1ull) tab[pre + below] = 64 * w + lane;
    pre += (uint32_t)__builtin_popcountll(ps.rem[w]);
  }
  wave_lds_sync();
  int a[G::AP];
#pragma unroll
  for (int q = 0; q < G::AP; ++q) a[q] = (lane + 64 * q < count) ? tab[v[q]] : 0;
  wave_lds_sync();
#pragma unroll
  for (int q = 0; q < G::AP; ++q) {
    const int j = lane + 64 * q;
    if (j < count) {
      out[i0 + j] = a[q];
      if (gout)
        __hip_atomic_store(gout + i0 + j, (unsigned long long)gtag << 32 | (unsigned)a[q], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (st) st->wave_add(67, st->now() - t0);
}

// PUCT over the eligible, all expanded children elig (self_play.py:290-308;
// main.py:338-364): q = W/N min-max normalised over them, u = c_puct * P *
// sqrt(max(1, N_parent)) / (1 + n) (main.py: sqrt(N_parent + 1)); root priors
// f64, child priors f32 with an f32 c_puct * P (NEP 50); the first strict
// maximum in ascending action order.  Returns the action (-1: no finite
// score) and, in best_c, its child id.  Wave-level.
template <class G>
__device__ __forceinline__ int puct_pick(const double (&P)[G::AP], const int (&n)[G::AP], const double (&w)[G::AP],
                                         const uint64_t (&elig)[G::AP], const int (&ch)[G::AP], int nvis,
                                         bool root, const SearchParams& sp, int& best_c, Stamp* st = nullptr) {
  const int lane = lane_id_local();
  double q[G::AP];
  double lo = INFINITY, hi = -INFINITY;
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    q[j] = 0.0;
    if ((elig[j] >> lane) & 1ull) {
      q[j] = n[j] > 0 ? ddiv(w[j], (double)n[j]) : 0.0;
      lo = fmin_(lo, q[j]);
      hi = fmax_(hi, q[j]);
    }
  }
  if (st) st->lap(25);
  wave_minmax(lo, hi);
  if (st) st->lap(26);
  // sqrt(max(1, N)) (self_play.py:316) or sqrt(N + 1) (main.py:354)
  const double sq = dsqrt((double)(sp.variant == 1 ? nvis + 1 : (nvis > 1 ? nvis : 1)));
  double sc[G::AP];
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    sc[j] = -INFINITY;
    if ((elig[j] >> lane) & 1ull) {
      const double qn = hi > lo ? ddiv(q[j] - lo, hi - lo) : q[j];
      double u;
      if (root) u = ddiv((sp.c_puct * P[j]) * sq, (double)(1 + n[j]));
      else u = ddiv((double)((float)sp.c_puct * (float)P[j]) * sq, (double)(1 + n[j]));
      sc[j] = qn + u;
    }
  }
  if (st) st->lap(27);
  // the wave's maximum score, then the lowest action holding it
  double best_s = sc[0];
#pragma unroll
  for (int j = 1; j < G::AP; ++j) best_s = sc[j] > best_s ? sc[j] : best_s;
  best_s = wave_max(best_s);
  best_c = -1;
  if (!(best_s > -INFINITY)) return -1;
  int best_a = -1;
#pragma unroll
  for (int j = 0; j < G::AP; ++j) {
    const uint64_t hit = __ballot(sc[j] == best_s);
    if (best_a < 0 && hit) {
      const int l = __ffsll((long long)hit) - 1;
      best_a = 64 * j + l;
      best_c = __builtin_amdgcn_readlane(ch[j], l);
    }
  }
  return best_a;
}

// ---------------------------------------------------------------------------
// select_leaf (self_play.py:239-335).  Wave 0.  Returns the action to expand
// at t.leaf, or -1 when the walk ends at a terminal node (t.leaf).  The path
// (node ids, root first) is written to T.path[0..depth].
// ---------------------------------------------------------------------------
template <class G, class Acc>
__device__ __forceinline__ int select_leaf(TreeLds<G>& t, const Acc& T, const SearchParams& sp,
                                  uint64_t key, int sim, Stamp* st = nullptr, int node0 = 0, int depth0 = 0) {
  const int lane = lane_id_local();
  // (node0, depth0): resume a walk that returned kNeedLogits at that node
  int node = node0, depth = depth0, par = -1, pact = -1;
  if (st) { st->lap(35); st->wave_add(51, 1); }
#ifdef MZGO_STAMPS
  // (stamps builds: the wave's outstanding vector-memory operations -- its
  // HBM stores -- drained here, so slot 38 is their ack wait and the levels'
  // slots below hold their loads alone)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (st) st->lap(38);
#endif
  // a lazily expanded node reached for the first time: its policy sums
  // first (the caller), unless t.logits holds them already
  auto need_logits = [&]() {
    t.leaf = node; t.depth = depth; t.lpar = par; t.lact = pact;
    return kNeedLogits;
  };
  for (int guard = 0; guard <= sp.num_simulations + 1; ++guard) {
    const bool root = node == 0;
    const int nvis = T.vis(node);
    const float* pr_row = T.T.prior + (size_t)node * G::A;
    // the newest node's priors may still be in the making (wave 1)
    const bool fresh = !root && node == t.newest;
    if (fresh) {
      if (st) st->lap(36);
      while (__hip_atomic_load(&t.newp_node, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != node)
        __builtin_amdgcn_s_sleep(1);
      if (st) st->lap(39);
    }
    double P[G::AP], rw[G::AP];
    int ch[G::AP], rn[G::AP];
    // all of this node's loads first (one round trip); three sources, chosen
    // by wave-uniform branches (a select between an LDS and a global pointer
    // would compile to a flat load).  A fresh node has no children yet.
    if (root) {
      asm volatile("" ::: "memory");          // keep the LDS and HBM loads apart (no flat merge)
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane + 64 * j;
        P[j] = a < G::A ? T.root_prior(a) : 0.0;
        ch[j] = a < G::A ? T.child(0, a) : -1;
        if constexpr (Acc::LDS) {
          rn[j] = a < G::A ? t.rvis[a] : 0;
          rw[j] = a < G::A ? t.rws[a] : 0.0;
        }
      }
    } else if (fresh) {
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane + 64 * j;
        P[j] = a < G::A ? (double)t.newp[a] : 0.0;
        ch[j] = -1;
      }
    } else if (Acc::LDS && node == t.rowc_node) {
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane + 64 * j;
        P[j] = a < G::A ? (double)t.rowc_prior[a] : 0.0;
        ch[j] = a < G::A ? t.rowc_child[a] : -1;
      }
    } else if (t.is_raw(node)) {               // first arrival at a lazily expanded node
      if (t.lognode != node) return need_logits();
      // t.fbuf / t.dbuf are wave 1's while it forms the newest node's priors
      if (t.newest >= 0)
        while (__hip_atomic_load(&t.newp_node, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != t.newest)
          __builtin_amdgcn_s_sleep(1);
      float q[G::AP];
      if (st) st->lap(36);
      settle_lazy<G>(t, const_cast<float*>(pr_row), T.T.child + (size_t)node * G::A, sp.variant, t.fbuf, t.dbuf, q);
      if (lane == 0) atomicAnd(&t.rawp[node >> 5], ~(1u << (node & 31)));
      if (st) { st->lap(49); st->wave_add(50, 1); }
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane + 64 * j;
        P[j] = a < G::A ? (double)q[j] : 0.0;
        ch[j] = -1;
      }
    } else {
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const int a = lane + 64 * j;
        P[j] = a < G::A ? (double)pr_row[a] : 0.0;
        ch[j] = a < G::A ? T.T.child[(size_t)node * G::A + a] : -1;
      }
      if constexpr (!Acc::LDS) {
        // first arrival at a lazily expanded node (HBM trees): its policy
        // sums (kLazyRow) or the logits its row holds (kRawRow, the tower
        // engine) -> priors in place, its child row -> -1s
        const int c0 = __builtin_amdgcn_readfirstlane(ch[0]);
        if (c0 == kLazyRow) {
          if (t.lognode != node) return need_logits();
          if (t.newest >= 0)                      // t.fbuf / t.dbuf: wave 1's while it forms newp
            while (__hip_atomic_load(&t.newp_node, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != t.newest)
              __builtin_amdgcn_s_sleep(1);
          float q[G::AP];
          settle_lazy<G>(t, const_cast<float*>(pr_row), T.T.child + (size_t)node * G::A, sp.variant, t.fbuf,
                         t.dbuf, q);
#pragma unroll
          for (int j = 0; j < G::AP; ++j) {
            const int a = lane + 64 * j;
            P[j] = a < G::A ? (double)q[j] : 0.0;
            ch[j] = -1;
          }
        } else if (c0 == kRawRow) {
          if (t.newest >= 0)                      // t.fbuf / t.dbuf: wave 1's while it forms newp
            while (__hip_atomic_load(&t.newp_node, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != t.newest)
              __builtin_amdgcn_s_sleep(1);
          float x[G::AP], q[G::AP];
#pragma unroll
          for (int j = 0; j < G::AP; ++j) x[j] = (float)P[j];
          child_prior_regs<G>(t, x, q, sp.variant, t.fbuf, t.dbuf);
          float* prow = const_cast<float*>(pr_row);
          int* crow = T.T.child + (size_t)node * G::A;
#pragma unroll
          for (int j = 0; j < G::AP; ++j) {
            const int a = lane + 64 * j;
            if (a < G::A) { prow[a] = q[j]; crow[a] = -1; }
            P[j] = a < G::A ? (double)q[j] : 0.0;
            ch[j] = -1;
          }
        }
      }
    }
    // eligible = valid_mask[a] > 0 and prior > 0 (:255-264); every prior is 0
    // where the root mask is (root_priors, child_priors), so prior > 0 decides
    uint64_t anypos = 0, anych = 0, elig[G::AP], unexp[G::AP];
    int n_unexp = 0;
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      const bool pos = P[j] > 0.0;
      anypos |= __ballot(pos);
      anych |= __ballot(ch[j] >= 0);
      elig[j] = __ballot(pos);
      unexp[j] = __ballot(pos && ch[j] < 0);
      n_unexp += __popcll(unexp[j]);
    }
    uint64_t any_elig = 0;
#pragma unroll
    for (int j = 0; j < G::AP; ++j) any_elig |= elig[j];
    if (st) st->lap(root ? 24 : 36);
    if (sp.variant == 1) {
      // main.py:318-364 has no terminal test; with no positive-prior child the
      // walk ends without an action and the simulation does nothing (:296)
      if (!any_elig) { t.leaf = node; t.depth = depth; return -2; }
    } else if ((nvis > 0 && !anypos) || !any_elig) {
      t.leaf = node; t.depth = depth; return -1;
    }

    if (n_unexp > 0) {
      // random.choice over the ascending list of unexpanded eligible actions
      uint32_t k = randbelow(draw(key, TAG_SELECT, (uint64_t)sim), (uint32_t)n_unexp);
      int best = -1;
#pragma unroll
      for (int j = 0; j < G::AP; ++j) {
        const uint32_t c = __popcll(unexp[j]);
        if (best < 0 && k < c) {
          best = 64 * j + kth_set_bit(unexp[j], k);
        } else if (best < 0) {
          k -= c;
        }
      }
      t.leaf = node;
      t.depth = depth;
      t.yready = anych != 0 ? 1 : 0;
      t.nunexp = n_unexp;
#pragma unroll
      for (int j = 0; j < G::AP; ++j) t.umask[j] = unexp[j];
      if (root) t.ract = best;
      if (st) st->lap(37);
      return best;
    }

    // PUCT over the (all expanded) eligible children
    int n[G::AP];
    double w[G::AP];
#pragma unroll
    for (int j = 0; j < G::AP; ++j) {
      n[j] = 0;
      w[j] = 0.0;
      if ((elig[j] >> lane) & 1ull) {
        if (Acc::LDS && root) { n[j] = rn[j]; w[j] = rw[j]; }     // root-child mirror (no gather)
        else { n[j] = T.vis(ch[j]); w[j] = T.ws(ch[j]); }
      }
    }
    int best_c = -1;
    const int best_a = puct_pick<G>(P, n, w, elig, ch, nvis, root, sp, best_c, root ? st : nullptr);
    if (best_a < 0) { t.leaf = node; t.depth = depth; return sp.variant == 1 ? -2 : -1; }
    if (root) t.ract = best_a;
    depth += 1;
    if (lane == 0) const_cast<Acc&>(T).set_path(depth, best_c);
    par = node;
    pact = best_a;
    node = best_c;
    if (st) {
      st->lap(depth == 1 ? 22 : 23);
      if (depth >= 2) st->wave_add(91, 1);
    }
  }
  t.leaf = node;
  t.depth = depth;
  return -1;
}

// Backup along path[0..depth] (+ the new node nid if >= 0): leaf-most gets
// +v, alternating sign upward (self_play.py:337-343).  Wave 0; path nodes are
// distinct, so each lane updates its own node.  Path entry 0 is the root.
template <class G, class Acc>
__device__ __forceinline__ void backup(Acc& T, int depth, int nid, double v, bool alternate = true) {
  const int lane = lane_id_local();
  const int off = nid >= 0 ? 1 : 0;
  const int count = depth + 1 + off;              // nodes on the backed-up path
  const int ract = T.t.ract;
  for (int i = lane; i < count; i += 64) {
    const int node = (off && i == 0) ? nid : T.path(depth - (i - off));
    // self_play.py:337-343 alternates the sign; main.py:366-368 does not
    const double dv = (alternate && (i & 1)) ? -v : v;
    T.add(node, dv);
    if (i == count - 2) T.add_root_child(ract, dv);   // the path's depth-1 node, by its root action
  }
  wave_lds_sync();
}

// Reset a tree to a bare root (children unexpanded, stats zero).  All threads.
template <class G, class Acc>
__device__ __forceinline__ void tree_reset_root(Acc& T) {
  for (int a = tid_local(); a < G::A; a += G::THREADS) T.set_child(0, a, -1);
  if constexpr (G::TREE_CAP > 0)
    for (int i = tid_local(); i < (G::TREE_CAP + 31) / 32; i += G::THREADS) T.t.rawp[i] = 0u;
  if (tid_local() == 0) { T.init(0); T.set_path(0, 0); }
}

// Write LDS-resident stats of nodes [0, nodes) back to HBM.  All threads.
template <class G, class Acc>
__device__ __forceinline__ void tree_flush(Acc& T, int nodes) {
  if constexpr (Acc::LDS) {
    for (int n = tid_local(); n < nodes; n += G::THREADS) {
      T.T.visits[n] = T.t.svis[n];
      T.T.wsum[n] = T.t.sws[n];
    }
  }
}

}  // namespace mzgo

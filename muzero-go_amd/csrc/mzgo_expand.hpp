// mzgo_expand.hpp -- the factored dynamics expansion.
//
// DynamicsNetwork.forward (self_play.py:85-95) computes, for a leaf latent x
// and action a,   relu(conv3x3(x + emb[a] (broadcast over cells)) + b).
// The convolution is linear and zero-padded, so
//     conv3x3(x + emb[a]) + b  =  Y_x + E[a][region(cell)]
// with Y_x = conv3x3(x) + b (one conv per distinct LEAF, not per child) and
//     E[a][r][co] = sum over the taps (ky, kx) that stay on the board for a
//                   cell of region r of  sum_ci W[co][ci][ky][kx] * emb[a][ci]
// where r = (row class)*3 + (column class), classes {first, interior, last}.
// E is a per-network table [A][9][C] built once on the host in f64
// (mzgo_capi.hip: action_taps).
//
// A search therefore runs the full 3x3 conv only for nodes that become
// parents (3-11 per 200-400-simulation search in the reference's trees; the
// unexpanded-first rule, self_play.py:283-287, makes trees wide and shallow),
// and every expansion is an elementwise pass over Y_leaf:
//     child latent = relu(Y_leaf + E[a])            (never stored: rebuilt by
//                                                    materialize() if the child
//                                                    ever becomes a parent)
//     reward/value/policy 1x1 heads over it         (self_play.py:91-94, :105-112)
// Every output of recurrent_inference is still computed for every
// simulation; only the conv of a leaf is shared by its children.  The fp32
// sums differ from torch's by rounding only (emb is added after the conv
// rather than before), like the Winograd conv.
//
// Y is stored cell-major, [CELLS][C] per node, so 8 lanes read one cell's
// channels as contiguous float4s.
#pragma once
#include "mzgo_common.hpp"

namespace mzgo {

template <class G>
struct ExpandShape {
  static constexpr int C4 = G::C / 4;         // float4 per cell
  static constexpr int LPC = 8;               // lanes per cell
  static constexpr int PERL = C4 / LPC;       // float4 per lane
  static constexpr int CPP = G::THREADS / LPC;   // cells per pass
  static constexpr int PASSES = (G::CELLS + CPP - 1) / CPP;
  static_assert(G::C % 32 == 0, "8 lanes x whole float4s per cell");
};

// LDS of the expansion (a member of the conv union, UF floats): the heads,
// and, if they fit, a copy of one node's Y and of the 1x1 head weights (so
// that consecutive expansions of the same leaf read them from LDS instead of
// L2; a conv overwrites the union and the next expansion refills it), and
// the per-wave buffers of the batches (batch_expand).  Boards whose Y does
// not fit (19x19) still batch, each wave streaming Y from L2 (GLOBAL_Y) with
// smaller per-wave buffers: the policy row only, E[a], and E's space reused
// as the ordered-sum scratch of child_priors.
template <class G, int UF>
struct ExpandLds {
  static constexpr int YC = G::CELLS * G::C;
  static constexpr int BASE = YC + 3 * G::CS + 3 * G::C;
  static constexpr bool CACHE = BASE <= UF;
  static constexpr int PERW = 3 * G::CS + 9 * G::C + 3 * 64 * G::AP;   // one wave's batch buffers
  static constexpr int PERW_G = G::CS + 18 * G::C;                     // ... with Y streamed from L2 (two E rows)
  static_assert(CACHE || 9 * G::C >= 2 * 64 * G::AP, "E's space holds child_priors' scratch (f32 then f64, in turn)");
  // tail arrays: bv (A+16 doubles = 2(A+16) floats) and acts (A ints)
  static constexpr int TAIL = 2 * (G::A + 16) + G::A + 64;
  static constexpr bool BATCH = CACHE ? BASE + G::WAVES * PERW + TAIL <= UF
                                      : 3 * G::CS + 3 * G::C + 8 * ((G::CELLS + 15) / 16) + G::WAVES * PERW_G + TAIL <= UF;
  static constexpr bool GLOBAL_Y = BATCH && !CACHE;
  static constexpr int XW = CACHE ? 3 * G::CS : G::CS;   // a wave's head rows; the policy row at PROW
  static constexpr int PROW = CACHE ? 2 * G::CS : 0;
  alignas(16) float yc[CACHE ? YC : 4];
  alignas(16) float hw[CACHE || BATCH ? 3 * G::C : 4];
  // (Y streamed from L2) expand_wave's E-row offsets of pass pairs (load_y):
  // lane group cg, passes 2pp / 2pp+1 -> rpair[pp*8 + cg], two 16-bit halves
  static constexpr int RPAIRS = 8 * ((G::CELLS + 15) / 16);
  uint32_t rpair[GLOBAL_Y ? RPAIRS : 1];
  float xh[3 * G::CS];
  struct Wave {
    alignas(16) float xw[XW];             // the child's policy sums per cell (at PROW)
    alignas(16) float ew[9 * G::C];       // E[a] of the child
    alignas(16) float ew2[CACHE ? 4 : 9 * G::C];   // (Y streamed from L2) E[a] of the pair's second child
    float fb[CACHE ? 64 * G::AP : 1];     // ordered-sum scratch (child_priors)
    double db[CACHE ? 64 * G::AP : 1];
    __device__ float* fscratch() { if constexpr (CACHE) return fb; else return ew; }
    __device__ double* dscratch() { if constexpr (CACHE) return db; else return reinterpret_cast<double*>(ew); }
  };
  Wave wv[BATCH ? G::WAVES : 1];          // (after the batch: verify_batch's arrays)
  double bv[BATCH ? G::A + 16 : 1];       // backup value of each batched child (+ tail read by prefix_sums)
  int acts[BATCH ? G::A : 1];             // action of each batched child
};

// board region class of a cell: (row class) * 3 + (column class)
template <class G>
__device__ __forceinline__ int region_of(int cell) {
  const int y = cell / G::N, x = cell - y * G::N;
  const int ry = y == 0 ? 0 : (y == G::N - 1 ? 2 : 1);
  const int rx = x == 0 ? 0 : (x == G::N - 1 ? 2 : 1);
  return ry * 3 + rx;
}

// 8-lane sum (lanes 8k .. 8k+7) via DPP: quad xor 1, xor 2, then half-row mirror
__device__ __forceinline__ float sum8(float v) {
  v = v + dpp::mov<dpp::XOR1>(v);
  v = v + dpp::mov<dpp::XOR2>(v);
  return v + dpp::mov<0x141>(v);              // row_half_mirror: lane i <-> 7 - i
}

// Child heads of expansion (leaf, a): L.xh [3][CS] gets, per cell, the
// reward, value and policy 1x1-conv sums (no biases) of relu(Y + E[a]).
// Y: the leaf's [CELLS][C] (global; read from the LDS copy L.yc when
// ``hit``, else copied into it); ea: E[a] [9][C]; hw [3][C] (global: reward,
// value, policy conv weights; L.hw is their LDS copy, valid with L.yc).  All
// threads; the caller synchronises before reading xh.
template <class G, class L>
__device__ __forceinline__ void expand_heads(L& lds, const float* __restrict__ Y, bool hit,
                                             const float* __restrict__ ea, const float* hw) {
  typedef ExpandShape<G> X;
  const f32x4* Y4 = reinterpret_cast<const f32x4*>(Y);
  const f32x4* E4 = reinterpret_cast<const f32x4*>(ea);
  const bool lw = L::CACHE && hit;
  const f32x4* W4 = reinterpret_cast<const f32x4*>(hw);
  f32x4* C4 = reinterpret_cast<f32x4*>(lds.yc);
  f32x4* CW = reinterpret_cast<f32x4*>(lds.hw);
  const int j = tid_local() & (X::LPC - 1);
#pragma unroll
  for (int pass = 0; pass < X::PASSES; ++pass) {
    const int cell = pass * X::CPP + tid_local() / X::LPC;
    const int cl = cell < G::CELLS ? cell : G::CELLS - 1;
    const int reg = region_of<G>(cl);
    f32x4 y[X::PERL], e[X::PERL];
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) {
      e[k] = E4[reg * X::C4 + j + X::LPC * k];
    }
    if (L::CACHE && hit) {
#pragma unroll
      for (int k = 0; k < X::PERL; ++k) y[k] = C4[(size_t)cl * X::C4 + j + X::LPC * k];
    } else {
#pragma unroll
      for (int k = 0; k < X::PERL; ++k) y[k] = Y4[(size_t)cl * X::C4 + j + X::LPC * k];
      if (L::CACHE && cell < G::CELLS) {
#pragma unroll
        for (int k = 0; k < X::PERL; ++k) C4[(size_t)cl * X::C4 + j + X::LPC * k] = y[k];
      }
    }
    float hr = 0.f, hv = 0.f, hp = 0.f;
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) {
      const int c4 = j + X::LPC * k;
      f32x4 wr, wv, wp;
      if (lw) {
        wr = CW[c4]; wv = CW[X::C4 + c4]; wp = CW[2 * X::C4 + c4];
      } else {
        wr = W4[c4]; wv = W4[X::C4 + c4]; wp = W4[2 * X::C4 + c4];
        if (L::CACHE && pass == 0 && tid_local() < X::LPC) {   // one writer per weight
          CW[c4] = wr; CW[X::C4 + c4] = wv; CW[2 * X::C4 + c4] = wp;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v = y[k][q] + e[k][q];
        v = v > 0.f ? v : 0.f;
        hr = __builtin_fmaf(wr[q], v, hr);
        hv = __builtin_fmaf(wv[q], v, hv);
        hp = __builtin_fmaf(wp[q], v, hp);
      }
    }
    hr = sum8(hr);
    hv = sum8(hv);
    hp = sum8(hp);
    if (j == 0 && cell < G::CELLS) {
      lds.xh[cell] = hr;
      lds.xh[G::CS + cell] = hv;
      lds.xh[2 * G::CS + cell] = hp;
    }
  }
}

// Per-lane plan of a wave's expansion passes (expand_wave): lane (j, cg)
// takes cells cg + 8 p in pass p; off packs, per pass, the byte offset of
// the cell's region row E[a][region] (two 16-bit halves per dword: passes 2pp
// and 2pp + 1; cells past the board read region 0 and are discarded).  Built
// once per batch, in registers -- or, on boards of more than 16 passes
// (19x19: 46), read per pass pair from the LDS table ExpandLds::rpair.
template <class G>
struct ExpandPlan {
  static constexpr int PASSES = (G::CELLS + 7) / 8;
  static constexpr bool TABLE = PASSES <= 16;
  uint32_t off[TABLE ? (PASSES + 1) / 2 : 1];
  const uint32_t* tab;
  static_assert(8 * PASSES <= G::CS, "the last pass's cells stay inside the head rows");
  static_assert(8 * 4 * G::C < 65536, "16-bit region offsets");
  // the packed offsets of one lane group's pass pairs (cells cg + 16 pp, + 8): the table entry
  __device__ __forceinline__ static uint32_t pair_entry(int pp, int cg) {
    auto off1 = [](int cell) { return cell < G::CELLS ? (uint32_t)region_of<G>(cell) * (uint32_t)G::C * 4u : 0u; };
    return off1(cg + 16 * pp) | (off1(cg + 16 * pp + 8) << 16);
  }
  __device__ __forceinline__ uint32_t pair(int pp, int cg) const {
    if constexpr (TABLE) return off[pp];
    else return tab[pp * 8 + cg];
  }
  __device__ __forceinline__ void init(const uint32_t* t = nullptr) {
    if constexpr (!TABLE) tab = t;
    if constexpr (TABLE) {
      const int cg = lane_id_local() >> 3;
#pragma unroll
      for (int i = 0; i < (PASSES + 1) / 2; ++i) off[i] = 0;
#pragma unroll
      for (int p = 0; p < PASSES; ++p) {
        const int cell = cg + 8 * p;
        const uint32_t reg = cell < G::CELLS ? (uint32_t)region_of<G>(cell) : 0u;
        off[p >> 1] |= (reg * (uint32_t)G::C * 4u) << (16 * (p & 1));
      }
    }
  }
};

// One child's heads by ONE wave (batch_expand), Y [CELLS][C] (LDS, or L2 for
// GLOBAL_Y boards), E[a] [9][C] and the head weights hw [3][C] (reward,
// value, policy) in LDS:
//   * the policy 1x1-conv sum of relu(Y + E[a]) per cell -> xw[PROW + cell];
//   * the reward and value heads only enter the network through their means
//     over the cells (self_play.py:91-94, :105-110), and a 1x1 conv is
//     linear, so their totals are taken channel-first:
//         sum_cells sum_c w_c relu(v)  =  sum_c w_c S_c,  S_c = sum_cells relu(v)
//     -> rsum, vsum (no biases; every lane).  One packed add per channel pair
//     and cell instead of two FMAs and two per-cell reductions.
// Lane (j, cg): channel float4s c4 = j + 8k, cells cg + 8p (every pass
// unrolled: Y at immediate offsets, E through the plan's offsets).  The 8
// lanes of a cell end with its full policy sum and all write it (same value,
// same address), so no lane is masked off; the last pass's cells past the
// board land in the row padding and stay out of S.  Wave-level; the caller
// orders xw for the wave's readers (wave_lds_sync).
// POL = false (lazy policy head, batched children): the totals only; the
// policy sums are formed if a select ever reaches the child (policy_sums_wg).
// GLOBAL_Y boards: Y loads one pass ahead (+0.5 % at 19x19 in the same call
// against none, round 4)
template <class G, int PROW, bool POL = true>
__device__ __forceinline__ void expand_wave(float* xw, const float* yc, const float* ew, const float* hw,
                                            const ExpandPlan<G>& plan, float& rsum, float& vsum) {
  typedef ExpandShape<G> X;
  constexpr int P = ExpandPlan<G>::PASSES;
  const int lane = lane_id_local();
  const int j = lane & 7, cg = lane >> 3;
  const f32x4* W4 = reinterpret_cast<const f32x4*>(hw);
  f32x4 wp[X::PERL];
  f32x2 s2[X::PERL][2];
#pragma unroll
  for (int k = 0; k < X::PERL; ++k) {
    if constexpr (POL) wp[k] = W4[2 * X::C4 + j + 8 * k];
    s2[k][0] = f32x2{0.f, 0.f};
    s2[k][1] = f32x2{0.f, 0.f};
  }
  const f32x4* Y4 = reinterpret_cast<const f32x4*>(yc) + cg * X::C4 + j;   // + pass * 8 * C4 + 8 k
  const char* Eb = reinterpret_cast<const char*>(reinterpret_cast<const f32x4*>(ew) + j);
  float* xr = xw + PROW + cg;
  // every pass unrolled on small boards; two at a time on 19x19 (46 passes)
  // one pass: cells cg + 8 p, E rows at byte offset eoff of ew (LAST: the
  // final pass, whose cells past the board stay out of the sums)
  // one pass over Y values already in registers
  auto pass_y = [&](int p, const f32x4 (&y)[X::PERL], uint32_t eoff, bool last) {
    const f32x4* E4 = reinterpret_cast<const f32x4*>(Eb + eoff);
    f32x4 e[X::PERL];
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) e[k] = E4[8 * k];
    const bool live = G::CELLS % 8 == 0 || !last || cg + 8 * p < G::CELLS;
    f32x2 hp2 = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) {
#pragma unroll
      for (int q = 0; q < 4; q += 2) {
        f32x2 v = f32x2{y[k][q], y[k][q + 1]} + f32x2{e[k][q], e[k][q + 1]};
        v.x = v.x > 0.f ? v.x : 0.f;
        v.y = v.y > 0.f ? v.y : 0.f;
        if constexpr (POL) hp2 = __builtin_elementwise_fma(f32x2{wp[k][q], wp[k][q + 1]}, v, hp2);
        if (!live) v = f32x2{0.f, 0.f};
        s2[k][q >> 1] = s2[k][q >> 1] + v;
      }
    }
    if constexpr (POL) xr[8 * p] = sum8(hp2.x + hp2.y);
  };
  (void)pass_y;
  auto pass = [&](int p, uint32_t eoff, bool last) {
    const f32x4* E4 = reinterpret_cast<const f32x4*>(Eb + eoff);
    f32x4 y[X::PERL], e[X::PERL];
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) {
      y[k] = Y4[p * 8 * X::C4 + 8 * k];
      e[k] = E4[8 * k];
    }
    const bool live = G::CELLS % 8 == 0 || !last || cg + 8 * p < G::CELLS;
    f32x2 hp2 = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) {
#pragma unroll
      for (int q = 0; q < 4; q += 2) {
        f32x2 v = f32x2{y[k][q], y[k][q + 1]} + f32x2{e[k][q], e[k][q + 1]};
        v.x = v.x > 0.f ? v.x : 0.f;
        v.y = v.y > 0.f ? v.y : 0.f;
        if constexpr (POL) hp2 = __builtin_elementwise_fma(f32x2{wp[k][q], wp[k][q + 1]}, v, hp2);
        if (!live) v = f32x2{0.f, 0.f};
        s2[k][q >> 1] = s2[k][q >> 1] + v;
      }
    }
    if constexpr (POL) xr[8 * p] = sum8(hp2.x + hp2.y);
  };
  if constexpr (ExpandPlan<G>::TABLE) {
    // every pass unrolled, offsets from the plan's registers
#pragma unroll
    for (int p = 0; p < P; ++p) pass(p, (plan.off[p >> 1] >> (16 * (p & 1))) & 0xFFFFu, p == P - 1);
  } else {
    // pass pairs, one LDS table read per pair (19x19: 23 pairs), Y streamed
    // from L2 one pass ahead: pass p + 1's loads are in flight while pass p
    // is computed (each wave's passes are latency-bound on L2)
    static_assert(P % 2 == 0, "whole pass pairs");
    f32x4 ya[X::PERL], yb[X::PERL];
    auto ldy = [&](int p, f32x4 (&y)[X::PERL]) {
#pragma unroll
      for (int k = 0; k < X::PERL; ++k) y[k] = Y4[p * 8 * X::C4 + 8 * k];
    };
    ldy(0, ya);
#pragma unroll 1
    for (int pp = 0; pp < P / 2; ++pp) {
      const uint32_t w2 = plan.pair(pp, cg);
      ldy(2 * pp + 1, yb);
      pass_y(2 * pp, ya, w2 & 0xFFFFu, false);
      if (pp + 1 < P / 2) ldy(2 * pp + 2, ya);
      pass_y(2 * pp + 1, yb, w2 >> 16, pp + 1 == P / 2);
    }
  }
  f32x2 dr2 = {0.f, 0.f}, dv2 = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < X::PERL; ++k) {
    const f32x4 wr = W4[j + 8 * k], wv = W4[X::C4 + j + 8 * k];
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
      dr2 = __builtin_elementwise_fma(f32x2{wr[q], wr[q + 1]}, s2[k][q >> 1], dr2);
      dv2 = __builtin_elementwise_fma(f32x2{wv[q], wv[q + 1]}, s2[k][q >> 1], dv2);
    }
  }
  rsum = wave_sum(dr2.x + dr2.y);
  vsum = wave_sum(dv2.x + dv2.y);
}

// Two children of one parent by ONE wave, Y streamed from L2 (GLOBAL_Y
// boards, 19x19; expand_wave's pass-pair loop): every Y value a lane loads
// serves both children, so a batch reads its parent's Y (139 KB at 19x19)
// once per pair of children instead of once per child.  Per child the
// operations and their order are expand_wave<..., true>'s, so both results
// are bit-identical to two expand_wave calls: child 0's policy sums go to
// xw[PROW + cell] as there; child 1's stay in registers, lane j of a lane
// group keeping passes p = j (mod 8) (pol1[p / 8]; its 8 lanes hold the same
// sum), until store_policy2 writes them over child 0's row.
template <class G>
struct Pol2 {
  static constexpr int SLOTS = (ExpandPlan<G>::PASSES + 7) / 8;
  float v[SLOTS];
};
template <class G, int PROW, bool POL = true>
__device__ __forceinline__ void expand_wave2(float* xw, const float* yc, const float* ew0, const float* ew1,
                                             const float* hw, const ExpandPlan<G>& plan, float& rsum0,
                                             float& vsum0, float& rsum1, float& vsum1, Pol2<G>& pol1) {
  typedef ExpandShape<G> X;
  constexpr int P = ExpandPlan<G>::PASSES;
  static_assert(!ExpandPlan<G>::TABLE && P % 2 == 0, "the pass-pair loop of Y-streaming boards");
  const int lane = lane_id_local();
  const int j = lane & 7, cg = lane >> 3;
  const f32x4* W4 = reinterpret_cast<const f32x4*>(hw);
  f32x4 wp[X::PERL];
  f32x2 sa[X::PERL][2], sb[X::PERL][2];
#pragma unroll
  for (int k = 0; k < X::PERL; ++k) {
    if constexpr (POL) wp[k] = W4[2 * X::C4 + j + 8 * k];
    sa[k][0] = sa[k][1] = sb[k][0] = sb[k][1] = f32x2{0.f, 0.f};
  }
  if constexpr (POL) {
#pragma unroll
    for (int i = 0; i < Pol2<G>::SLOTS; ++i) pol1.v[i] = 0.f;
  }
  const f32x4* Y4 = reinterpret_cast<const f32x4*>(yc) + cg * X::C4 + j;
  const char* Eb0 = reinterpret_cast<const char*>(reinterpret_cast<const f32x4*>(ew0) + j);
  const char* Eb1 = reinterpret_cast<const char*>(reinterpret_cast<const f32x4*>(ew1) + j);
  float* xr = xw + PROW + cg;
  auto pass_y = [&](int p, const f32x4 (&y)[X::PERL], uint32_t eoff, bool last) {
    const f32x4* E0 = reinterpret_cast<const f32x4*>(Eb0 + eoff);
    const f32x4* E1 = reinterpret_cast<const f32x4*>(Eb1 + eoff);
    f32x4 e0[X::PERL], e1[X::PERL];
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) { e0[k] = E0[8 * k]; e1[k] = E1[8 * k]; }
    const bool live = G::CELLS % 8 == 0 || !last || cg + 8 * p < G::CELLS;
    f32x2 ha = {0.f, 0.f}, hb = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) {
#pragma unroll
      for (int q = 0; q < 4; q += 2) {
        const f32x2 yy = f32x2{y[k][q], y[k][q + 1]};
        f32x2 va = yy + f32x2{e0[k][q], e0[k][q + 1]};
        va.x = va.x > 0.f ? va.x : 0.f;
        va.y = va.y > 0.f ? va.y : 0.f;
        if constexpr (POL) ha = __builtin_elementwise_fma(f32x2{wp[k][q], wp[k][q + 1]}, va, ha);
        if (!live) va = f32x2{0.f, 0.f};
        sa[k][q >> 1] = sa[k][q >> 1] + va;
        f32x2 vb = yy + f32x2{e1[k][q], e1[k][q + 1]};
        vb.x = vb.x > 0.f ? vb.x : 0.f;
        vb.y = vb.y > 0.f ? vb.y : 0.f;
        if constexpr (POL) hb = __builtin_elementwise_fma(f32x2{wp[k][q], wp[k][q + 1]}, vb, hb);
        if (!live) vb = f32x2{0.f, 0.f};
        sb[k][q >> 1] = sb[k][q >> 1] + vb;
      }
    }
    if constexpr (POL) {
      xr[8 * p] = sum8(ha.x + ha.y);
      const float pb = sum8(hb.x + hb.y);
#pragma unroll
      for (int i = 0; i < Pol2<G>::SLOTS; ++i) pol1.v[i] = p == 8 * i + j ? pb : pol1.v[i];
    }
  };
  f32x4 ya[X::PERL], yb[X::PERL];
  auto ldy = [&](int p, f32x4 (&y)[X::PERL]) {
#pragma unroll
    for (int k = 0; k < X::PERL; ++k) y[k] = Y4[p * 8 * X::C4 + 8 * k];
  };
  ldy(0, ya);
#pragma unroll 1
  for (int pp = 0; pp < P / 2; ++pp) {
    const uint32_t w2 = plan.pair(pp, cg);
    ldy(2 * pp + 1, yb);
    pass_y(2 * pp, ya, w2 & 0xFFFFu, false);
    if (pp + 1 < P / 2) ldy(2 * pp + 2, ya);
    pass_y(2 * pp + 1, yb, w2 >> 16, pp + 1 == P / 2);
  }
  f32x2 ra = {0.f, 0.f}, va2 = {0.f, 0.f}, rb = {0.f, 0.f}, vb2 = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < X::PERL; ++k) {
    const f32x4 wr = W4[j + 8 * k], wv = W4[X::C4 + j + 8 * k];
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
      ra = __builtin_elementwise_fma(f32x2{wr[q], wr[q + 1]}, sa[k][q >> 1], ra);
      va2 = __builtin_elementwise_fma(f32x2{wv[q], wv[q + 1]}, sa[k][q >> 1], va2);
      rb = __builtin_elementwise_fma(f32x2{wr[q], wr[q + 1]}, sb[k][q >> 1], rb);
      vb2 = __builtin_elementwise_fma(f32x2{wv[q], wv[q + 1]}, sb[k][q >> 1], vb2);
    }
  }
  rsum0 = wave_sum(ra.x + ra.y);
  vsum0 = wave_sum(va2.x + va2.y);
  rsum1 = wave_sum(rb.x + rb.y);
  vsum1 = wave_sum(vb2.x + vb2.y);
}

// child 1's policy sums (expand_wave2's registers) -> xw[PROW + cell]; the
// caller orders xw (wave_lds_sync) before and after
template <class G, int PROW>
__device__ __forceinline__ void store_policy2(float* xw, const Pol2<G>& pol1) {
  const int lane = lane_id_local();
  const int j = lane & 7, cg = lane >> 3;
#pragma unroll
  for (int i = 0; i < Pol2<G>::SLOTS; ++i) {
    const int p = 8 * i + j;
    if (p < ExpandPlan<G>::PASSES) xw[PROW + cg + 8 * p] = pol1.v[i];
  }
}

// Lazy policy head.  A batched child's policy logits are read only when a
// select first reaches it (~3 % of children: the reference's trees are wide),
// so batch expansions skip the policy 1x1 conv (expand_wave<..., false>) and
// the logits of such a node are formed on its first arrival from its parent's
// Y and its E[a] -- the child latent relu(Y + E[a]) rebuilt -- with
// expand_wave's operations in its order per cell (8 lanes per cell, lane j
// channels c4 = j + 8k, packed FMAs, the 3-step DPP sum): bit-identical to
// the sums the eager expansion wrote (self_play.py:104-112 on the child's
// latent, :204-207).
//
// One cell's policy sum (no bias) by the 8 lanes of a lane group.
template <class G>
__device__ __forceinline__ float policy_cell(const float* __restrict__ Y, const float* __restrict__ ea,
                                             const f32x4 (&wp)[ExpandShape<G>::PERL], int cell, int j) {
  typedef ExpandShape<G> X;
  const int cl = cell < G::CELLS ? cell : G::CELLS - 1;
  const f32x4* Y4 = reinterpret_cast<const f32x4*>(Y) + (size_t)cl * X::C4 + j;
  const f32x4* E4 = reinterpret_cast<const f32x4*>(ea) + region_of<G>(cl) * X::C4 + j;
  f32x4 y[X::PERL], e[X::PERL];
#pragma unroll
  for (int k = 0; k < X::PERL; ++k) {
    y[k] = Y4[8 * k];
    e[k] = E4[8 * k];
  }
  f32x2 hp2 = {0.f, 0.f};
#pragma unroll
  for (int k = 0; k < X::PERL; ++k) {
#pragma unroll
    for (int q = 0; q < 4; q += 2) {
      f32x2 v = f32x2{y[k][q], y[k][q + 1]} + f32x2{e[k][q], e[k][q + 1]};
      v.x = v.x > 0.f ? v.x : 0.f;
      v.y = v.y > 0.f ? v.y : 0.f;
      hp2 = __builtin_elementwise_fma(f32x2{wp[k][q], wp[k][q + 1]}, v, hp2);
    }
  }
  return sum8(hp2.x + hp2.y);
}

template <class G>
__device__ __forceinline__ void policy_weights(const float* hw, f32x4 (&wp)[ExpandShape<G>::PERL], int j) {
  typedef ExpandShape<G> X;
  const f32x4* W4 = reinterpret_cast<const f32x4*>(hw);
#pragma unroll
  for (int k = 0; k < X::PERL; ++k) wp[k] = W4[2 * X::C4 + j + 8 * k];
}

// The policy sums of every cell of one node -> out[CELLS] (LDS), by the whole
// workgroup: lane group (wave, cg) takes cells 8 wave + cg + 8 WAVES r.  Y: the
// parent's [CELLS][C] (HBM), ea: E[a] [9][C], hw: head weights [3][C].  All
// threads; the caller synchronises before reading out.
template <class G>
__device__ __forceinline__ void policy_sums_wg(float* out, const float* __restrict__ Y, const float* __restrict__ ea,
                                               const float* hw) {
  const int lane = lane_id_local(), j = lane & 7;
  const int slot = 8 * (tid_local() >> 6) + (lane >> 3);
  constexpr int SLOTS = 8 * G::WAVES, R = (G::CELLS + SLOTS - 1) / SLOTS;
  f32x4 wp[ExpandShape<G>::PERL];
  policy_weights<G>(hw, wp, j);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int cell = slot + SLOTS * r;
    const float s = policy_cell<G>(Y, ea, wp, cell, j);
    if (cell < G::CELLS) out[cell] = s;
  }
}

// The same by one wave (lane group cg: cells cg + 8 p) -> out[CELLS] (LDS).
// The caller orders out for the wave's readers (wave_lds_sync).
template <class G>
__device__ __forceinline__ void policy_sums_wave(float* out, const float* __restrict__ Y,
                                                 const float* __restrict__ ea, const float* hw) {
  const int lane = lane_id_local(), j = lane & 7, cg = lane >> 3;
  f32x4 wp[ExpandShape<G>::PERL];
  policy_weights<G>(hw, wp, j);
  for (int p = 0; p < (G::CELLS + 7) / 8; ++p) {
    const int cell = cg + 8 * p;
    const float s = policy_cell<G>(Y, ea, wp, cell, j);
    if (cell < G::CELLS) out[cell] = s;
  }
}

// The latent of a node that is about to become a parent: relu(Y_par + E[a])
// -> dst [C][CS] (channel-major, pad cells 0), the layout the 3x3 conv reads.
// Y is cell-major, so 32-channel slabs are transposed through LDS (lds: at
// least 32 * (CS + 1) floats, free until the conv): coalesced reads and
// writes; the next slab's loads are in flight during the current slab's
// transpose.  (One round over all channels at once measured slower.)  All
// threads; returns synchronised.
template <class G>
__device__ __forceinline__ void materialize(float* __restrict__ dst, const float* __restrict__ Ypar,
                                            const float* __restrict__ ea, float* lds) {
  constexpr int CB = 32, CSP = G::CS + 1, C4 = G::C / 4;
  static_assert(G::C % CB == 0, "32-channel slabs");
  const f32x4* Y4 = reinterpret_cast<const f32x4*>(Ypar);
  const f32x4* E4 = reinterpret_cast<const f32x4*>(ea);
  // each slab's loads are issued before the previous slab's barrier
  constexpr int NI = G::CELLS * (CB / 4), R = (NI + G::THREADS - 1) / G::THREADS;
  f32x4 y[R], e[R];
  auto load = [&](int c0) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = min(tid_local() + r * G::THREADS, NI - 1);
      const int p = i / (CB / 4), q = i - p * (CB / 4);
      y[r] = Y4[p * C4 + c0 / 4 + q];
      e[r] = E4[region_of<G>(p) * C4 + c0 / 4 + q];
    }
  };
  load(0);
  for (int c0 = 0; c0 < G::C; c0 += CB) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int i = tid_local() + r * G::THREADS;
      if (i < NI) {
        const int p = i / (CB / 4), q = i - p * (CB / 4);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float v = y[r][k] + e[r][k];
          lds[(4 * q + k) * CSP + p] = v > 0.f ? v : 0.f;
        }
      }
    }
    if (c0 + CB < G::C) load(c0 + CB);
    __syncthreads();
    for (int i = tid_local(); i < CB * G::CS; i += G::THREADS) {
      const int c = i / G::CS, p = i - c * G::CS;
      dst[(size_t)(c0 + c) * G::CS + p] = p < G::CELLS ? lds[c * CSP + p] : 0.f;
    }
    __syncthreads();
  }
}

}  // namespace mzgo

// mzgo_tower.hpp -- BASELINE config 5: MuZero with 20-block residual networks
// at 19x19 / 1600 simulations (no reference
// counterpart -- the architecture is mzgo/resnet.py's torch module, which is
// also the parity reference).
//
// The reference's dynamics is ONE conv (self_play.py:85-95), so the main
// engine can factor it (mzgo_expand.hpp); a residual tower is nonlinear after
// its first conv, so every simulation needs the whole tower on its leaf.  The
// per-game-per-CU megakernel cannot feed the MFMA pipes with 41 C=256 convs
// per simulation, so this engine splits the search from the evaluation:
//
//   k_tselect   one wave per game: select_leaf (self_play.py:239-335) on the
//               game's HBM tree -> (leaf latent slot, action, new node slot)
//   k_tconv_chain: the tower's 41 convs, ALL games' leaves, in one launch --
//               implicit GEMM on bf16 MFMA (v_mfma_f32_16x16x32_bf16, fp32
//               accumulate), one (board, 64-cout chunk) per workgroup through
//               every layer (k_tconv_ks: the same conv, one launch per layer)
//   k_texpand   one wave per game: heads -> child priors, backup (:198-230)
//
// Each game contributes exactly one leaf per simulation step, so the batch
// keeps every game's sequential semantics (no virtual loss).
//
// Activations (bf16) are stored per board as [C/64 chunks][P][64], P = (N+2)^2
// padded pixels with a zero border (the conv's zero padding, never written),
// each pixel's 128-byte row of 64 channels in 8 pieces of 16 bytes, piece j
// at position j ^ tswz(q) (q = padded pixel index): the LDS image of a
// chunk is a straight copy (global_load_lds) and the A-fragment reads of 16
// consecutive pixels are bank-conflict free (tswz below).  Weights are packed the same way
// per (cout chunk, cin chunk, tap): [64 cout rows][64 cin], piece swizzled by
// row.
#pragma once
#include "mzgo_kernels.hpp"

namespace mzgo {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int N_>
struct TGeo {
  static constexpr int N = N_;
  static constexpr int CELLS = N * N;
  static constexpr int A = CELLS + 1;
  static constexpr int AP = (A + 63) / 64;
  static constexpr int CS = (CELLS + 15) / 16 * 16;     // head-partial row stride
  static constexpr int W = N + 2;                       // padded board side
  static constexpr int P = W * W;                       // padded pixels
  static constexpr int TT = (CELLS + 15) / 16;          // 16-pixel M tiles of a board
  // tree kernels: one wave per game
  static constexpr int THREADS = 64, WAVES = 1, TREE_CAP = 0;
};

// Tower-conv geometry for NW waves per workgroup (one workgroup per CU).  The
// k-loop runs in steps of one kernel row (3 taps x one 64-channel cin chunk):
// a step's weight tile is 3 x 64 x 64 bf16 = 24 KiB.
template <int N, int NW>
struct TConvGeo {
  typedef TGeo<N> G;
  static constexpr int PBYTES = G::P * 128;             // one 64-channel chunk of the padded board
  static constexpr int PPIECES = (PBYTES + 1023) / 1024;   // 1-KiB DMA pieces of a chunk (last one partial)
  static constexpr int PB = (PBYTES + 15) / 16 * 16;    // its LDS buffer (the partial piece is masked)
  static constexpr int NPW = (PPIECES + NW - 1) / NW;   // pieces of a chunk per wave (some waves one less)
  static constexpr int WSLOT = 3 * 64 * 64 * 2;         // one step's weight tile
  static constexpr int WPW = WSLOT / 1024 / NW;         // its 1-KiB pieces per wave
  static constexpr int MT = (G::TT + NW - 1) / NW;      // 16-pixel tiles per wave
  // + bias and head weights (1 KiB) + the landing area of L2 touches (256 B)
  static constexpr int LDS = 2 * PB + 2 * WSLOT + 4 * 64 * 4 + 256;
  static_assert(WPW * NW * 1024 == WSLOT, "whole weight pieces per wave");
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(2 * PB >= G::CELLS * 272 + 9 * 64 * 4, "epilogue staging (+ E rows) must fit the patch buffers");
  // next chunk's patch pieces a wave issues at step ky (0, 1) of the current chunk
  __device__ static int pieces_at(int ky, int wave) {
    const int k0 = ky == 0 ? 0 : (NPW + 1) / 2, k1 = ky == 0 ? (NPW + 1) / 2 : NPW;
    int n = 0;
    for (int k = k0; k < k1; ++k) n += (k * NW + wave < PPIECES) ? 1 : 0;
    return n;
  }
};

// GEMM row m -> board cell (raster order), -1 for a pad row.  (Tiles of 16
// pixels of one board row, with the conflict-free swizzle below, took the
// fragment reads' LDS bank conflicts from 0.326 to 0.064 of the LDS cycles
// and made the conv no faster, round 4: removed in round 5.)
template <int N>
__device__ __forceinline__ int tcell(int m) { return m < N * N ? m : -1; }

// The position of 16-byte piece j of padded pixel q's 128-byte row is
// j ^ tswz(q): 16 consecutive pixel rows then read their MFMA fragments with
// few bank conflicts (a chunk's LDS image is still a straight LDS-DMA copy).
__device__ __forceinline__ int tswz(int q) {
  return (q >> 1) & 7;
}
// element offset of (padded pixel q, channel c) inside one 64-channel chunk
__device__ __forceinline__ int tpix(int q, int piece) { return q * 64 + ((piece ^ tswz(q)) << 3); }

// ---------------------------------------------------------------------------
// One 3x3 conv (+ bias [+ E-table term] [+ residual], ReLU) for nboards
// boards: out[b] = relu(conv(in[b]) + bias + E[act[b]][region] + res[b]).
// Optional fused 1x1 heads: hpart[b][cout chunk][h][cell] = sum over the
// chunk's 64 channels of headw[h][c] * out (the bf16-rounded output).
// ---------------------------------------------------------------------------
struct TConvArgs {
  const bf16* in; const int* in_idx; long long in_stride;       // board b: in + idx(b) * stride
  bf16* out; const int* out_idx; long long out_stride;
  const bf16* res; const int* res_idx; long long res_stride;    // nullable
  const bf16* w;                                                // [co][ci][9][64][64] packed
  const float* bias;                                            // [CO]
  const float* etab; const int* act;                            // nullable: E [A][9][CO], act[b]
  const float* headw; float* hpart;                             // nullable: [3][CO], [b][co][3][CS]
  const int* active;                                            // nullable: board b skipped if 0
  int nboards, ci_chunks, co_chunks;
};

template <class G, int T>
struct TapOff { static constexpr int v = (T / 3) * G::W + (T % 3); };

#ifdef MZGO_TCONV_STAMPS
// diagnostic build: per-workgroup cycle sums (wave 0): 0 total, 1 prologue,
// 2 vmcnt waits, 3 barriers, 4 MFMA steps, 5 epilogue, 6 launches
__device__ unsigned long long g_tstamps[4096][8][16];   // [block][wave][field]; 8 = s_memrealtime ticks (100 MHz)
#endif

// 16 bytes of an MFMA fragment (one ds_read_b128).  (Two ds_read_b64 with
// the halves of odd k-groups swapped on both operands are bank-conflict free
// for 16 consecutive pixel rows, but measured 1.6x slower: b64 reads need
// more waves per SIMD than this kernel has.)
template <int K, typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int K, typename F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl<K>(f, std::make_integer_sequence<int, K>{}); }

__device__ __forceinline__ bf16x8 frag_ld(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

#ifdef MZGO_TCONV_STAMPS
#define STAMP_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define STAMP_T(v) do {} while (0)
#endif

// ---------------------------------------------------------------------------
// k_tconv_ks: the same conv with the K dimension split across the two waves
// of a SIMD.  Wave w = (kh, mg), kh = w >> 2, mg = w & 3: waves kh = 0 take
// channels 0-31 of every (cin chunk, tap) slice, waves kh = 1 channels 32-63,
// and each wave owns 6 M tiles (96 pixels) x all 64 couts (24 accumulator
// tiles) instead of 3 x 64.  Per 16x16x32 MFMA a wave reads 0.42 fragments
// (6 A + 4 B per 24 MFMAs) instead of 0.58 (3 A + 4 B per 12): 30 instead of
// 42 ds_read_b128 per wave and kernel-row step for the same 72 MFMAs.  The
// two halves' partial sums meet once in the epilogue's fp32 staging (kh = 0
// stores, kh = 1 adds), so a cout's sum is (chain over cin 0-31 of every
// chunk) + (chain over cin 32-63) -- a different fp32 order, nothing else.
// (The M-split k_tconv it replaced -- 3 M tiles x 64 couts per wave, 0.58
// fragment reads per MFMA -- measured 26.75 vs 26.57 us per conv and was
// removed in round 5.)
// ---------------------------------------------------------------------------
// (s_setprio around every MFMA group or for waves 4-7 changed nothing, round
// 3.)  The timing ablations (wrong results) live in mzgo_diag.hpp, compiled
// only into diagnostic builds.
constexpr int kDmaSpread = 1;   // one DMA piece every kDmaSpread MFMA groups (2 / 3: 27.05 / 30.9 us, round 3)
#ifdef MZGO_DIAG_BUILD
#include "mzgo_diag.hpp"
#else
constexpr bool kAblNoDma = false, kAblNoBar = false;
#endif

template <int N>
struct TConvKsGeo {
  typedef TConvGeo<N, 8> T;
  static constexpr int MT = (TGeo<N>::TT + 3) / 4;      // tiles per wave (4 M groups)
  // 1 since round 4: 0 B scratch in k_tconv_ks and k_tconv_chain (2 left the
  // chain kernel 40 B of spills), config 5 1535-1537 -> 1514-1516 ms per move
  // (same call); 3 spills
  static constexpr int ADIST = 1;
  static_assert(ADIST >= 1 && ADIST <= 3 * MT, "A prefetch distance");
  static_assert(8 * MT * 2 * 1024 <= 2 * T::PB + 2 * T::WSLOT, "the epilogue's accumulator exchange fits the patch buffers + ring");
};

// workgroup -> (board, cout chunk): with nboards % 8 == 0 a board's CO
// workgroups are bid = x + 8 (j CO + cg) (board x + 8 j), all on XCD x (the
// dispatcher deals workgroups to the 8 XCDs in turn), so a board's chunks
// stay in one L2 from conv to conv
__device__ __forceinline__ void tconv_slot(int nboards, int CO, int& b, int& cg) {
  const int bid = blockIdx.x;
  if (nboards % 8 == 0) {
    const int x = bid & 7, k = bid >> 3;
    b = x + 8 * (k / CO);
    cg = k % CO;
  } else {
    b = bid / CO;
    cg = bid % CO;
  }
}

// This workgroup's (board, cout chunk) of conv a (tconv_slot; the body of
// k_tconv_ks and of each layer of k_tconv_chain).  All threads.
// the conv's LDS (patch buffers, weight ring, bias / head weights)
template <int N>
__device__ __forceinline__ char* tconv_lds() {
  __shared__ __attribute__((aligned(16))) char lds[TConvGeo<N, 8>::LDS];
  return lds;
}

// step 0's weight tile of conv a into ring slot 0 (k_tconv_chain issues it
// for the next layer before it waits for the board: slot 0 is free from
// the previous conv's last step on).  All threads.
template <int N>
__device__ __forceinline__ void tconv_issue_w0(const TConvArgs& a, int cg) {
  typedef TConvGeo<N, 8> T;
  char* const slot = tconv_lds<N>() + 2 * T::PB;
  const char* src = reinterpret_cast<const char*>(a.w + (size_t)cg * a.ci_chunks * 9 * 64 * 64);
  const int wave = __builtin_amdgcn_readfirstlane(tid_local() >> 6), lane = tid_local() & 63;
#pragma unroll
  for (int k = 0; k < T::WPW; ++k) {
    const int ii = k * 8 + wave;
    dma16(src + ii * 1024 + lane * 16, lds_addr(slot + ii * 1024));
  }
}

// The patch pieces bypass L1 (dma16_l2, agent-scope `sc1` loads): an input
// chunk is read once per conv and workgroup, and in k_tconv_chain it was
// written by other CUs of the XCC since the last read, so no L1 invalidate is
// needed between layers.  (Round 5 issued them `sc0`, workgroup scope, which
// hits L1 like a plain load: correct only because each conv streams far more
// than the 32 KiB L1 between two reads of a buffer)
__device__ __forceinline__ void dma_patch(const void* g, uint32_t lds_dst) {
  dma16_l2(g, lds_dst);
}

// w0_issued: tconv_issue_w0 ran for this conv already
template <int N>
__device__ __forceinline__ void tconv_ks_board(const TConvArgs& a, bool w0_issued = false) {
  typedef TGeo<N> G;
  typedef TConvGeo<N, 8> T;
  typedef TConvKsGeo<N> K;
  constexpr int NW = 8, MT = K::MT, AD = K::ADIST, NG = 3 * MT;
  char* const lds = tconv_lds<N>();
  STAMP_T(tstart);
#ifdef MZGO_TCONV_STAMPS
  unsigned long long acc_wait = 0, acc_bar = 0, acc_mfma = 0;
  const unsigned long long rstart = __builtin_amdgcn_s_memrealtime();
#endif
  const int CO = a.co_chunks, CC = a.ci_chunks;
  const int bid = blockIdx.x;
  int b, cg;
  tconv_slot(a.nboards, CO, b, cg);
  const int tid = tid_local(), lane = tid & 63;   // (tid_local: nothing lane-derived is hoisted out of k_tconv_chain's layer loop)
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = wave >> 2, mg = wave & 3;
  char* const patch0 = lds;
  char* const wring = lds + 2 * T::PB;
  float* const sbias = reinterpret_cast<float*>(lds + 2 * T::PB + 2 * T::WSLOT);
  float* const shw = sbias + 64;
  const bf16* in = a.in + (long long)(a.in_idx ? a.in_idx[b] : b) * a.in_stride;
  const bf16* wsrc = a.w + (size_t)cg * CC * 9 * 64 * 64;
  if (tid < 64) {
    sbias[tid] = a.bias[cg * 64 + tid];
    if (a.headw)
      for (int h = 0; h < 3; ++h) shw[h * 64 + tid] = a.headw[h * CO * 64 + cg * 64 + tid];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  auto issue_patch_pieces = [&](int cc, int buf, int k0, int k1) {
    const char* src = reinterpret_cast<const char*>(in + (size_t)cc * G::P * 64);
    for (int k = k0; k < k1; ++k) {
      const int ii = k * NW + wave;
      if (ii >= T::PPIECES) break;
      const int off = ii * 1024 + lane * 16;
      if (off < T::PBYTES) dma_patch(src + off, lds_addr(patch0 + buf * T::PB + ii * 1024));
    }
  };
  auto issue_w = [&](int s) {
    const char* src = reinterpret_cast<const char*>(wsrc + (size_t)s * 3 * 64 * 64);
    char* slot = wring + (s & 1) * T::WSLOT;
#pragma unroll
    for (int k = 0; k < T::WPW; ++k) {
      const int ii = k * NW + wave;
      dma16(src + ii * 1024 + lane * 16, lds_addr(slot + ii * 1024));
    }
  };
  const int nsteps = 3 * CC;
  issue_patch_pieces(0, 0, 0, T::NPW);
  if (!w0_issued) issue_w(0);

  // this wave's half of a 64-channel row: byte 64 * kh of the pixel's 128
  const int hx = kh * 64;
  int qb[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int p = tcell<N>((mg * MT + i) * 16 + (lane & 15));
    qb[i] = p >= 0 ? (p / N) * G::W + (p % N) : 0;
  }
  int boff[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) {
    const int r = n * 16 + (lane & 15);
    boff[n] = (r * 128 + (((lane >> 4) ^ ((r >> 1) & 7)) << 4)) ^ hx;
  }
  f32x4 acc[MT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[i][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto touch_epilogue = [&]() {
    if (!a.res) return;
    const char* r = reinterpret_cast<const char*>(a.res + (long long)(a.res_idx ? a.res_idx[b] : b) * a.res_stride +
                                                  (size_t)cg * G::P * 64);
    constexpr int L0 = G::W + 1, NL = (G::N - 1) * G::W + G::N;
    if (tid < NL) dma4(r + (size_t)(L0 + tid) * 128, lds_addr(lds) + (uint32_t)(T::LDS - 256));
  };
  STAMP_T(tpro);

  // A wave whose last tile lies past the board (19x19: tile 23 of wave mg = 3)
  // skips that tile's MFMAs: the chip holds a lower clock under MFMA load,
  // so a dead tile's MFMAs cost the live ones time.
  const bool lastdead = __builtin_amdgcn_readfirstlane((mg + 1) * MT > G::TT);
  for (int cc = 0; cc < CC; ++cc) {
    const bool nextp = cc + 1 < CC;
    const char* pbuf = patch0 + (cc & 1) * T::PB;
    bf16x8 afn[AD];
    auto frag_a = [&](int kyv, int kx, int i) {
      const int q = qb[i] + kyv * G::W + kx;
      return frag_ld(pbuf + ((q * 128 + (((lane >> 4) ^ tswz(q)) << 4)) ^ hx));
    };
    auto step = [&](auto kyc) {
      constexpr int ky = decltype(kyc)::value;
      const int s = cc * 3 + ky;
      STAMP_T(ts0);
      int younger = 0;
      if (ky >= 1 && ky - 1 < 2 && nextp) younger = T::pieces_at(ky - 1, wave);
      wait_vmcnt_dyn(younger);
      STAMP_T(ts1);
      if constexpr (kAblNoBar) {
      } else if constexpr (ky > 0) {
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(AD) : "memory");
        __builtin_amdgcn_s_barrier();
      } else {
        lds_barrier();
      }
      STAMP_T(ts2);
      auto issue_dma = [&]() {
        if constexpr (kAblNoDma) if (s > 0) return;
        if (s + 1 < nsteps) issue_w(s + 1);
        if (nextp && ky < 2) {
          constexpr int k0 = ky == 0 ? 0 : (T::NPW + 1) / 2, k1 = ky == 0 ? (T::NPW + 1) / 2 : T::NPW;
          issue_patch_pieces(cc + 1, (cc + 1) & 1, k0, k1);
        }
        if (s == nsteps - 1) touch_epilogue();
      };
      // DMA piece j of this step (spread over the groups with kDmaSpread):
      // weight pieces first, then the next chunk's patch pieces (the vmcnt
      // accounting of the next step counts the patch pieces issued after W(s+1))
      constexpr int PK0 = ky == 0 ? 0 : (T::NPW + 1) / 2, PK1 = ky == 0 ? (T::NPW + 1) / 2 : T::NPW;
      constexpr int NPC = ky < 2 ? PK1 - PK0 : 0, NDMA = T::WPW + NPC;
      auto dma_piece = [&](int j) {
        if (j < T::WPW) {
          if (s + 1 < nsteps) {
            const int ii = j * NW + wave;
            dma16(reinterpret_cast<const char*>(wsrc + (size_t)(s + 1) * 3 * 64 * 64) + ii * 1024 + lane * 16,
                  lds_addr(wring + ((s + 1) & 1) * T::WSLOT + ii * 1024));
          }
        } else if (nextp) {
          const int ii = (PK0 + j - T::WPW) * NW + wave;
          const int off = ii * 1024 + lane * 16;
          if (ii < T::PPIECES && off < T::PBYTES)
            dma_patch(reinterpret_cast<const char*>(in + (size_t)(cc + 1) * G::P * 64) + off,
                  lds_addr(patch0 + ((cc + 1) & 1) * T::PB + ii * 1024));
        }
      };
      const char* ws = wring + (s & 1) * T::WSLOT;
      bf16x8 bf[2][4], af[AD + 1];
      auto load_b = [&](int kx, bf16x8 (&d)[4]) {
        const char* wt = ws + kx * 64 * 64 * 2;
#pragma unroll
        for (int n = 0; n < 4; ++n) d[n] = frag_ld(wt + boff[n]);
      };
      auto load_a = [&](auto gc) {
        constexpr int g = decltype(gc)::value, kx = g / MT, i = g % MT;
        af[g % (AD + 1)] = frag_a(ky, kx, i);
      };
      load_b(0, bf[0]);
      if constexpr (ky > 0) {
#pragma unroll
        for (int g = 0; g < AD; ++g) af[g] = afn[g];
      } else {
        static_for<AD>([&](auto gc) { load_a(gc); });
      }
      constexpr bool SPREAD = kDmaSpread > 0 && (NDMA - 1) * kDmaSpread < NG;
      if constexpr (!SPREAD) issue_dma();
      else if (s == nsteps - 1) touch_epilogue();
      auto group = [&](auto gc) {
        constexpr int g = decltype(gc)::value, kx = g / MT, i = g % MT;
        if constexpr (SPREAD && g % kDmaSpread == 0 && g / kDmaSpread < NDMA) {
          dma_piece(g / kDmaSpread);
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (i == 0 && kx + 1 < 3) load_b(kx + 1, bf[(kx + 1) & 1]);
        if constexpr (g + AD < NG) load_a(std::integral_constant<int, g + AD>{});
        constexpr int nrd = (i == 0 && kx + 1 < 3 ? 4 : 0) + (g + AD < NG ? 1 : 0);
        if constexpr (nrd > 0) __builtin_amdgcn_sched_group_barrier(0x100, nrd, 0);
          if (!(i == MT - 1 && lastdead)) {
#pragma unroll
          for (int n = 0; n < 4; ++n)
            acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[kx & 1][n], af[g % (AD + 1)], acc[i][n], 0, 0, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      static_for<NG>([&](auto gc) { group(gc); });
      if constexpr (ky < 2) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < AD; ++g) afn[g] = frag_a(ky + 1, g / MT, g % MT);
      }
      STAMP_T(ts3);
#ifdef MZGO_TCONV_STAMPS
      acc_wait += ts1 - ts0; acc_bar += ts2 - ts1; acc_mfma += ts3 - ts2;
#endif
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
  }
  lds_barrier();
  STAMP_T(tloop);

  // Epilogue straight from the accumulators (no fp32 staging image).  The
  // MFMAs above put couts on the output rows: lane l of acc[i][n] holds couts
  // 16n + 4(l >> 4) .. +3 of pixel (l & 15) of tile i.  1. The two K halves
  // meet: each wave hands its partner (same mg) the n-tiles the partner
  // finishes (kh = 0 finishes n = 0, 1; kh = 1 n = 2, 3) through LDS, one
  // ds_write_b128 / ds_read_b128 per tile (a + b == b + a: the sum is the
  // same whichever wave forms it).  2. v_permlane16_swap of the two kept
  // n-tiles gives every lane 8 consecutive couts of its pixel -- one 16-byte
  // piece: bias, E[a] region term, residual, ReLU, bf16, one store.
  bf16* out = a.out + (long long)(a.out_idx ? a.out_idx[b] : b) * a.out_stride + (size_t)cg * G::P * 64;
  const bf16* res = a.res ? a.res + (long long)(a.res_idx ? a.res_idx[b] : b) * a.res_stride + (size_t)cg * G::P * 64
                          : nullptr;
  constexpr int XBYTES = 8 * MT * 2 * 1024;            // exchange area
  float* const set = reinterpret_cast<float*>(lds + XBYTES);          // E rows [9][64]
  float* const hxs = set + 9 * 64;                                     // head partials of kh = 1 [4][MT][16][3]
  static_assert(XBYTES + (9 * 64 + 4 * MT * 16 * 3) * 4 <= 2 * T::PB + 2 * T::WSLOT, "epilogue LDS");
  // lane indices re-read here (tid_local: an empty asm), so nothing the
  // epilogue derives from them is hoisted above the k-loop and kept live through it
  const int elane = tid_local() & 63;
  const int row = elane >> 4, col = elane & 15;
  int qv[MT];
  bool okv[MT];
  bf16x8 r8[MT];
  float hsum[MT][3];
  f32x4* const xch = reinterpret_cast<f32x4*>(lds);
  // The per-wave parts take kh as a constant (no dynamic register indexing of
  // acc); every barrier sits between them, in code all waves run.
  // 1. hand the partner its n-tiles; the residual pieces
  auto give = [&](auto khc) {
    constexpr int KH = decltype(khc)::value, GIVE = KH == 0 ? 2 : 0, KEEP = 2 - GIVE;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn) xch[(((mg * 2 + KH) * MT + i) * 2 + nn) * 64 + lane] = acc[i][GIVE + nn];
    // this lane's piece after the swap and its 8 couts
    const int pc = 2 * (KEEP + (row & 1)) + (row >> 1);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int p = tcell<N>((mg * MT + i) * 16 + col);
      okv[i] = (mg * MT + i) < G::TT && p >= 0;
      qv[i] = okv[i] ? (p / N + 1) * G::W + (p % N) + 1 : 0;
    }
    if (res) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
        if (okv[i]) r8[i] = *reinterpret_cast<const bf16x8*>(res + tpix(qv[i], pc));
    }
  };
  if (kh == 0) give(std::integral_constant<int, 0>{});
  else give(std::integral_constant<int, 1>{});
  STAMP_T(tgive);
  if (a.etab) {
    const float* eb = a.etab + (size_t)a.act[b] * 9 * CO * 64 + cg * 64;
    for (int k = tid; k < 9 * 64; k += NW * 64) set[k] = eb[(size_t)(k >> 6) * CO * 64 + (k & 63)];
  }
  __syncthreads();
  // 2. the partner's half added, the epilogue, the head partials of kh = 1 staged
  auto finish = [&](auto khc) {
    constexpr int KH = decltype(khc)::value, KEEP = KH == 0 ? 0 : 2;
    const int pc = 2 * (KEEP + (row & 1)) + (row >> 1), c0 = pc * 8;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int nn = 0; nn < 2; ++nn) acc[i][KEEP + nn] += xch[(((mg * 2 + (KH ^ 1)) * MT + i) * 2 + nn) * 64 + lane];
    float bias[8];
    {
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(sbias + c0), b1 = *reinterpret_cast<const f32x4*>(sbias + c0 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { bias[e] = b0[e]; bias[e + 4] = b1[e]; }
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][KEEP][r]),
                                                         __float_as_uint(acc[i][KEEP + 1][r]), false, false);
        v[r] = __uint_as_float(sw[0]);
        v[r + 4] = __uint_as_float(sw[1]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bias[e];
      if (a.etab) {
        const int p = tcell<N>((mg * MT + i) * 16 + col);
        const int y = okv[i] ? p / N : 0, x = okv[i] ? p % N : 0;
        const int reg = 3 * (y == 0 ? 0 : (y == N - 1 ? 2 : 1)) + (x == 0 ? 0 : (x == N - 1 ? 2 : 1));
        const f32x4 e0 = *reinterpret_cast<const f32x4*>(set + reg * 64 + c0);
        const f32x4 e1 = *reinterpret_cast<const f32x4*>(set + reg * 64 + c0 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[e] += e0[e]; v[e + 4] += e1[e]; }
      }
      if (res) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (float)r8[i][e];
      }
      bf16x8 o8;
#pragma unroll
      for (int e = 0; e < 8; ++e) o8[e] = (bf16)(v[e] > 0.f ? v[e] : 0.f);
      if (okv[i]) *reinterpret_cast<bf16x8*>(out + tpix(qv[i], pc)) = o8;
      if (a.headw) {
#pragma unroll
        for (int hh = 0; hh < 3; ++hh) {
          float sum = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) sum += shw[hh * 64 + c0 + e] * (float)o8[e];
          sum += __shfl_xor(sum, 16);
          sum += __shfl_xor(sum, 32);
          hsum[i][hh] = sum;
        }
      }
    }
    // the pixel's head sums over this chunk's 64 couts: (kh = 0's 32) + (kh = 1's 32)
    if (KH == 1 && a.headw && row == 0)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int hh = 0; hh < 3; ++hh) hxs[((mg * MT + i) * 16 + col) * 3 + hh] = hsum[i][hh];
  };
  if (kh == 0) finish(std::integral_constant<int, 0>{});
  else finish(std::integral_constant<int, 1>{});
  STAMP_T(tfin);
  // 3. kh = 0 stores the chunk's head partials
  if (a.headw) {
    __syncthreads();
    if (kh == 0 && row == 0)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int p = tcell<N>((mg * MT + i) * 16 + col);
        if (!okv[i]) continue;
        float* hp = a.hpart + ((size_t)b * CO + cg) * 3 * G::CS + p;
#pragma unroll
        for (int hh = 0; hh < 3; ++hh) hp[hh * G::CS] = hsum[i][hh] + hxs[((mg * MT + i) * 16 + col) * 3 + hh];
      }
  }
  STAMP_T(txch);
#ifdef MZGO_TCONV_STAMPS
  if (lane == 0 && bid < 4096) {
    const unsigned long long tend = __builtin_amdgcn_s_memtime();
    const unsigned long long rend = __builtin_amdgcn_s_memrealtime();
    unsigned long long* g = g_tstamps[bid][wave];
    g[8] += rend - rstart;
    g[0] += tend - tstart; g[1] += tpro - tstart; g[2] += acc_wait; g[3] += acc_bar; g[4] += acc_mfma;
    g[5] += tend - tloop; g[6] += 1; g[7] += txch - tloop;
    g[9] += tgive - tloop; g[10] += tfin - tgive; g[11] += txch - tfin;
  }
#endif
}

template <int N>
__global__ void __launch_bounds__(512) k_tconv_ks(TConvArgs a) {
  int b, cg;
  tconv_slot(a.nboards, a.co_chunks, b, cg);
  if (a.active && !a.active[b]) return;
  tconv_ks_board<N>(a);
}

// ---------------------------------------------------------------------------
// k_tconv_chain: the nl convs of one tower (layers[0..nl), each a
// k_tconv_ks conv) in ONE launch.  Workgroup (b, cg) computes cout chunk cg
// of board b for every layer in turn; layer l + 1 reads all CO chunks of
// board b's layer-l output (and a residual it wrote itself earlier), so
// before it starts, the workgroup waits until the board's CO workgroups
// have published layer l: flags[b * CO + k] = seq0 + l + 1 (monotonic
// across launches; compared modulo 2^32).  A board's workgroups only wait on
// each other, and the launch has at most one workgroup per CU (T::LDS), so
// the host uses it only when all nboards * CO workgroups fit the chip at
// once; every wait is bounded (~1 s): on expiry *err is set and the
// workgroup stops waiting (wrong results, reported, never a hung GPU).
//
// Hand-off.  Agent scope (cdna_hip_programming.md G16: drained stores, a
// barrier, buffer_wbl2 + flag; flag, buffer_inv sc1) writes back and
// invalidates the XCD's L2 per workgroup and layer, so every later read of
// the weights misses L2 -- measured 14 % slower than one launch per conv.
// Each workgroup therefore first publishes its XCC id (HW_REG_XCC_ID); when
// all CO workgroups of its board run on one XCC (the usual placement,
// tconv_slot) the board's hand-offs stay inside that XCC's L2, the
// coherence point of its CUs: the producer drains its stores to L2 and
// stores the flag, the consumer sees the flag and reads the patch from L2
// past its CU's L1 (dma_patch: `sc1` loads).  Every other load of the chain
// reads bytes no other workgroup writes in the launch (weights, bias, E
// table, and the residual: chunk cg of a board is only ever written by
// workgroup (b, cg), whose own earlier stores its L1 reflects).  A board split
// over XCCs keeps the agent-scope protocol.  Replaces 2 blocks + 1 launches per tower: no per-launch
// dispatch ramp and drain, and a board starts its next conv as soon as its
// own chunks are done.
// ---------------------------------------------------------------------------
struct TConvChain {
  const TConvArgs* layers;   // [nl] (device memory)
  int nl;
  unsigned* flags;           // [nboards * co_chunks]: layers published
  unsigned long long* xcc;   // [nboards * co_chunks]: seq0 << 32 | XCC id of the launch
  unsigned seq0;
  int* err;
  long long spin_max;        // bound of every wait in s_sleep rounds (1 << 24 ~ 1 s; a test hook may lower it)
};

// bounded wait until (int)(*p - want) >= 0 (thread 0); false on expiry
// (spin_max < 0, a test hook: every wait expires, ready or not)
__device__ __forceinline__ bool chain_wait(const unsigned* p, unsigned want, long long spin_max) {
  if (spin_max < 0) return false;
  for (long long spins = 0; (int)(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0;
       ++spins) {
    if (spins > spin_max) return false;
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

template <int N>
__global__ void __launch_bounds__(512) k_tconv_chain(TConvChain c, const TConvArgs* __restrict__ layers) {
  // (layers: c.layers as a restrict pointer, so the fields are scalar loads
  // -- read-only for the launch -- not vector loads in every epilogue)
  __shared__ int s_local;
  const int nboards = layers[0].nboards, CO = layers[0].co_chunks;
  int b, cg;
  tconv_slot(nboards, CO, b, cg);
  const int* active = layers[0].active;
  if (active && !active[b]) return;
  unsigned* fl = c.flags + (size_t)b * CO;
  bool bad = false;
  // this launch's placement: is every chunk of board b on this XCC?
  if (threadIdx.x == 0) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    x &= 0xFu;
    unsigned long long* xs = c.xcc + (size_t)b * CO;
    __hip_atomic_store(xs + cg, (unsigned long long)c.seq0 << 32 | x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int local = 1;
    for (int k = 0; k < CO; ++k) {
      unsigned long long v = __hip_atomic_load(xs + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (long long spins = 0; (unsigned)(v >> 32) != c.seq0; ++spins) {
        if (spins > c.spin_max) { bad = true; break; }
        __builtin_amdgcn_s_sleep(1);
        v = __hip_atomic_load(xs + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (bad) break;
      local &= (unsigned)(v & 0xFu) == x ? 1 : 0;
    }
    if (bad) atomicOr(c.err, 2);
    s_local = bad ? 0 : local;
  }
  __syncthreads();
  const bool local = s_local != 0;
  for (int l = 0; l < c.nl; ++l) {
    if (l > 0) {
      // lanes 0..CO-1 of wave 0 poll the board's CO flags at once (one round trip each)
      if (threadIdx.x < (unsigned)CO && !bad) {
        if (!chain_wait(fl + threadIdx.x, c.seq0 + (unsigned)l, c.spin_max)) {
          atomicOr(c.err, 1);
          bad = true;
        }
        // local: the data is in the XCC's L2, which the patch reads go to
        // (dma_patch, sc1 loads past this CU's L1); otherwise the agent-scope
        // acquire (buffer_inv sc1) drops this CU's stale lines
        if (!local) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the invalidate done before the barrier
        }
      }
      __syncthreads();
    }
    const TConvArgs& a = layers[l];   // (fields read where used: fewer live SGPRs)
    tconv_ks_board<N>(a, l > 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      if (!local) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (ROCm 7.2 may drop the fence's own wait)
      }
      __hip_atomic_store(fl + cg, c.seq0 + (unsigned)l + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the next conv's first weight tile lands while the board's other chunks finish
    if (l + 1 < c.nl) tconv_issue_w0<N>(layers[l + 1], cg);
  }
}

// ---------------------------------------------------------------------------
// Per-game tree kernels (one wave per game; the tree is in HBM between
// launches, exactly the arrays of the main engine's EngineArrays).
// ---------------------------------------------------------------------------
struct TowerArrays {
  bf16* pool;            // [G*(S+1)] node latents (slot g*(S+1) + node)
  long long slot;        // elements per latent slot: (C/64) * P * 64
  bf16* rep_in;          // [G][P*64] representation input (6 planes, 64-channel chunk)
  float* hpart;          // [G][C/64][3][CS] fused head partials
  uint8_t* rootmask;     // [G][A] valid_board (INVD == 0), 1 for pass
  double* passp;         // [G] pass prior
  uint64_t* key;         // [G] RNG stream key of the current search
  int* playing;          // [G] representation / root / choose run for this slot
  int* evalact;          // [G] this simulation step evaluates a leaf
  int* in_idx;           // [G] latent slot of the leaf being expanded
  int* out_idx;          // [G] latent slot of the new node
  int* root_idx;         // [G] g*(S+1)
  int* act;              // [G] action applied to the leaf
  int* job;              // [G][3] leaf, depth, new node id
  int* simc;             // [G] simulation index
  int C, co_chunks;
  HeadScalars hs;
  const float* headw;    // [3][C]: reward_conv, value_conv, policy_conv
  float* node_out;       // test hook (mzgo_tower_record_nodes): [G][S+1][A+2] logits, reward, value; or null
  // batched simulation steps (k_tbatch / k_tboards / k_tbexpand): each game's
  // pending batch -- the leaf, its first node id, and per entry the action and
  // the tower's reward and value once evaluated
  int bq_cap;            // entries per game
  int* bq_n;             // [G] entries of the pending batch (0: none)
  int* bq_leaf;          // [G][bq_cap] the node entry i expands
  int* bq_nid0;          // [G] node id of entry 0 (entry i's latent: pool slot g*(S+1) + nid0 + i)
  int* bq_act;           // [G][bq_cap]
  float* bq_rv;          // [G][bq_cap][2] reward, value
  int* nbg;              // [G] boards this step
  // this step's boards, all games (k_tboards): leaf slot, output slot, action, game, entry
  int* b_in; int* b_out; int* b_act; int* b_game; int* b_ent;
  int* b_total;          // [1] boards this step
};

template <class G>
__device__ __forceinline__ void tload_mask(TreeLds<G>& t, const TowerArrays& T, int g) {
  for (int a = threadIdx.x; a < G::A; a += 64) t.valid[a] = T.rootmask[(size_t)g * G::A + a];
  if (threadIdx.x == 0) t.pass_prior = T.passp[g];
  t.newest = -1;
  t.newp_node = -1;
  t.rowc_node = -1;
  wave_lds_sync();
}

// sum of a board's head partials over the cout chunks (ascending) -> hp [3][CS]
// (up to 4 chunks, C <= 256: every load of the wave issued before the first
// add -- one memory round trip instead of one per 64 entries; the sums keep
// the ascending chunk order)
template <class G>
__device__ __forceinline__ void tsum_heads(const TowerArrays& T, int b, float* hp) {
  const float* src = T.hpart + (size_t)b * T.co_chunks * 3 * G::CS;
  constexpr int PER = (3 * G::CS + 63) / 64;
  const int lane = threadIdx.x & 63;
  if (T.co_chunks <= 4) {
    float v[4][PER];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const int i = lane + 64 * p;
        v[c][p] = (c < T.co_chunks && i < 3 * G::CS) ? src[(size_t)c * 3 * G::CS + i] : 0.f;
      }
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int i = lane + 64 * p;
      float s = v[0][p];
#pragma unroll
      for (int c = 1; c < 4; ++c)
        if (c < T.co_chunks) s += v[c][p];
      if (i < 3 * G::CS) hp[i] = s;
    }
  } else {
    for (int i = lane; i < 3 * G::CS; i += 64) {
      float s = src[i];
      for (int c = 1; c < T.co_chunks; ++c) s += src[(size_t)c * 3 * G::CS + i];
      hp[i] = s;
    }
  }
  wave_lds_sync();
}

template <class G>
__device__ __forceinline__ float tplane(const int8_t* stone, const uint8_t* invd, const BoardMeta& m, int c, int j) {
  switch (c) {
    case 0: return stone[j] == 1 ? 1.f : 0.f;
    case 1: return stone[j] == 2 ? 1.f : 0.f;
    case 2: return (float)m.turn;
    case 3: return (float)invd[j];
    case 4: return (float)m.passed;
    default: return (float)m.done;
  }
}

// representation input board + root mask from 6 observation planes plane(c, cell)
template <class G, class PlaneFn>
__device__ __forceinline__ void tstage_root(const TowerArrays& T, int g, double pass_epsilon, PlaneFn plane) {
  bf16* dst = T.rep_in + (size_t)g * G::P * 64;
  for (int i = threadIdx.x; i < G::CELLS * 8; i += 64) {
    const int p = i >> 3, j = i & 7;
    const int y = p / G::N, x = p - y * G::N;
    const int q = (y + 1) * G::W + (x + 1);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)((j == 0 && k < 6) ? plane(k, p) : 0.f);
    *reinterpret_cast<bf16x8*>(dst + tpix(q, j)) = o;
  }
  int any = 0;
  for (int a = threadIdx.x; a < G::A; a += 64) {
    const uint8_t v = a < G::CELLS ? (plane(3, a) == 0.f ? 1 : 0) : 1;
    T.rootmask[(size_t)g * G::A + a] = v;
    any |= (a < G::CELLS) && v;
  }
  any = __any(any);
  if (threadIdx.x == 0) T.passp[g] = any ? pass_epsilon : 1.0;
}

// self-play move start: observation record, representation input, root mask
template <int N>
__global__ void __launch_bounds__(64) k_tobs(TowerArrays T, SearchParams sp, PlayParams pp, EngineArrays E) {
  typedef TGeo<N> G;
  const int g = blockIdx.x;
  __shared__ int8_t stone[G::CELLS];
  __shared__ uint8_t invd[G::CELLS];
  if (E.status[g] != 0) { if (threadIdx.x == 0) T.playing[g] = 0; return; }
  for (int c = threadIdx.x; c < G::CELLS; c += 64) {
    stone[c] = E.stones[(size_t)g * G::CELLS + c];
    invd[c] = E.invd[(size_t)g * G::CELLS + c];
  }
  BoardMeta m;
  const int* mm = E.meta + g * 4;
  m.turn = mm[0]; m.passed = mm[1]; m.done = mm[2]; m.moves = mm[3];
  wave_lds_sync();
  const size_t rec = (size_t)g * E.max_moves + m.moves;
  for (int c = threadIdx.x; c < G::CELLS; c += 64) {
    E.rec_stones[rec * G::CELLS + c] = stone[c];
    E.rec_invd[rec * G::CELLS + c] = invd[c];
  }
  if (threadIdx.x == 0) {
    E.rec_flags[rec] = (uint8_t)(m.turn | (m.passed << 1) | (m.done << 2));
    T.playing[g] = 1;
    const uint32_t gid = (uint32_t)(pp.game_base + g) ^ ((uint32_t)pp.epoch << 24);
    T.key[g] = stream_key(sp.seed, gid, (uint32_t)m.moves);
  }
  tstage_root<G>(T, g, sp.pass_epsilon, [&](int c, int j) { return tplane<G>(stone, invd, m, c, j); });
}

// search API start: root observations f32 [G][6][N][N]
template <int N>
__global__ void __launch_bounds__(64) k_tobs_search(TowerArrays T, SearchParams sp, const float* __restrict__ obs,
                                                    int game_base, int move_index) {
  typedef TGeo<N> G;
  const int g = blockIdx.x;
  const float* o = obs + (size_t)g * 6 * G::CELLS;
  if (threadIdx.x == 0) {
    T.playing[g] = 1;
    T.key[g] = stream_key(sp.seed, (uint32_t)(game_base + g), (uint32_t)move_index);
  }
  tstage_root<G>(T, g, sp.pass_epsilon, [&](int c, int j) { return o[c * G::CELLS + j]; });
}

// root priors (self_play.py:148-182) from the representation's heads, tree reset
template <int N>
__global__ void __launch_bounds__(64) k_troot(TowerArrays T, SearchParams sp, EngineArrays E,
                                              const double* __restrict__ noise, long long game_stride,
                                              int per_move) {
  typedef TGeo<N> G;
  const int g = blockIdx.x;
  if (!T.playing[g]) return;
  __shared__ TreeLds<G> t;
  __shared__ float hp[3 * G::CS];
  tload_mask<G>(t, T, g);
  stage_head_scalars(T.hs, t.hsc);
  tsum_heads<G>(T, g, hp);
  // representation: no reward head; value, then policy (rows 1, 2 of hp)
  heads_logits<G, 1>(hp + G::CS, false, t.hsc, t.logits);
  wave_lds_sync();
  if (T.node_out) {                       // (test hook) node 0: the root's logits and value
    float* o = T.node_out + (size_t)g * (E.S + 1) * (G::A + 2);
    float r, v;
    heads_value<G, 1>(hp + G::CS, false, t.hsc, r, v);
    for (int a = threadIdx.x; a < G::A; a += 64) o[a] = t.logits[a];
    if (threadIdx.x == 0) { o[G::A] = 0.f; o[G::A + 1] = v; }
  }
  const TreeView TV = TreeViewOf<G>::make(E, g);
  // injected Dirichlet samples (test hook): [G][A] (search) or [G][M][A] (self-play)
  const double* nz = noise ? noise + (size_t)g * game_stride + (per_move ? (size_t)E.meta[g * 4 + 3] * G::A : 0)
                           : nullptr;
  root_priors<G>(t, TV, sp, nz, T.key[g]);
  TreeAcc<G, false> acc(TV, t);
  tree_reset_root<G>(acc);
  if (threadIdx.x == 0) { E.nodes[g] = 1; T.simc[g] = 0; T.bq_n[g] = 0; }
}

// select_leaf for one simulation of every game -> the conv jobs
template <int N>
__global__ void __launch_bounds__(64) k_tselect(TowerArrays T, SearchParams sp, EngineArrays E) {
  typedef TGeo<N> G;
  const int g = blockIdx.x;
  if (!T.playing[g]) { if (threadIdx.x == 0) T.evalact[g] = 0; return; }
  __shared__ TreeLds<G> t;
  tload_mask<G>(t, T, g);
  const TreeView TV = TreeViewOf<G>::make(E, g);
  TreeAcc<G, false> acc(TV, t);
  const int sim = T.simc[g];
  const int a = select_leaf<G>(t, acc, sp, T.key[g], sim);
  if (a >= 0) {
    const int nid = E.nodes[g];
    if (threadIdx.x == 0) {
      const int base = g * (E.S + 1);
      T.in_idx[g] = base + t.leaf;
      T.out_idx[g] = base + nid;
      T.act[g] = a;
      T.job[g * 3] = t.leaf; T.job[g * 3 + 1] = t.depth; T.job[g * 3 + 2] = nid;
      T.evalact[g] = 1;
    }
  } else {
    // self_play.py: a terminal leaf backs up 0 (:188-191); main.py: nothing (:296)
    if (a == -1) backup<G>(acc, t.depth, -1, 0.0);
    if (threadIdx.x == 0) { T.evalact[g] = 0; T.simc[g] = sim + 1; }
  }
}

// heads -> the new node's child priors, reward / value -> backup (:198-230)
template <int N>
__global__ void __launch_bounds__(64) k_texpand(TowerArrays T, SearchParams sp, EngineArrays E) {
  typedef TGeo<N> G;
  const int g = blockIdx.x;
  if (!T.evalact[g]) return;
  __shared__ TreeLds<G> t;
  __shared__ float hp[3 * G::CS];
  tload_mask<G>(t, T, g);
  stage_head_scalars(T.hs, t.hsc);
  tsum_heads<G>(T, g, hp);
  const int leaf = T.job[g * 3], depth = T.job[g * 3 + 1], nid = T.job[g * 3 + 2], a = T.act[g];
  const TreeView TV = TreeViewOf<G>::make(E, g);
  TreeAcc<G, false> acc(TV, t);
  float r, v;
  heads_value<G, 1>(hp, true, t.hsc, r, v);
  float x[G::AP];
  logits_regs<G, 1>(hp, true, t.hsc, x);
  // lazy child priors (as the main engine's HBM trees): the new node's prior
  // row keeps its policy logits and its child row the sentinel kRawRow in
  // entry 0; select_leaf forms the priors (softmax x root mask, numpy-order
  // sum) and the -1 child row when a select first reaches the node -- most
  // leaves never are, so most softmaxes disappear from the simulation
  {
    float* prow = TV.prior + (size_t)nid * G::A;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < G::AP; ++j)
      if (lane + 64 * j < G::A) prow[lane + 64 * j] = x[j];
    if (lane == 0) TV.child[(size_t)nid * G::A] = kRawRow;
    if (T.node_out) {                     // (test hook) the node as the tower evaluated it
      float* o = T.node_out + ((size_t)g * (E.S + 1) + nid) * (G::A + 2);
#pragma unroll
      for (int j = 0; j < G::AP; ++j)
        if (lane + 64 * j < G::A) o[lane + 64 * j] = x[j];
      if (lane == 0) { o[G::A] = r; o[G::A + 1] = v; }
    }
  }
  if (threadIdx.x == 0) acc.init(nid);
  if (threadIdx.x == (a & 63)) acc.set_child(leaf, a, nid);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  backup<G>(acc, depth, nid, (double)r + sp.discount * (double)v, sp.variant == 0);
  if (threadIdx.x == 0) {
    E.nodes[g] = nid + 1;
    T.simc[g] += 1;
    atomicAdd(&E.counters[3], 1ull);      // towers evaluated
  }
}

// ---------------------------------------------------------------------------
// Batched simulation steps.  The tree stays the sequential one because
// every simulation still runs the real select on the real tree: k_tbatch
// commits a pending entry (leaf L_i, action a_i) only when the select asks
// for exactly that expansion as the next node id, and otherwise drops the
// batch's remaining entries and starts a new batch at the select's own leaf.
// A batch is a prediction of the next simulations' expansions:
//  * the root's children: while the root has unexpanded eligible children
//    every simulation picks one by its draw alone (random.choice,
//    self_play.py:283-287), no value involved -- so the first min(#eligible,
//    S) simulations are ONE batch per game, always committed whole;
//  * after that, each simulation's PUCT walk (:296-330) goes to the root
//    child of highest score, whose score then drops (its visit count rises:
//    the exploration term shrinks), so the next simulations are predicted by
//    replaying the root's choice with virtual visits -- q held at its current
//    mean, n and N raised by each predicted visit: entry k >= 1 is the root
//    child c that choice takes for simulation sim + k and the pick sim + k
//    would make there, the randbelow(draw(sim + k), n)-th of c's unexpanded
//    eligible children less those this batch already gave to c.  The batch
//    stops at a child with no unexpanded child left (the walk would go
//    deeper) or at cap_spec entries.
// Entry i's latent is written straight into node nid0 + i's pool slot, its
// logits into that node's prior row (the lazy kRawRow form of k_texpand): a
// committed entry is in place; a dropped one's slot and rows belong to the
// node that later takes its id, which overwrites them before any select can
// reach it.
// ---------------------------------------------------------------------------
constexpr int kSpecMax = 128;   // entries of a speculative (non-root) batch

template <int N>
__global__ void __launch_bounds__(64) k_tbatch(TowerArrays T, SearchParams sp, EngineArrays E, int cap_root,
                                               int cap_spec) {
  typedef TGeo<N> G;
  const int g = blockIdx.x;
  const int lane = threadIdx.x;
  if (!T.playing[g]) {
    if (lane == 0) { T.nbg[g] = 0; T.bq_n[g] = 0; }
    return;
  }
  __shared__ TreeLds<G> t;
  __shared__ int sl_leaf[kSpecMax], sl_act[kSpecMax];   // the batch being formed (LDS copy)
  tload_mask<G>(t, T, g);
  const TreeView TV = TreeViewOf<G>::make(E, g);
  TreeAcc<G, false> acc(TV, t);
  const uint64_t key = T.key[g];
  const int S = sp.num_simulations;
  int sim = T.simc[g], nodes = E.nodes[g];
  const int bn = T.bq_n[g], bnid0 = T.bq_nid0[g];
  int* const bact = T.bq_act + (size_t)g * T.bq_cap;
  int* const bleaf = T.bq_leaf + (size_t)g * T.bq_cap;
  const float* const brv = T.bq_rv + (size_t)g * T.bq_cap * 2;
  int next = 0, B = 0;
  while (sim < S) {
    const int a = select_leaf<G>(t, acc, sp, key, sim);
    if (a < 0) {
      // self_play.py: a terminal leaf backs up 0 (:188-191); main.py: nothing (:296)
      if (a == -1) backup<G>(acc, t.depth, -1, 0.0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ++sim;
      continue;
    }
    if (next < bn && nodes == bnid0 + next && t.leaf == __builtin_amdgcn_readfirstlane(bleaf[next]) &&
        a == __builtin_amdgcn_readfirstlane(bact[next])) {
      // the expansion this simulation asks for was evaluated: k_texpand's commit
      const float r = brv[2 * next], v = brv[2 * next + 1];
      if (lane == 0) acc.init(nodes);
      if (lane == (a & 63)) acc.set_child(t.leaf, a, nodes);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      backup<G>(acc, t.depth, nodes, (double)r + sp.discount * (double)v, sp.variant == 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      ++nodes;
      ++sim;
      ++next;
      continue;
    }
    const int room = S - sim;
    if (t.leaf == 0) {
      // the root's unexpanded children, in the order the draws take them
      B = t.nunexp < room ? t.nunexp : room;
      B = B < cap_root ? B : cap_root;
      PickSeq<G> ps(t.umask, t.nunexp, B, key, sim);
      for (int i = 0; i < B; ++i) {
        const int ai = ps.pick(i);
        if (lane == 0) { bact[i] = ai; bleaf[i] = 0; }
      }
    } else {
      // this simulation's expansion, then the next ones predicted by
      // replaying the root's PUCT choice with virtual visits
      if (lane == 0) { bact[0] = a; bleaf[0] = t.leaf; sl_leaf[0] = t.leaf; sl_act[0] = a; }
      B = 1;
      int lim = cap_spec < room ? cap_spec : room;
      lim = lim < kSpecMax ? lim : kSpecMax;
      if (lim > 1) {
        // the root children's stats, updated by each predicted visit: n (and
        // the root's N) + 1, and the child's q moved toward the mean q of the
        // root's children (the visit's value is unknown; a child chosen for
        // its high q tends to fall back: on the oracle's config-5 trees this
        // predicted 15 of the next 16 choices, against 11 with q held and 14
        // with the static ranking); puct_pick's formula on the
        // virtual statistics
        double P[G::AP], q[G::AP];
        int ch[G::AP], n[G::AP];
        uint64_t elig[G::AP];
#pragma unroll
        for (int j = 0; j < G::AP; ++j) {
          const int aa = lane + 64 * j;
          P[j] = aa < G::A ? TV.root_prior[aa] : 0.0;
          ch[j] = aa < G::A ? TV.child[aa] : -1;
        }
        double qsum = 0.0;
        int ne = 0;
#pragma unroll
        for (int j = 0; j < G::AP; ++j) {
          const bool e = P[j] > 0.0 && ch[j] >= 0;
          elig[j] = __ballot(e);
          n[j] = e ? TV.visits[ch[j]] : 0;
          const double w = e ? TV.wsum[ch[j]] : 0.0;
          q[j] = e && n[j] > 0 ? ddiv(w, (double)n[j]) : 0.0;
          if (e) { qsum += q[j]; ++ne; }
        }
        qsum = wave_sum(qsum);
        ne = (int)wave_sum((double)ne);
        const double qmean = ne > 0 ? qsum / ne : 0.0;
        int nvis = TV.visits[0];
        auto virtual_visit = [&](int act) {
#pragma unroll
          for (int j = 0; j < G::AP; ++j)
            if (lane + 64 * j == act) { q[j] = (q[j] * n[j] + qmean) / (double)(n[j] + 1); n[j] += 1; }
          ++nvis;
        };
        virtual_visit(t.ract);                      // this simulation's own visit
        while (B < lim) {
          double lo = INFINITY, hi = -INFINITY;
#pragma unroll
          for (int j = 0; j < G::AP; ++j)
            if ((elig[j] >> lane) & 1ull) { lo = fmin_(lo, q[j]); hi = fmax_(hi, q[j]); }
          wave_minmax(lo, hi);
          const double sq = dsqrt((double)(sp.variant == 1 ? nvis + 1 : (nvis > 1 ? nvis : 1)));
          double best = -INFINITY;
          double sc[G::AP];
#pragma unroll
          for (int j = 0; j < G::AP; ++j) {
            sc[j] = -INFINITY;
            if ((elig[j] >> lane) & 1ull) {
              const double qn = hi > lo ? ddiv(q[j] - lo, hi - lo) : q[j];
              sc[j] = qn + ddiv((sp.c_puct * P[j]) * sq, (double)(1 + n[j]));
            }
            best = sc[j] > best ? sc[j] : best;
          }
          best = wave_max(best);
          if (!(best > -INFINITY)) break;
          int ca = -1, c = -1;
#pragma unroll
          for (int j = 0; j < G::AP; ++j) {
            const uint64_t hit = __ballot(sc[j] == best);
            if (ca < 0 && hit) {
              const int l = __ffsll((long long)hit) - 1;
              ca = 64 * j + l;
              c = __builtin_amdgcn_readlane(ch[j], l);
            }
          }
          // c's unexpanded eligible children (prior > 0, child -1: select's
          // test), less the ones this batch already gave to c.  A row still
          // in the lazy kRawRow form is settled here, exactly as select_leaf
          // settles it on its first arrival (the priors depend on the logits
          // and the root mask alone, so settling early changes nothing)
          int* crow = TV.child + (size_t)c * G::A;
          float* prow = TV.prior + (size_t)c * G::A;
          float pr[G::AP];
          int cr[G::AP];
#pragma unroll
          for (int j = 0; j < G::AP; ++j) {
            const int aa = lane + 64 * j;
            pr[j] = aa < G::A ? prow[aa] : 0.f;
            cr[j] = aa < G::A ? crow[aa] : 0;
          }
          if (__builtin_amdgcn_readfirstlane(cr[0]) == kRawRow) {
            float qq[G::AP];
            child_prior_regs<G>(t, pr, qq, sp.variant, t.fbuf, t.dbuf);
#pragma unroll
            for (int j = 0; j < G::AP; ++j) {
              const int aa = lane + 64 * j;
              if (aa < G::A) { prow[aa] = qq[j]; crow[aa] = -1; }
              pr[j] = qq[j];
              cr[j] = -1;
            }
          }
          bool taken[G::AP];
#pragma unroll
          for (int j = 0; j < G::AP; ++j) taken[j] = false;
          for (int e = 0; e < B; ++e)
            if (sl_leaf[e] == c) {
              const int ae = sl_act[e];
#pragma unroll
              for (int j = 0; j < G::AP; ++j) taken[j] |= lane + 64 * j == ae;
            }
          uint64_t un[G::AP];
          int nun = 0;
#pragma unroll
          for (int j = 0; j < G::AP; ++j) {
            const int aa = lane + 64 * j;
            un[j] = __ballot(aa < G::A && pr[j] > 0.f && cr[j] < 0 && !taken[j]);
            nun += __popcll(un[j]);
          }
          if (nun == 0) break;                     // c is fully expanded: the walk would go deeper
          uint32_t k = randbelow(draw(key, TAG_SELECT, (uint64_t)(sim + B)), (uint32_t)nun);
          int pick = -1;
#pragma unroll
          for (int j = 0; j < G::AP; ++j) {
            const uint32_t cnt = __popcll(un[j]);
            if (pick < 0 && k < cnt) pick = 64 * j + kth_set_bit(un[j], k);
            else if (pick < 0) k -= cnt;
          }
          if (lane == 0) { bact[B] = pick; bleaf[B] = c; sl_leaf[B] = c; sl_act[B] = pick; }
          wave_lds_sync();
          ++B;
          virtual_visit(ca);
        }
      }
    }
    if (lane == 0) T.bq_nid0[g] = nodes;
    break;
  }
  if (lane == 0) {
    T.bq_n[g] = B;
    T.nbg[g] = B;
    T.simc[g] = sim;
    E.nodes[g] = nodes;
  }
}

// This step's boards of all games, in game order (one block): board
// off[g] + i = game g's entry i; the count to b_total, and to counters[3]
// (towers evaluated).
template <int N>
__global__ void __launch_bounds__(256) k_tboards(TowerArrays T, EngineArrays E, int G) {
  __shared__ int part[256];
  const int tid = threadIdx.x;
  // per-thread sums of a contiguous range of games, then an exclusive scan
  const int per = (G + 255) / 256;
  int s = 0;
  for (int k = 0; k < per; ++k) {
    const int g = tid * per + k;
    if (g < G) s += T.nbg[g];
  }
  part[tid] = s;
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int i = 0; i < 256; ++i) { const int v = part[i]; part[i] = acc; acc += v; }
    *T.b_total = acc;
    if (acc > 0) atomicAdd(&E.counters[3], (unsigned long long)acc);
  }
  __syncthreads();
  int o = part[tid];
  for (int k = 0; k < per; ++k) {
    const int g = tid * per + k;
    if (g >= G) break;
    const int nb = T.nbg[g];
    const int base = g * (E.S + 1);
    const int nid0 = nb > 0 ? T.bq_nid0[g] : 0;
    for (int i = 0; i < nb; ++i) {
      const int b = o + i;
      T.b_in[b] = base + T.bq_leaf[(size_t)g * T.bq_cap + i];
      T.b_out[b] = base + nid0 + i;
      T.b_act[b] = T.bq_act[(size_t)g * T.bq_cap + i];
      T.b_game[b] = g;
      T.b_ent[b] = i;
    }
    o += nb;
  }
}

// heads of this step's boards (one wave per board): the entry's reward and
// value for the commit, its logits into node nid0 + i's prior row (kRawRow:
// select_leaf forms the priors on its first arrival, as after k_texpand)
template <int N>
__global__ void __launch_bounds__(64) k_tbexpand(TowerArrays T, SearchParams sp, EngineArrays E) {
  typedef TGeo<N> G;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  __shared__ float hp[3 * G::CS];
  __shared__ float hsc[64];
  stage_head_scalars(T.hs, hsc);
  tsum_heads<G>(T, b, hp);
  const int g = T.b_game[b], i = T.b_ent[b];
  const int nid = T.b_out[b] - g * (E.S + 1);
  float r, v;
  heads_value<G, 1>(hp, true, hsc, r, v);
  float x[G::AP];
  logits_regs<G, 1>(hp, true, hsc, x);
  const TreeView TV = TreeViewOf<G>::make(E, g);
  float* prow = TV.prior + (size_t)nid * G::A;
#pragma unroll
  for (int j = 0; j < G::AP; ++j)
    if (lane + 64 * j < G::A) prow[lane + 64 * j] = x[j];
  if (lane == 0) {
    TV.child[(size_t)nid * G::A] = kRawRow;
    T.bq_rv[((size_t)g * T.bq_cap + i) * 2] = r;
    T.bq_rv[((size_t)g * T.bq_cap + i) * 2 + 1] = v;
  }
  if (T.node_out) {                       // (test hook) the node as the tower evaluated it
    float* o = T.node_out + ((size_t)g * (E.S + 1) + nid) * (G::A + 2);
#pragma unroll
    for (int j = 0; j < G::AP; ++j)
      if (lane + 64 * j < G::A) o[lane + 64 * j] = x[j];
    if (lane == 0) { o[G::A] = r; o[G::A + 1] = v; }
  }
}

// action choice, record, board step (self_play.py:465-507), as k_selfplay_move's tail
template <int N>
__global__ void __launch_bounds__(64) k_tchoose(TowerArrays T, SearchParams sp, PlayParams pp, EngineArrays E) {
  typedef TGeo<N> G;
  const int g = blockIdx.x;
  if (!T.playing[g]) return;
  __shared__ TreeLds<G> t;
  __shared__ int8_t stone[G::CELLS];
  __shared__ uint8_t invd[G::CELLS];
  __shared__ int label[G::CELLS], libs[G::CELLS], gsize[G::CELLS];
  __shared__ int killed[4], misc[8];
  tload_mask<G>(t, T, g);
  for (int c = threadIdx.x; c < G::CELLS; c += 64) {
    stone[c] = E.stones[(size_t)g * G::CELLS + c];
    invd[c] = E.invd[(size_t)g * G::CELLS + c];
  }
  BoardMeta m;
  const int* mm = E.meta + g * 4;
  m.turn = mm[0]; m.passed = mm[1]; m.done = mm[2]; m.moves = mm[3];
  const int mv = m.moves;
  const size_t rec = (size_t)g * E.max_moves + mv;
  const TreeView TV = TreeViewOf<G>::make(E, g);
  const uint64_t key = T.key[g];
  const double temp = mv < pp.temperature_moves ? pp.temperature : 0.0;
  const int a = sp.variant == 1 ? choose_action_main<G>(t, TV, key, E.rec_policy + rec * G::A)
                                : choose_action<G>(t, TV, sp.compat, temp, key, E.rec_policy + rec * G::A);
  if (threadIdx.x == 0) {
    E.rec_action[rec] = a;
    const int n = TV.visits[0];
    E.rec_value[rec] = n > 0 ? TV.wsum[0] / (double)n : 0.0;
  }
  __syncthreads();
  BoardLds<G> bl;
  bl.stone = stone; bl.invd = invd; bl.label = label; bl.libs = libs; bl.gsize = gsize;
  bl.killed = killed; bl.misc = misc;
  const int st = board_step<G>(bl, m, a);
  __syncthreads();
  double w = 0.0;
  if (st == BOARD_OK && m.done) w = board_winning<G>(bl, pp.komi);
  for (int c = threadIdx.x; c < G::CELLS; c += 64) {
    E.stones[(size_t)g * G::CELLS + c] = stone[c];
    E.invd[(size_t)g * G::CELLS + c] = invd[c];
  }
  if (threadIdx.x == 0) {
    int* mw = E.meta + g * 4;
    mw[0] = m.turn; mw[1] = m.passed; mw[2] = m.done; mw[3] = m.moves;
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
}

// search API end: every prior row a select never reached (lazy, k_texpand)
// turned into priors, so exported trees are complete (as k_search's
// settle_all_priors); then the root visits / value
template <int N>
__global__ void __launch_bounds__(64) k_tsearch_out(TowerArrays T, SearchParams sp, EngineArrays E, int* out_visits,
                                                    double* out_value) {
  typedef TGeo<N> G;
  const int g = blockIdx.x;
  __shared__ TreeLds<G> t;
  tload_mask<G>(t, T, g);
  const TreeView TV = TreeViewOf<G>::make(E, g);
  const int lane = threadIdx.x & 63, nodes = E.nodes[g];
  for (int n = 1; n < nodes; ++n) {
    int* crow = TV.child + (size_t)n * G::A;
    if (__builtin_amdgcn_readfirstlane(crow[0]) != kRawRow) continue;
    float* prow = TV.prior + (size_t)n * G::A;
    float x[G::AP], q[G::AP];
#pragma unroll
    for (int j = 0; j < G::AP; ++j) x[j] = lane + 64 * j < G::A ? prow[lane + 64 * j] : 0.f;
    child_prior_regs<G>(t, x, q, sp.variant, t.fbuf, t.dbuf);
#pragma unroll
    for (int j = 0; j < G::AP; ++j)
      if (lane + 64 * j < G::A) { prow[lane + 64 * j] = q[j]; crow[lane + 64 * j] = -1; }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  search_outputs<G>(E, g, out_visits, out_value);
}

// ---------------------------------------------------------------------------
// Drop-in inference plumbing: f32 NCHW <-> bf16 chunked boards, heads.
// ---------------------------------------------------------------------------
// latent f32 [B][C][N][N] -> boards (C channels); obs f32 [B][6][N][N] ->
// one 64-channel chunk (6 planes + zeros) when obs6
template <int N>
__global__ void __launch_bounds__(256) k_tin(const float* __restrict__ src, bf16* dst, int C, int obs6,
                                             long long dst_stride) {
  typedef TGeo<N> G;
  const int b = blockIdx.x;
  const int CC = obs6 ? 1 : C / 64, CIN = obs6 ? 6 : C;
  const float* s = src + (size_t)b * CIN * G::CELLS;
  bf16* d = dst + (size_t)b * dst_stride;
  for (int i = threadIdx.x; i < CC * G::CELLS * 8; i += 256) {
    const int cc = i / (G::CELLS * 8), r = i - cc * G::CELLS * 8;
    const int p = r >> 3, j = r & 7;
    const int y = p / N, x = p - y * N;
    const int q = (y + 1) * G::W + (x + 1);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = cc * 64 + j * 8 + k;
      o[k] = (bf16)(c < CIN ? s[(size_t)c * G::CELLS + p] : 0.f);
    }
    *reinterpret_cast<bf16x8*>(d + (size_t)cc * G::P * 64 + tpix(q, j)) = o;
  }
}

template <int N>
__global__ void __launch_bounds__(256) k_tout(const bf16* __restrict__ src, float* dst, int C) {
  typedef TGeo<N> G;
  const int b = blockIdx.x;
  const int CC = C / 64;
  const bf16* s = src + (size_t)b * CC * G::P * 64;
  float* d = dst + (size_t)b * C * G::CELLS;
  for (int i = threadIdx.x; i < CC * G::CELLS * 8; i += 256) {
    const int cc = i / (G::CELLS * 8), r = i - cc * G::CELLS * 8;
    const int p = r >> 3, j = r & 7;
    const int y = p / N, x = p - y * N;
    const int q = (y + 1) * G::W + (x + 1);
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(s + (size_t)cc * G::P * 64 + tpix(q, j));
#pragma unroll
    for (int k = 0; k < 8; ++k) d[(size_t)(cc * 64 + j * 8 + k) * G::CELLS + p] = (float)v[k];
  }
}

template <int N>
__global__ void __launch_bounds__(64) k_theads(TowerArrays T, int has_reward, float* reward, float* value,
                                               float* logits) {
  typedef TGeo<N> G;
  const int b = blockIdx.x;
  __shared__ float hp[3 * G::CS];
  __shared__ float hsc[64];
  stage_head_scalars(T.hs, hsc);
  tsum_heads<G>(T, b, hp);
  const float* h = has_reward ? hp : hp + G::CS;
  float r, v;
  heads_value<G, 1>(h, has_reward != 0, hsc, r, v);
  heads_logits<G, 1>(h, has_reward != 0, hsc, logits + (size_t)b * G::A);
  if (threadIdx.x == 0) {
    value[b] = v;
    if (has_reward) reward[b] = r;
  }
}

}  // namespace mzgo

// mzgo_conv.hpp -- 3x3/pad-1 convolution of one board on one workgroup, on
// fp32 MFMA (v_mfma_f32_16x16x4_f32), with the MuZero heads fused into the
// epilogue.
//
// Implicit GEMM, transposed so the epilogue's head reductions run over the
// accumulator's row index:
//     out[cout][cell] = sum_k W[cout][k] * im2col[k][cell],  k = tap*CINP + cin
// A operand (16 couts x 4 k)  : pre-packed weights streamed from L2
//                               (layout written by pack_conv_weights, host side)
// B operand (4 k x 16 cells)  : the input board staged in LDS as [cin][CPAD],
//                               gathered per lane with the tap's cell offset
// Each wave owns jobs of MG cout tiles x NG cell tiles (3x3 tiles of 16x16 at
// C=96) so every A and B fragment feeds 3 MFMAs.
//
// Replaces the torch conv2d calls of self_play.py:66-74 (representation),
// :80/:90 (dynamics) and the 1x1 head convs of :81, :100, :102.
#pragma once
#include "mzgo_common.hpp"

namespace mzgo {

// cout tiles per wave job for a conv with COUT outputs
template <int COUT>
struct ConvShape {
  static constexpr int MT = COUT / 16;
  static constexpr int MG = (MT % 3 == 0) ? 3 : ((MT % 4 == 0 && MT >= 8) ? 4 : 2);
  static constexpr int MGP = (MG == 3) ? 4 : MG;  // packed floats per lane per k-step
  static constexpr int NCOG = MT / MG;            // cout groups
  static_assert(MT % MG == 0, "cout tiles");
};

template <int MGP>
struct WFrag;
template <> struct WFrag<2> { typedef float2 T; };
template <> struct WFrag<4> { typedef float4 T; };

__device__ __forceinline__ float frag_get(const float2& v, int i) { return i == 0 ? v.x : v.y; }
__device__ __forceinline__ float frag_get(const float4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// Stage ``nch`` channels of a board held as [ch][src_stride] (f32, global) into
// LDS [ch][CPAD]; optionally add emb[ch] to every cell (the action embedding
// broadcast-add of self_play.py:87-89).  When src_stride == CS the copy moves
// whole 16-byte chunks (pad cells included; the conv never reads them).
template <class G>
__device__ __forceinline__ void stage_board(float* __restrict__ lds, const float* __restrict__ src,
                                   int src_stride, int nch, const float* __restrict__ emb) {
  if (src_stride == G::CS) {
    constexpr int Q = G::CS / 4;
    const float4* s4 = reinterpret_cast<const float4*>(src);
    for (int i = tid_local(); i < nch * Q; i += G::THREADS) {
      int c = i / Q, q = i - c * Q;
      float4 v = s4[c * Q + q];
      if (emb) {
        const float e = emb[c];
        // cells >= N*N are pad: keep them 0 (the zero slot of conv3x3_ring)
        const int j0 = q * 4;
        v.x = j0 + 0 < G::CELLS ? v.x + e : 0.f;
        v.y = j0 + 1 < G::CELLS ? v.y + e : 0.f;
        v.z = j0 + 2 < G::CELLS ? v.z + e : 0.f;
        v.w = j0 + 3 < G::CELLS ? v.w + e : 0.f;
      }
      *reinterpret_cast<float4*>(lds + c * G::CPAD + q * 4) = v;
    }
  } else {
    for (int i = tid_local(); i < nch * G::CELLS; i += G::THREADS) {
      int c = i / G::CELLS, j = i - c * G::CELLS;
      float v = src[c * src_stride + j];
      if (emb) v += emb[c];
      lds[c * G::CPAD + j] = v;
    }
    for (int c = tid_local(); c < nch; c += G::THREADS) lds[c * G::CPAD + G::CELLS] = 0.f;
  }
}

// Cell N*N of every staged LDS row is 0 (the "zero slot"): invalid taps of
// conv3x3_ring read it instead of being masked with v_cndmask.  Pooled
// latents (stride CS) keep 0 in their pad cells, so the 16-byte staging copy
// carries it (and the emb add skips pad cells); the scalar path writes it.
static_assert(Geo<9, 96>::CELLS < Geo<9, 96>::CS && Geo<19, 96>::CELLS < Geo<19, 96>::CS &&
              Geo<5, 96>::CELLS < Geo<5, 96>::CS && Geo<6, 96>::CELLS < Geo<6, 96>::CS,
              "every supported board has a pad cell to serve as the zero slot");

// Zero channels [c0, c1) of an LDS board (input padding of conv1: 6 -> 8 ch).
template <class G>
__device__ __forceinline__ void zero_channels(float* lds, int c0, int c1) {
  for (int i = tid_local(); i < (c1 - c0) * G::CPAD; i += G::THREADS) lds[c0 * G::CPAD + i] = 0.f;
}

// Head accumulation target: hp[cog][h][cell] in LDS, summed in fixed order later.
template <class G>
struct HeadPart {
  float* base;  // [2][3][CS]
  __device__ float* at(int cog, int h) const { return base + (cog * 3 + h) * G::CS; }
};

// The convolution with A fragments loaded straight from global memory (used
// for representation.conv1, K = 72, where a weight ring does not pay).
// lds_in: [CINP][CPAD] staged input.  wpk: packed weights.
// out: [COUT][out_stride] (global), cells >= out_cells are not stored.
// NH heads (0..3): head_w[h*COUT + cout]; partial sums land in hp.
// NGJ: 16-cell tiles per wave job (default the geometry's; conv1 passes 1 so
// that its (cout group, cell tile) jobs cover every wave).
template <class G, int CIN, int COUT, int NH, int NGJ = G::NG>
__device__ __forceinline__ void conv3x3_direct(const float* __restrict__ lds_in, const float* __restrict__ wpk,
                               const float* __restrict__ bias, float* __restrict__ out,
                               int out_stride, int out_cells, const float* __restrict__ head_w,
                               HeadPart<G> hp) {
  typedef ConvShape<COUT> S;
  constexpr int CINP = (CIN + 3) / 4 * 4;
  constexpr int CQ = CINP / 4;                 // k-steps per tap
  constexpr int KS = 9 * CQ;                   // k-steps
  constexpr int MG = S::MG, MGP = S::MGP, NG = NGJ;
  constexpr int JOBS = S::NCOG * ((G::CT + NG - 1) / NG);
  // A-fragment prefetch ring depth: the whole weight stream of a job when it
  // is short (conv1: 18 k-steps -- one memory latency instead of one per
  // k-step), else 4 or 2 k-steps ahead
  constexpr int PF = (9 * CQ * S::MGP <= 48) ? 9 * CQ : ((CQ % 4 == 0) ? 4 : 2);
  constexpr int WSTEP = S::NCOG * 64 * MGP;    // floats per k-step in the packed weights
  static_assert(CQ % PF == 0 || PF == 9 * CQ, "ring depth must divide the k-steps of a tap");
  static_assert(NH == 0 || S::NCOG == 2, "head partials assume two cout groups");
  typedef typename WFrag<MGP>::T wfrag;

  const int lane = lane_id_local();
  const int wave = wave_id();
  const int kq = lane >> 4;       // k row of this lane inside a k-step (B operand)
  const int col = lane & 15;      // cell column of this lane (B operand / accumulator)

  for (int job = wave; job < JOBS; job += G::WAVES) {
    const int cog = job % S::NCOG;
    const int cg = job / S::NCOG;

    // cell and (row, col) of this lane's column in each of the NG cell tiles
    int cy[NG], cx[NG];
    bool live[NG];
#pragma unroll
    for (int ni = 0; ni < NG; ++ni) {
      int j = (cg * NG + ni) * 16 + col;
      live[ni] = j < G::CELLS;
      cy[ni] = j / G::N;
      cx[ni] = j - cy[ni] * G::N;
    }

    f32x4 acc[MG][NG];
#pragma unroll
    for (int mi = 0; mi < MG; ++mi)
#pragma unroll
      for (int ni = 0; ni < NG; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

    const wfrag* wp = reinterpret_cast<const wfrag*>(wpk) + (cog * 64 + lane);
    constexpr int WSTEP_F = WSTEP / MGP;  // in wfrag units
    wfrag ring[PF];
#pragma unroll
    for (int p = 0; p < (PF == KS ? PF : PF - 1); ++p) ring[p] = wp[p * WSTEP_F];

#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3 - 1, dx = t - (t / 3) * 3 - 1;
      int off[NG];
      bool ok[NG];
#pragma unroll
      for (int ni = 0; ni < NG; ++ni) {
        int yy = cy[ni] + dy, xx = cx[ni] + dx;
        ok[ni] = live[ni] && yy >= 0 && yy < G::N && xx >= 0 && xx < G::N;
        off[ni] = ok[ni] ? yy * G::N + xx : 0;
      }
      const float* lrow = lds_in + kq * G::CPAD;
#pragma unroll
      for (int c4 = 0; c4 < CQ; ++c4) {
        const int s = t * CQ + c4;
        // prefetch the weights PF-1 k-steps ahead (a linear stream)
        const int sp = s + PF - 1;
        if (PF < KS && sp < KS) ring[(s + PF - 1) % PF] = wp[sp * WSTEP_F];
        float b[NG];
#pragma unroll
        for (int ni = 0; ni < NG; ++ni) {
          float v = lrow[(c4 * 4) * G::CPAD + off[ni]];
          b[ni] = ok[ni] ? v : 0.f;
        }
        const wfrag a = ring[s % PF];
#pragma unroll
        for (int mi = 0; mi < MG; ++mi) {
          const float am = frag_get(a, mi);
#pragma unroll
          for (int ni = 0; ni < NG; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(am, b[ni], acc[mi][ni], 0, 0, 0);
        }
      }
    }

    // ---- epilogue: bias + ReLU, store, fused 1x1 heads ----
    float hsum[NH > 0 ? NH : 1][NG];
#pragma unroll
    for (int h = 0; h < (NH > 0 ? NH : 1); ++h)
#pragma unroll
      for (int ni = 0; ni < NG; ++ni) hsum[h][ni] = 0.f;

#pragma unroll
    for (int mi = 0; mi < MG; ++mi) {
      const int cout0 = (cog * MG + mi) * 16 + kq * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cout0 + r;
        const float bb = bias[co];
        float hw[NH > 0 ? NH : 1];
#pragma unroll
        for (int h = 0; h < NH; ++h) hw[h] = head_w[h * COUT + co];
#pragma unroll
        for (int ni = 0; ni < NG; ++ni) {
          float v = acc[mi][ni][r] + bb;
          v = v > 0.f ? v : 0.f;
          const int cell = (cg * NG + ni) * 16 + col;
          v = cell < G::CELLS ? v : 0.f;                    // pad cells stay 0 (zero slot)
          if (out != nullptr && cell < out_cells) out[co * out_stride + cell] = v;
#pragma unroll
          for (int h = 0; h < NH; ++h) hsum[h][ni] = __builtin_fmaf(hw[h], v, hsum[h][ni]);
        }
      }
    }
    if constexpr (NH > 0) {
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int ni = 0; ni < NG; ++ni) {
          float v = hsum[h][ni];
          v += __shfl_xor(v, 16);
          v += __shfl_xor(v, 32);
          const int cell = (cg * NG + ni) * 16 + col;
          if (kq == 0 && cell < G::CS) hp.at(cog, h)[cell] = v;
        }
    }
  }
}

// ---------------------------------------------------------------------------
// The main convolution: each wave streams ITS OWN cout group's weights
// global -> LDS by DMA (global_load_lds_dwordx4) into a private NSLOT-slot
// ring, so the k-loop has no workgroup barrier at all -- only per-wave
// s_waitcnt vmcnt (MI355X guide: LDS-DMA data is visible to the issuing wave
// after its own vmcnt wait).  Both MFMA operands come from LDS.  One wave
// serves one cout group and JW cell groups, so each A fragment feeds
// MG x NG x JW MFMAs.  Weights are packed cog-major ([cog][k-step][lane][MGP],
// pack_conv(..., cog_major=true)) so a wave's stream is contiguous.
//
//   wave chunk c (KC k-steps, SLOT bytes) lands in slot c % NSLOT.
//   iteration c: issue chunk c+NSLOT-1 (into the slot read in iteration c-1)
//   -> wait until chunk c landed -> compute chunk c.
// ---------------------------------------------------------------------------
template <class G, int COUT>
struct Ring {
  typedef ConvShape<COUT> S;
  static constexpr int KSTEP_BYTES = 64 * S::MGP * 4;       // one cog, one k-step (1 KiB or 512 B)
  static constexpr int JPW = 4 / S::NCOG;                   // waves of one k-half sharing a cout group
  static constexpr int JW = (G::NCG + JPW - 1) / JPW;       // cell-group jobs per wave
  static constexpr int KC = JW >= 2 ? (1024 / KSTEP_BYTES)  // k-steps per chunk
                                    : (G::KSPLIT == 2 ? 4096 / KSTEP_BYTES : 8);
  static constexpr int NSLOT = JW >= 2 ? 2 : 3;
  static constexpr int SLOT = KC * KSTEP_BYTES;             // bytes per slot (multiple of 1 KiB)
  static constexpr int NGLDS = SLOT / 1024;                 // DMA instructions per chunk
  static_assert(4 % S::NCOG == 0, "a k-half's 4 waves must split evenly over cout groups");
  static_assert(SLOT % 1024 == 0, "slots are whole 1-KiB DMA pieces");
};

template <class G>
struct RingBytes {
  static constexpr int a = Ring<G, 64>::NSLOT * Ring<G, 64>::SLOT;
  static constexpr int b = Ring<G, G::C>::NSLOT * Ring<G, G::C>::SLOT;
  static constexpr int value = G::WAVES * (a > b ? a : b);  // all waves' private rings
};

// 16 bytes per lane global -> LDS (global_load_lds_dwordx4).  Issued from
// inline asm so that hipcc neither counts it nor guards every later ds_read
// with s_waitcnt vmcnt(0) (it cannot tell which LDS bytes the DMA writes);
// completion is tracked by hand with wait_vmcnt<N>() (MI355X guide §5.7).
// lds_dst must be wave-uniform; the LDS destination is lds_dst + lane*16.
__device__ __forceinline__ void dma16(const void* g, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds_dst)
      : "memory");
}

// dma16 with sc1 (agent scope): the read misses this CU's L1 and is served by
// the XCC's L2, so it sees what other CUs of the XCC stored there since
// (k_tconv_chain's same-XCC layer hand-offs).  Until round 6 this was `sc0`,
// which is WORKGROUP scope: an sc0 load hits L1 like a plain one and could
// return a line cached before a sibling CU rewrote it (tools/l1_visibility_probe,
// DESIGN.md §7).  Same speed: config 5 1526.7-1528.1 ms per move with sc1,
// 1528.0-1528.2 with sc0, 1527.5-1528.6 with "sc0 sc1", 1533-1534 with nt
// (profiles/r6b_patch_policy_ab.txt, one call).
__device__ __forceinline__ void dma16_l2(const void* g, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off sc1\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds_dst)
      : "memory");
}

// 4 bytes per lane (LDS destination base + lane*4): an L2 prefetch whose data
// lands in a dummy LDS area
__device__ __forceinline__ void dma4(const void* g, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(lds_dst)
      : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// s_barrier after this wave's LDS accesses completed (raw: no vmcnt drain, so
// LDS-DMA requests stay in flight across it)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 63]
__device__ __forceinline__ void wait_vmcnt_dyn(int n) {
  switch (n) {
#define MZGO_W(k) case k: wait_vmcnt<k>(); break;
    MZGO_W(0) MZGO_W(1) MZGO_W(2) MZGO_W(3) MZGO_W(4) MZGO_W(5) MZGO_W(6) MZGO_W(7) MZGO_W(8) MZGO_W(9)
    MZGO_W(10) MZGO_W(11) MZGO_W(12) MZGO_W(13) MZGO_W(14) MZGO_W(15) MZGO_W(16) MZGO_W(17) MZGO_W(18)
    MZGO_W(19) MZGO_W(20) MZGO_W(21) MZGO_W(22) MZGO_W(23) MZGO_W(24) MZGO_W(25) MZGO_W(26) MZGO_W(27)
    MZGO_W(28) MZGO_W(29) MZGO_W(30) MZGO_W(31)
#undef MZGO_W
    default: wait_vmcnt<0>(); break;
  }
}


template <int MGP>
__device__ __forceinline__ typename WFrag<MGP>::T lds_frag(const float* p) {
  return *reinterpret_cast<const typename WFrag<MGP>::T*>(p);
}

// hp_lds: head partials [2][3][CS]; written after a workgroup barrier, so it
// may alias lds_in.  Returns with all waves synchronised.
template <class G, int CIN, int COUT, int NH, bool YM = false>
__device__ __forceinline__ void conv3x3_ring(const float* lds_in, float* ring, const float* __restrict__ wpk,
                                    const float* __restrict__ bias, float* __restrict__ out,
                                    int out_stride, int out_cells, const float* __restrict__ head_w,
                                    float* hp_lds, Stamp* st = nullptr) {
  typedef ConvShape<COUT> S;
  typedef Ring<G, COUT> R;
  constexpr int CINP = (CIN + 3) / 4 * 4;
  constexpr int CQ = CINP / 4;
  constexpr int KSPLIT = G::KSPLIT;
  constexpr int CQH = CQ / KSPLIT;                // channel quads of one k-half per tap
  constexpr int KSH = 9 * CQH;                    // k-steps per wave
  constexpr int KC = R::KC, NCH = KSH / KC, JW = R::JW, NG = G::NG, MG = S::MG, MGP = S::MGP;
  constexpr int NSLOT = R::NSLOT;
  static_assert(CQ % KSPLIT == 0 && CQH % KC == 0, "a chunk must not straddle two taps");
  static_assert(NH == 0 || S::NCOG == 2, "head partials assume two cout groups");
  typedef typename WFrag<MGP>::T wfrag;

  const int lane = lane_id_local();
  const int wave = __builtin_amdgcn_readfirstlane(wave_id());   // scalar: uniform branches
  const int half = wave / 4, wl = wave % 4;                      // k-half, wave within the half
  const int kq = lane >> 4, col = lane & 15;
  const int cog = wl % S::NCOG;
  const int cg0 = wl / S::NCOG;
  // this wave's contiguous weight stream ([cog][half][tap][c4'] order) and private ring
  const char* wsrc = reinterpret_cast<const char*>(wpk) + (size_t)(cog * KSPLIT + half) * KSH * R::KSTEP_BYTES +
                     lane * 16;
  float* myring = ring + wave * (RingBytes<G>::value / G::WAVES / 4);
  const uint32_t ring0 = __builtin_amdgcn_readfirstlane(lds_addr(myring));

  // every job of every wave covers a real cell group unless NCG % JPW != 0
  // (5x5, 6x6: JW == 1 and the second pair of waves has no cells)
  constexpr bool ALL_LIVE = G::NCG % R::JPW == 0;
  static_assert(ALL_LIVE || JW == 1, "partial job sets only with one job per wave");
  const bool active = ALL_LIVE || cg0 < G::NCG;                // scalar

  int cy[JW][NG], cx[JW][NG];
  bool live[JW][NG];
#pragma unroll
  for (int j = 0; j < JW; ++j)
#pragma unroll
    for (int ni = 0; ni < NG; ++ni) {
      const int cell = ((cg0 + j * R::JPW) * NG + ni) * 16 + col;
      live[j][ni] = cell < G::CELLS;
      cy[j][ni] = cell / G::N;
      cx[j][ni] = cell - cy[j][ni] * G::N;
    }

  f32x4 acc[JW][MG][NG];
#pragma unroll
  for (int j = 0; j < JW; ++j)
#pragma unroll
    for (int mi = 0; mi < MG; ++mi)
#pragma unroll
      for (int ni = 0; ni < NG; ++ni) acc[j][mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (active) {
    auto issue = [&](int c) {
#pragma unroll
      for (int p = 0; p < R::NGLDS; ++p)
        dma16(wsrc + (size_t)c * R::SLOT + p * 1024, ring0 + (uint32_t)((c % NSLOT) * R::SLOT + p * 1024));
    };
#pragma unroll
    for (int c = 0; c < NSLOT - 1; ++c)
      if (c < NCH) issue(c);
    int off[JW][NG];
    for (int c = 0; c < NCH; ++c) {
      if (c + NSLOT - 1 < NCH) {
        issue(c + NSLOT - 1);
        wait_vmcnt<R::NGLDS * (NSLOT - 1)>();
      } else {
        wait_vmcnt<0>();
      }
      const int s0 = c * KC;
      const int t = s0 / CQH;
      const int c4h = s0 - t * CQH;
      const int c40 = half * CQH + c4h;           // channel quad of this chunk's first k-step
      if (c4h == 0) {
        const int dy = t / 3 - 1, dx = t - (t / 3) * 3 - 1;
#pragma unroll
        for (int j = 0; j < JW; ++j)
#pragma unroll
          for (int ni = 0; ni < NG; ++ni) {
            const int yy = cy[j][ni] + dy, xx = cx[j][ni] + dx;
            const bool ok = live[j][ni] && yy >= 0 && yy < G::N && xx >= 0 && xx < G::N;
            off[j][ni] = ok ? yy * G::N + xx : G::CELLS;      // zero slot
          }
      }
      const float* slot = myring + (c % NSLOT) * (R::SLOT / 4) + lane * MGP;
      const float* lrow = lds_in + (c40 * 4 + kq) * G::CPAD;
      // operands of k-step kk+1 are fetched before the MFMAs of k-step kk
      // (one wave per SIMD: LDS latency must hide behind this wave's MFMAs)
      wfrag a_nx = lds_frag<MGP>(slot);
      float b_nx[JW][NG];
#pragma unroll
      for (int j = 0; j < JW; ++j)
#pragma unroll
        for (int ni = 0; ni < NG; ++ni) b_nx[j][ni] = lrow[off[j][ni]];
#pragma unroll
      for (int kk = 0; kk < KC; ++kk) {
        const wfrag a = a_nx;
        float b[JW][NG];
#pragma unroll
        for (int j = 0; j < JW; ++j)
#pragma unroll
          for (int ni = 0; ni < NG; ++ni) b[j][ni] = b_nx[j][ni];
        if (kk + 1 < KC) {
          a_nx = lds_frag<MGP>(slot + (kk + 1) * 64 * MGP);
#pragma unroll
          for (int j = 0; j < JW; ++j)
#pragma unroll
            for (int ni = 0; ni < NG; ++ni) b_nx[j][ni] = lrow[(kk + 1) * 4 * G::CPAD + off[j][ni]];
        }
#pragma unroll
        for (int j = 0; j < JW; ++j)
#pragma unroll
          for (int mi = 0; mi < MG; ++mi) {
            const float am = frag_get(a, mi);
#pragma unroll
            for (int ni = 0; ni < NG; ++ni)
              acc[j][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(am, b[j][ni], acc[j][mi][ni], 0, 0, 0);
          }
      }
    }
  }
  if (st) st->lap(6);
  // The epilogue is run by the LAST k-half (EPI): with KSPLIT == 2 that keeps
  // waves 0-3, which run the tree phases, free of outstanding HBM stores
  // (a later load's vmcnt wait would wait for their acks).  Its bias and head
  // weights are loaded here, before any store is issued, for the same reason.
  constexpr int EPI = KSPLIT - 1;
  float bb[MG][4], hw[NH > 0 ? NH : 1][MG][4];
  if (active && half == EPI) {
#pragma unroll
    for (int mi = 0; mi < MG; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = (cog * MG + mi) * 16 + kq * 4 + r;
        bb[mi][r] = bias[co];
#pragma unroll
        for (int h = 0; h < NH; ++h) hw[h][mi][r] = head_w[h * COUT + co];
      }
  }
  __syncthreads();   // every wave is done with lds_in and its ring
  if constexpr (KSPLIT == 2) {
    // the first k-half hands its partial accumulators to its partner through
    // the (now idle) rings; the second half adds them (a + b == b + a)
    float* red = ring + wl * (JW * MG * NG * 4 * 64);
    static_assert(4 * JW * MG * NG * 4 * 64 * 4 <= RingBytes<G>::value, "reduction fits the rings");
    if (half == 0 && active) {
#pragma unroll
      for (int j = 0; j < JW; ++j)
#pragma unroll
        for (int mi = 0; mi < MG; ++mi)
#pragma unroll
          for (int ni = 0; ni < NG; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[(((j * MG + mi) * NG + ni) * 4 + r) * 64 + lane] = acc[j][mi][ni][r];
    }
    __syncthreads();
    if (half == 1 && active) {
#pragma unroll
      for (int j = 0; j < JW; ++j)
#pragma unroll
        for (int mi = 0; mi < MG; ++mi)
#pragma unroll
          for (int ni = 0; ni < NG; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[j][mi][ni][r] += red[(((j * MG + mi) * NG + ni) * 4 + r) * 64 + lane];
    }
  }
  if (st) st->lap(7);

  // ---- epilogue: bias + ReLU, store, fused 1x1 heads ----
  float hsum[NH > 0 ? NH : 1][JW][NG];
#pragma unroll
  for (int h = 0; h < (NH > 0 ? NH : 1); ++h)
#pragma unroll
    for (int j = 0; j < JW; ++j)
#pragma unroll
      for (int ni = 0; ni < NG; ++ni) hsum[h][j][ni] = 0.f;
  if (active && half == EPI) {
#pragma unroll
    for (int mi = 0; mi < MG; ++mi) {
      const int cout0 = (cog * MG + mi) * 16 + kq * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = cout0 + r;
#pragma unroll
        for (int j = 0; j < JW; ++j) {
#pragma unroll
          for (int ni = 0; ni < NG; ++ni) {
            float v = acc[j][mi][ni][r] + bb[mi][r];
            if (!YM) v = v > 0.f ? v : 0.f;                 // YM: pre-activation conv + bias
            const int cell = ((cg0 + j * R::JPW) * NG + ni) * 16 + col;
            v = cell < G::CELLS ? v : 0.f;                  // pad cells stay 0 (zero slot)
            if constexpr (YM) {                             // cell-major [CELLS][COUT]
              if (cell < G::CELLS) out[(size_t)cell * COUT + co] = v;
            } else if (out != nullptr && cell < out_cells) {
              out[co * out_stride + cell] = v;
            }
#pragma unroll
            for (int h = 0; h < NH; ++h) hsum[h][j][ni] = __builtin_fmaf(hw[h][mi][r], v, hsum[h][j][ni]);
          }
        }
      }
    }
    if constexpr (NH > 0) {
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int j = 0; j < JW; ++j) {
#pragma unroll
          for (int ni = 0; ni < NG; ++ni) {
            float v = hsum[h][j][ni];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            const int cell = ((cg0 + j * R::JPW) * NG + ni) * 16 + col;
            if (kq == 0 && cell < G::CS) hp_lds[(cog * 3 + h) * G::CS + cell] = v;
          }
        }
    }
  }
  __syncthreads();
}

}  // namespace mzgo

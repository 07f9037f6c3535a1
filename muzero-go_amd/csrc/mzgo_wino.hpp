// mzgo_wino.hpp -- the 3x3/pad-1 convolution of one board as a Winograd
// F(2,3) x F(3,3) transform on fp32 MFMA (v_mfma_f32_16x16x4_f32), with the
// MuZero heads fused into the epilogue.
//
// Rows use F(2,3) (points 0, 1, -1, inf), columns F(3,3) (points 0, 1, -1,
// -2, inf): a 9x9 board is 5 x 3 = 15 output tiles of 2 x 3 cells, so the
// tile index fills one 16-column MFMA tile, and the conv becomes 20 GEMMs
//     M_xi[cout][tile] = sum_cin U_xi[cout][cin] * V_xi[cin][tile],  xi = (i, j)
// of 96 x 96 x 16 -- 2880 MFMAs per conv instead of 7776 for the direct
// implicit GEMM over 96 padded cells.  The device transforms are integer
// (BT, AT below); the fractions of G live in U, packed by the host
// (mzgo_capi.hip: pack_wino).  fp32 error is on par with the direct conv
// (the per-output sums run over 96 inputs instead of 864).
//
// Work split: 12 waves (3 per SIMD); wave w owns cout tile m = w / 2 and xi
// half h = w % 2 (xi rows i = 2h, 2h + 1; all cin), so each M_xi is computed
// and folded into the output transform once; A (U) is streamed straight from
// L2 into VGPRs -- nothing but the transformed input lives in LDS.  The two
// xi halves exchange half of their transformed outputs through LDS: wave h
// finalises output row oy = h of each tile.
//
// 19x19 (10 x 7 = 70 tiles) runs the same GEMM over 5 row strips of 2 tile
// rows (14 tiles each): 5 x 2880 MFMAs per conv instead of 29808 direct.
//
// Replaces the torch conv2d calls of self_play.py:72-74 (representation
// conv2/conv3), :90 (dynamics) and the 1x1 head convs of :81, :100, :102.
#pragma once
#include "mzgo_common.hpp"


namespace mzgo {
constexpr int kWinoXG = 2;   // xi per accumulation group (A stream order, pack_wino)
}

namespace mzgo {

template <class G>
struct Wino {
  static constexpr int TY = (G::N + 1) / 2;   // F(2,3) tiles along rows
  static constexpr int TX = (G::N + 2) / 3;   // F(3,3) tiles along columns
  static constexpr int TRS = (16 / TX < TY) ? 16 / TX : TY;   // tile rows per strip
  static constexpr int NSTRIP = (TY + TRS - 1) / TRS;          // strips (9x9: 1, 19x19: 5)
  static constexpr int T = TRS * TX;          // tiles per strip (MFMA columns)
  static constexpr int SROWS = 2 * TRS;       // output rows per strip
  static constexpr int SCELLS = SROWS * G::N; // output cells per strip (incl. rows >= N)
  static constexpr int XI = 20;               // 4 x 5 transform points
  static_assert(T <= 16, "a strip's tiles must fit one MFMA column tile");
  // cells of a staged output row: a strip's cells; the last strip also carries
  // the pooled layout's pad cells up to CS
  static constexpr int LAST_C0 = (NSTRIP - 1) * SCELLS;
  static constexpr int OCELLS = SCELLS > G::CS - LAST_C0 ? SCELLS : G::CS - LAST_C0;
  // output staging row stride: 4 cout rows apart (the kq lane groups) land 16
  // banks apart; one junk cell (OCELLS) past the stored cells
  static constexpr int OUT_STRIDE = OCELLS + (36 - OCELLS % 32) % 32;
  static_assert(OUT_STRIDE > OCELLS, "junk cell past the stored row");
  // head partials [m][3][HS] per strip (one strip: the whole pooled row)
  static constexpr int HS = NSTRIP == 1 ? G::CS : OCELLS;
  // V floats for CIN input channels: [xi][h][s4][kq][t16][e4]
  template <int CIN>
  static constexpr int v_floats() { return XI * CIN * 16; }
  // exchange buffer [m][h][ox*4 + r][lane]
  template <int COUT>
  static constexpr int red_floats() { return (COUT / 16) * 2 * 12 * 64; }
};

// Transform one board into V.  src: [cin][src_stride] (global, f32); emb:
// per-channel value added at on-board cells (the action-embedding
// broadcast-add of self_play.py:87-89) or null.  Channel c = h*CH +
// 4*(4*s4 + e) + kq is stored at V[((((xi*2 + h)*S4 + s4)*4 + kq)*16 + t)*4 + e]
// so a lane's B operand for 4 consecutive k-steps is one ds_read_b128.
//
// Work unit: a channel quad (h, s4, kq) = the 4 channels e = 0..3 that share
// one V row; lane (t, e) transforms tile t of channel e.  Each wave fetches
// its quads' rows itself (all loads in flight at once) and scatters them,
// embedding already added, into its own slice of raw: one zero-haloed plane
// per channel covering the strip's rows -1..SROWS and columns -1..N, so every
// tap of every tile is a plain load at a constant offset -- no bounds
// selects.  The only workgroup barrier is the one before the GEMM.
template <class G>
struct WinoRaw {
  static_assert(G::N == 9 || G::N == 19, "bank layout derived for 9x9 and 19x19 tiles");
  static constexpr int PW = G::N + 2;                    // padded width
  static constexpr int PH = Wino<G>::SROWS + 2;          // padded height (strip rows + halo)
  static constexpr int PLANE = PH * PW;
  // plane stride == 11 (mod 32): the lanes of channels e and e+1 (one 32-lane
  // half) share 2 of 15 tile banks at 9x9 (offsets 22*ty + 3*tx) and none at
  // 19x19 (42*ty + 3*tx)
  static constexpr int STRIDE = PLANE + ((11 - PLANE % 32) % 32 + 32) % 32;
  static_assert(STRIDE > PLANE, "a junk slot past each plane");
  // wino_input_rebuilt's scatter stores, per ds_write_b32, the 12 channel
  // quads of ~3 cells into the planes of waves j, j + 4, j + 8: waves j and
  // j + 8 sit 32 * STRIDE apart, on the same banks, so their slices are
  // skewed by 8 floats (simulated over both boards: 3.9-way -> 2-way
  // conflicts; 2-way is the floor at STRIDE = 11 mod 32)
#ifdef MZGO_STAMPS
  static constexpr int SKEW = G::N == 19 ? 0 : 8;   // (the 19x19 stamps build has no 32 B of LDS to spare)
#else
  static constexpr int SKEW = 8;
#endif
  __device__ static constexpr int base(int wave) { return wave * 4 * STRIDE + ((wave >> 2) == 2 ? SKEW : 0); }
  static constexpr int FLOATS = G::WAVES * 4 * STRIDE + SKEW;   // all waves' slices
};

// The 4 x 5 patch of tile (ty, tx) of channel e (plane my + e*RS) -> the 20
// V entries of that (channel, tile): BT2 along rows, then BT3 along columns.
template <class G, int CIN>
__device__ __forceinline__ void wino_transform_quad(float* __restrict__ V, const float* my, int quad, int t,
                                                    int e, int ty, int tx) {
  constexpr int S4 = CIN / 32, PW = WinoRaw<G>::PW, RS = WinoRaw<G>::STRIDE;
  // the last tile column's patch may run past its padded row (19x19: 3 * 7
  // columns + 2 > 21): into the next row's halo column and first cell, and
  // for the last row into the junk slot, which every writer leaves 0
  static_assert((WinoRaw<G>::PH - 1) * PW + 3 * (Wino<G>::TX - 1) + 4 < RS, "patch reads stay in the plane slot");
  const float* s = my + e * RS + (2 * ty) * PW + 3 * tx;   // tile's top-left (padded coords)
  float d[4][5];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 5; ++b) d[a][b] = s[a * PW + b];
  float* vb = V + (size_t)quad * 64 + t * 4 + e;         // quad index == (h*S4 + s4)*4 + kq
  constexpr int XSTRIDE = 2 * S4 * 4 * 64;    // floats between xi planes
  // rows in pairs (0,1), (2,3) as packed f32x2 (v_pk_add/v_pk_fma: two rows
  // per instruction); the factor-2 FMAs round exactly like mul + add
  f32x2 u[2][5];
#pragma unroll
  for (int b = 0; b < 5; ++b) {               // BT2 along rows
    u[0][b] = f32x2{d[0][b], d[1][b]} + f32x2{-d[2][b], d[2][b]};
    u[1][b] = f32x2{d[2][b], d[3][b]} - f32x2{d[1][b], d[1][b]};
  }
  const f32x2 two = {2.f, 2.f}, mtwo = {-2.f, -2.f}, three = {3.f, 3.f};
#pragma unroll
  for (int i = 0; i < 2; ++i) {               // BT3 along columns
    const f32x2* q = u[i];
    const f32x2 a = q[1] - q[3], b = q[0] - q[2];
    f32x2 v[5];
    v[0] = __builtin_elementwise_fma(two, b, a);
    v[1] = __builtin_elementwise_fma(three, q[2], __builtin_elementwise_fma(two, q[1], q[3]));
    v[2] = __builtin_elementwise_fma(mtwo, q[1], q[2] + q[3]);
    v[3] = a;
    v[4] = __builtin_elementwise_fma(mtwo, a, q[4] - q[2]);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      vb[((2 * i) * 5 + j) * XSTRIDE] = v[j].x;
      vb[((2 * i + 1) * 5 + j) * XSTRIDE] = v[j].y;
    }
  }
}

// The halo columns of every raw plane must be 0 before the first wino_input
// of a kernel (never written afterwards; halo rows are rewritten per strip).
// All threads; synchronises.
template <class G>
__device__ __forceinline__ void wino_raw_zero(float* raw) {
  for (int i = tid_local(); i < WinoRaw<G>::FLOATS; i += G::THREADS) raw[i] = 0.f;
  __syncthreads();
}

template <class G, int CIN>
__device__ __forceinline__ void wino_input(float* __restrict__ V, float* __restrict__ raw,
                                           const float* __restrict__ src, int src_stride,
                                           const float* __restrict__ emb, int strip = 0,
                                           Stamp* st = nullptr) {
  typedef Wino<G> W;
  typedef WinoRaw<G> R;
  constexpr int CH = CIN / 2, S4 = CH / 16, RS = R::STRIDE, PW = R::PW, PH = R::PH;
  static_assert(CIN % 32 == 0, "two cin halves of whole 4-k-step groups");
  constexpr int QUADS = 2 * S4 * 4;           // (h, s4, kq)
  constexpr int QPW = (QUADS + G::WAVES - 1) / G::WAVES;   // quads per wave
  // whole pooled rows (one strip: 16-byte loads of all CS cells) or, per
  // strip, the strip's PH rows of N cells (4-byte loads, any stride)
  const bool fast = W::NSTRIP == 1 && src_stride == G::CS;
  constexpr int Q4 = G::CS / 4;               // float4 per pooled channel row
  constexpr int NQ = 4 * Q4;                  // float4 per quad (fast path)
  constexpr int PER = (NQ + 63) / 64;
  constexpr int NE = 4 * PH * G::N;           // floats per quad (strip path)
  constexpr int PERS = (NE + 63) / 64;
  const int lane = lane_id_local();
  const int wave = __builtin_amdgcn_readfirstlane(wave_id());
  const int t = lane & 15, e = lane >> 4;
  const int tt = t < W::T ? t : W::T - 1;     // pad column: any valid tile (output unused)
  const int ty = tt / W::TX, tx = tt - ty * W::TX;
  const int row0 = strip * W::SROWS - 1;      // board row of padded row 0
  float* my = raw + R::base(wave);
  auto chan = [&](int quad, int ee) {         // channel of quad member ee
    const int h = quad / (S4 * 4), s4 = (quad / 4) % S4, kq = quad % 4;
    return h * CH + 4 * (4 * s4 + ee) + kq;
  };
  auto pidx = [&](int cell) { const int y = cell / G::N; return (y - row0) * PW + (cell - y * G::N) + 1; };
  const float* ebase = emb ? emb : src;

  if (strip > 0) __syncthreads();            // the previous strip's epilogue is done with LDS
  const unsigned long long t_in = st ? __builtin_amdgcn_s_memtime() : 0;
  if (fast) {
    // all of this wave's rows (and their embedding values) in flight at once;
    // loads are branch-free (clamped indices) so they stay outstanding together
    f32x4 rg[QPW][PER];
    float eg[QPW][PER];
    const f32x4* s4p = reinterpret_cast<const f32x4*>(src);
#pragma unroll
    for (int k = 0; k < QPW; ++k) {
      const int quad = min(wave + k * G::WAVES, QUADS - 1);
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const int i = min(lane + 64 * p, NQ - 1);
        rg[k][p] = s4p[chan(quad, i / Q4) * Q4 + i % Q4];
        eg[k][p] = ebase[chan(quad, i / Q4)];
      }
    }
    if (st) st->lap(20);
    // scatter targets of this lane's 4*PER floats (pad cells and surplus lanes
    // go to a junk slot past the plane): the same for every quad
    int widx[PER][4];
#pragma unroll
    for (int p = 0; p < PER; ++p) {
      const int i = lane + 64 * p, ee = min(i, NQ - 1) / Q4, c0 = (min(i, NQ - 1) % Q4) * 4;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        widx[p][r] = (i < NQ && c0 + r < G::CELLS) ? ee * RS + pidx(c0 + r) : R::PLANE;
    }
#pragma unroll
    for (int k = 0; k < QPW; ++k) {
      const int quad = wave + k * G::WAVES;
      if (quad >= QUADS) break;               // wave-uniform
      if (k) wave_lds_sync();                 // previous quad's reads are done
#pragma unroll
      for (int p = 0; p < PER; ++p) {
        const float ec = emb ? eg[k][p] : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) my[widx[p][r]] = widx[p][r] == R::PLANE ? 0.f : rg[k][p][r] + ec;
      }
      wave_lds_sync();
      if (st && k == 0) st->lap(29);
      wino_transform_quad<G, CIN>(V, my, quad, t, e, ty, tx);
    }
    if (st) st->lap(30);
  } else {
    // strip rows row0 .. row0+PH-1 of the quad's 4 channels (rows off the
    // board are written as 0: the plane is reused by every strip)
    float rv[QPW][PERS];
#pragma unroll
    for (int k = 0; k < QPW; ++k) {
      const int quad = min(wave + k * G::WAVES, QUADS - 1);
#pragma unroll
      for (int p = 0; p < PERS; ++p) {
        const int i = min(lane + 64 * p, NE - 1);
        const int ee = i / (PH * G::N), r = i - ee * (PH * G::N), py = r / G::N, x = r - py * G::N;
        const int y = row0 + py;
        const bool on = y >= 0 && y < G::N;
        const int c = chan(quad, ee);
        const float v = src[(size_t)c * src_stride + (on ? y * G::N + x : 0)];
        const float ec = emb ? ebase[c] : 0.f;
        rv[k][p] = on ? v + ec : 0.f;
      }
    }
    if (st) st->lap(20);
#pragma unroll
    for (int k = 0; k < QPW; ++k) {
      const int quad = wave + k * G::WAVES;
      if (quad >= QUADS) break;               // wave-uniform
      if (k) wave_lds_sync();
#pragma unroll
      for (int p = 0; p < PERS; ++p) {
        const int i = lane + 64 * p;
        const int ee = min(i, NE - 1) / (PH * G::N), r = min(i, NE - 1) - ee * (PH * G::N);
        const int py = r / G::N, x = r - py * G::N;
        // (surplus lanes write 0 to the junk slot: at 19x19 the last tile
        // column's 5-column patch of the last row runs 2 floats past the row
        // into it, and a value left there by an earlier conv would move that
        // tile's valid outputs by rounding -- the slot must be the same
        // whichever conv this workgroup ran before)
        my[i < NE ? ee * RS + py * PW + x + 1 : R::PLANE] = i < NE ? rv[k][p] : 0.f;
      }
      wave_lds_sync();
      wino_transform_quad<G, CIN>(V, my, quad, t, e, ty, tx);
    }
  }
  unsigned long long t_pre = 0;
  if (st) t_pre = __builtin_amdgcn_s_memtime();
  __syncthreads();
  if (st) {
    const unsigned long long t_post = __builtin_amdgcn_s_memtime();
    (void)t_in; (void)t_post;   // (slots 32-55 hold the shared-job laps)
    st->lap(21);
  }
}

// wino_input of a REBUILT latent relu(Y + E[a]) (materialize, mzgo_expand.hpp:
// the dynamics input of a node rebuilt from its parent's conv output Y,
// self_play.py:87-90) without the channel-major copy: the strip's rows are
// read straight from Y ([CELLS][C], cell-major, global) in slabs of 4 WAVES
// channels.  Slab k = channels 4Wk .. 4Wk + 4W-1 = quads Wk .. Wk + W-1 (quad
// = (h*S4 + s4)*4 + kq, channel 16*(h*S4 + s4) + 4e + kq), one quad per wave
// (19x19: 12 waves, 2 slabs of 48 channels).  The workgroup loads the slab's
// cells (W float4 per cell, contiguous), adds E's
// region row, applies the ReLU and scatters a float4's 4 channels (kq = 0..3)
// to 4 waves' planes; after a barrier each wave transforms its quad.  The
// next slab's loads are in flight during the transform.  Values are
// bit-identical to materialize + wino_input (the same f32 add and select).
//
// ylds: the parent's Y is the expansion's LDS copy (L.yc, which V overlays):
// every slab's Y is read from it into registers first, and the first barrier
// (before any V store) orders those reads before the transform overwrites it.
// Typical late in a game: the leaf is a child of the previous batch's leaf.
// (the steps of wino_input_rebuilt, also run piecewise under the GEMM by
// wino_conv_rebuilt)
template <class G, int CIN>
struct RebuiltInput {
  typedef Wino<G> W;
  typedef WinoRaw<G> R;
  static constexpr int RS = R::STRIDE, PW = R::PW, PH = R::PH, C4 = CIN / 4;
  static constexpr int F4 = G::WAVES;                   // float4 per cell per slab
  static_assert(CIN == G::C && G::WAVES % 4 == 0 && CIN % (4 * F4) == 0, "whole slabs, one quad per wave");
  static constexpr int SLABS = CIN / (4 * F4);
  static constexpr int NI = PH * G::N * F4;             // float4 per slab
  static constexpr int R4 = (NI + G::THREADS - 1) / G::THREADS;
  float* V;
  float* raw;
  const f32x4* Y4;
  const f32x4* E4;
  bool lds;
  int row0, wave, t, e, ty, tx;
  f32x4 yv[2][R4], ev[2][R4];                           // slabs k and k + 1
  __device__ __forceinline__ RebuiltInput(float* V_, float* raw_, const float* ypar, const float* ea, int strip,
                                          const float* ylds) {
    V = V_;
    raw = raw_;
    if constexpr (SLABS > 2) ylds = nullptr;            // (slabs past the 2nd would read overwritten LDS)
    lds = ylds != nullptr;
    Y4 = reinterpret_cast<const f32x4*>(ylds ? ylds : ypar);
    E4 = reinterpret_cast<const f32x4*>(ea);
    const int lane = lane_id_local();
    wave = __builtin_amdgcn_readfirstlane(wave_id());
    t = lane & 15;
    e = lane >> 4;
    const int tt = t < W::T ? t : W::T - 1;
    ty = tt / W::TX;
    tx = tt - ty * W::TX;
    row0 = strip * W::SROWS - 1;
  }
  __device__ __forceinline__ void load(int k) {
    f32x4 (&yd)[R4] = yv[k & 1];
    f32x4 (&ed)[R4] = ev[k & 1];
#pragma unroll
    for (int r = 0; r < R4; ++r) {
      const int i = min(tid_local() + r * G::THREADS, NI - 1);
      const int cl = i / F4, q4 = i - cl * F4, py = cl / G::N, x = cl - py * G::N, y = row0 + py;
      const bool on = y >= 0 && y < G::N;
      const int ry = y <= 0 ? 0 : (y >= G::N - 1 ? 2 : 1), rx = x == 0 ? 0 : (x == G::N - 1 ? 2 : 1);
      yd[r] = Y4[(on ? y * G::N + x : 0) * C4 + F4 * k + q4];
      ed[r] = E4[(ry * 3 + rx) * C4 + F4 * k + q4];
    }
  }
  // slab k's cells, E added and ReLU applied, into the waves' raw planes
  __device__ __forceinline__ void scatter(int k) {
    f32x4 (&yk)[R4] = yv[k & 1];
    f32x4 (&ek)[R4] = ev[k & 1];
#pragma unroll
    for (int r = 0; r < R4; ++r) {
      const int i = tid_local() + r * G::THREADS;
      if (i < NI) {
        const int cl = i / F4, q4 = i - cl * F4, py = cl / G::N, x = cl - py * G::N, y = row0 + py;
        const bool on = y >= 0 && y < G::N;
        float* dst = raw + R::base((q4 >> 2) * 4) + (q4 & 3) * RS + py * PW + x + 1;   // (+ j * 4 * RS: the same skew)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = yk[r][j] + ek[r][j];
          dst[j * 4 * RS] = on ? (v > 0.f ? v : 0.f) : 0.f;
        }
      }
    }
  }
  // this wave's quad of slab k: raw planes -> V
  __device__ __forceinline__ void transform(int k) {
    wino_transform_quad<G, CIN>(V, raw + R::base(wave), F4 * k + wave, t, e, ty, tx);
  }
  __device__ __forceinline__ void begin() {
    __syncthreads();                                    // the previous conv's epilogue is done with LDS
    load(0);
    // from LDS: slab 1 too, before the first barrier (V overwrites the copy)
    if (lds && SLABS > 1) load(1);
  }
  __device__ __forceinline__ void slab(int k) {
    scatter(k);
    // (HBM: the next slab's loads in flight during this slab's transform)
    if (k + 1 < SLABS && !lds) load(k + 1);
    __syncthreads();
    transform(k);
    __syncthreads();                                    // planes read before the next slab / V before the GEMM
  }
};

template <class G, int CIN>
__device__ __forceinline__ void wino_input_rebuilt(float* __restrict__ V, float* __restrict__ raw,
                                                   const float* __restrict__ ypar, const float* __restrict__ ea,
                                                   int strip, const float* ylds = nullptr) {
  RebuiltInput<G, CIN> in(V, raw, ypar, ea, strip, ylds);
  in.begin();
#pragma unroll
  for (int k = 0; k < RebuiltInput<G, CIN>::SLABS; ++k) in.slab(k);
}

// AT2 (2 x 4) and AT3 (3 x 5) of the output transform
__device__ __forceinline__ constexpr float wino_at2(int oy, int i) {
  return oy == 0 ? (i < 3 ? 1.f : 0.f) : (i == 0 ? 0.f : (i == 2 ? -1.f : 1.f));
}
__device__ __forceinline__ constexpr float wino_at3(int ox, int j) {
  return ox == 0 ? (j < 4 ? 1.f : 0.f)
                 : (ox == 1 ? (j == 0 ? 0.f : (j == 1 ? 1.f : (j == 2 ? -1.f : (j == 3 ? -2.f : 0.f))))
                            : (j == 0 ? 0.f : (j == 3 ? 4.f : 1.f)));
}

// GEMMs + output transform + bias/ReLU + store + fused 1x1 heads.
// V: transformed input (LDS, wino_input); red: exchange buffer (LDS, may
// alias V); hp: head partials [COUT/16][3][CS]; outs: output staging
// [COUT][CS] (LDS; red, hp and outs disjoint).  hp is complete on return;
// the stores to ``out`` are issued but not synchronised.
// upk: U packed [m][h][pos][lane][4], pos = ((xl/XG)*KP + k)*XG + xl%XG for
// xi = h*10 + xl and k-position k (pack_wino).  out: [COUT][out_stride]
// global; cells >= out_cells are not stored (pooled rows, stride == out_cells
// == CS, are stored whole with their zero pad cells).
//
// m0 / nm (tail helpers, 9x9 parent convs only: YM, NH = 0, one strip): only
// cout tiles m0 .. m0 + nm - 1, on waves 0 .. 2 nm - 1; red then needs room
// for nm tiles only and V is left intact (the next unit reuses it).  Every
// output is computed by the same operations as in the whole conv.
//
// One-strip boards (KHALF) run the K dimension in two halves, every xi's
// first half before any second half (pack_wino's khalf order; each xi's
// chain still adds k = 0 .. KP-1 in order, so the sums are the same bits):
// hook(s) runs between the MFMA groups of step s of the first half, and a
// hook that DEFERS the second half's V (wino_conv_rebuilt: that half is
// transformed during the first) finishes with hook.finish() before it.
struct WinoNoHook {
  static constexpr bool DEFERS = false;
  __device__ void operator()(int) const {}
  __device__ void finish() const {}
};
template <class G, int CIN, int COUT, int NH, bool YM = false, class Hook = WinoNoHook>
__device__ __forceinline__ void wino_conv(const float* V, float* red, float* hp, float* outs, float* hfin,
                                          const float* __restrict__ upk,
                                          const float* __restrict__ bias, float* __restrict__ out,
                                          int out_stride, int out_cells, const float* __restrict__ head_w,
                                          int strip = 0, Stamp* st = nullptr, float* ylds = nullptr, int m0 = 0,
                                          int nm = COUT / 16, Hook hook = Hook{}) {
  typedef Wino<G> W;
  constexpr int CH = CIN / 2, S4 = CH / 16, MT = COUT / 16, XI = W::XI;
  constexpr int OS = W::OUT_STRIDE;
  constexpr int XH = XI / 2;                  // xi per wave (two xi halves)
  constexpr int KP = CIN / 16;                // float4 k-positions per xi (4 k-steps each)
  constexpr int L = XH * KP;                  // float4 A loads (and B reads) per wave
  constexpr int PF = 8;             // A prefetch depth (float4 registers)
  static_assert(2 * MT <= G::WAVES, "one wave per (cout tile, xi half)");
  constexpr int XG = kWinoXG;
  static_assert(XH % XG == 0, "xi groups");
  const int lane = lane_id_local();
  const int wave = __builtin_amdgcn_readfirstlane(wave_id());
  const int ml = wave >> 1, m = m0 + ml, h = wave & 1;   // (ml: the tile's slot in red)
  const bool active = wave < 2 * nm;
  const int kq = lane >> 4, t = lane & 15;

  f32x4 yp[6];                                // Z [il*3 + ox] in the loop, then Y partial [oy*3 + ox]
#pragma unroll
  for (int o = 0; o < 6; ++o) yp[o] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bb[4];                                // this lane's 4 output channels' bias
#pragma unroll
  for (int r = 0; r < 4; ++r) bb[r] = active ? bias[m * 16 + kq * 4 + r] : 0.f;

  const unsigned long long t_loop = st ? __builtin_amdgcn_s_memtime() : 0ull;
  constexpr bool KHALF = true;                // (every Winograd board: pack_wino's khalf order)
  static_assert(!Hook::DEFERS || KHALF, "a deferred second half needs the split K loop");
  if (KHALF && active) {
    // (KHALF) all xi's accumulators live across the two K halves
    constexpr int KH = KP / 2, NG = XH / XG;
    static_assert(KP % 2 == 0, "two K halves");
    const f32x4* ap = reinterpret_cast<const f32x4*>(upk) + (size_t)(m * 2 + h) * L * 64 + lane;
    const f32x4* bp = reinterpret_cast<const f32x4*>(V) + (size_t)h * XH * KP * 64 + lane;
    auto bidx = [&](int xl, int k) { return (xl * KP + k) * 64; };
    f32x4 ar[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) ar[p] = ap[p * 64];
    f32x4 bn[XG];
#pragma unroll
    for (int q = 0; q < XG; ++q) bn[q] = bp[bidx(q, 0)];
    f32x4 acc[XH];
#pragma unroll
    for (int x = 0; x < XH; ++x) acc[x] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) {
      if (kh == 1 && Hook::DEFERS) {
        hook.finish();                        // the second half's V is complete
#pragma unroll
        for (int q = 0; q < XG; ++q) bn[q] = bp[bidx(q, KH)];
      }
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        // progress-ordered issue (see below): priority by the group's place in both halves
        const int pg = kh * NG + g;
        if (pg < 2) __builtin_amdgcn_s_setprio(3);
        else if (pg < 4) __builtin_amdgcn_s_setprio(2);
        else if (pg < 6) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int kk = 0; kk < KH; ++kk) {
          const int k = kh * KH + kk, s = (kh * NG + g) * KH + kk, pos0 = s * XG;
          f32x4 a[XG], b[XG];
#pragma unroll
          for (int q = 0; q < XG; ++q) { a[q] = ar[(pos0 + q) % PF]; b[q] = bn[q]; }
          if (kk + 1 < KH) {
#pragma unroll
            for (int q = 0; q < XG; ++q) bn[q] = bp[bidx(g * XG + q, k + 1)];
          } else if (g + 1 < NG) {
#pragma unroll
            for (int q = 0; q < XG; ++q) bn[q] = bp[bidx((g + 1) * XG + q, kh * KH)];
          } else if (kh == 0 && !Hook::DEFERS) {
#pragma unroll
            for (int q = 0; q < XG; ++q) bn[q] = bp[bidx(q, KH)];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int q = 0; q < XG; ++q)
              acc[g * XG + q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][e], b[q][e], acc[g * XG + q], 0, 0, 0);
#pragma unroll
          for (int q = 0; q < XG; ++q)
            if (pos0 + q + PF < L) ar[(pos0 + q) % PF] = ap[(pos0 + q + PF) * 64];
          __builtin_amdgcn_sched_barrier(0);
          if (kh == 0) hook(s);
        }
      }
    }
    // fold along the columns, xi ascending as below
#pragma unroll
    for (int xl = 0; xl < XH; ++xl) {
      const int il = xl / 5, j = xl % 5;
      const f32x4 mv = acc[xl];
#pragma unroll
      for (int ox = 0; ox < 3; ++ox) {
        const float cf = wino_at3(ox, j);
        if (cf == 1.f) yp[il * 3 + ox] += mv;
        else if (cf == -1.f) yp[il * 3 + ox] -= mv;
        else if (cf != 0.f) yp[il * 3 + ox] += cf * mv;
      }
    }
  } else if (KHALF && Hook::DEFERS) {
    // waves without a cout tile (m0 / nm): their share of the hook's work,
    // at the same barriers as the active waves
    constexpr int KH = KP / 2, NG = XH / XG;
#pragma unroll
    for (int s = 0; s < NG * KH; ++s) hook(s);
    hook.finish();
  } else if (!KHALF && active) {
    // this wave: xi in [h*XH, h*XH + XH), all CIN (KP float4 k-positions per xi).
    // A stream: positions pos = ((g*KP + k)*XG + q) for local xi g*XG + q, in
    // consumption order (pack_wino), PF float4 registers ahead
    const f32x4* ap = reinterpret_cast<const f32x4*>(upk) + (size_t)(m * 2 + h) * L * 64 + lane;
    const f32x4* bp = reinterpret_cast<const f32x4*>(V) + (size_t)h * XH * KP * 64 + lane;
    auto bidx = [&](int xl, int k) { return (xl * KP + k) * 64; };
    f32x4 ar[PF];
#pragma unroll
    for (int p = 0; p < PF; ++p) ar[p] = ap[p * 64];
    f32x4 bn[XG];
#pragma unroll
    for (int q = 0; q < XG; ++q) bn[q] = bp[bidx(q, 0)];
#pragma unroll
    for (int g = 0; g < XH / XG; ++g) {       // XG independent accumulation chains
      // progress-ordered issue: a wave that is ahead drops its priority, so
      // the SIMD's three waves advance together (oldest-first issue otherwise
      // leaves the youngest wave's two MFMA chains to finish alone)
      if (g == 0) __builtin_amdgcn_s_setprio(3);
      else if (g == 1) __builtin_amdgcn_s_setprio(2);
      else if (g == 2) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
      f32x4 acc[XG];
#pragma unroll
      for (int q = 0; q < XG; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KP; ++k) {
        const int pos0 = (g * KP + k) * XG;
        f32x4 a[XG], b[XG];
#pragma unroll
        for (int q = 0; q < XG; ++q) { a[q] = ar[(pos0 + q) % PF]; b[q] = bn[q]; }
        // next B operands
        if (k + 1 < KP) {
#pragma unroll
          for (int q = 0; q < XG; ++q) bn[q] = bp[bidx(g * XG + q, k + 1)];
        } else if (g + 1 < XH / XG) {
#pragma unroll
          for (int q = 0; q < XG; ++q) bn[q] = bp[bidx((g + 1) * XG + q, 0)];
        }
        __builtin_amdgcn_sched_barrier(0);      // issue the next B reads before these MFMAs
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int q = 0; q < XG; ++q)
            acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][e], b[q][e], acc[q], 0, 0, 0);
#pragma unroll
        for (int q = 0; q < XG; ++q)
          if (pos0 + q + PF < L) ar[(pos0 + q) % PF] = ap[(pos0 + q + PF) * 64];
        // keep the refill loads here: left alone, the scheduler sinks them
        // next to their use (to save VGPRs) and exposes the L2 latency
        __builtin_amdgcn_sched_barrier(0);
      }
      // fold M_xi along the columns: Z[il][ox] += AT3[ox][j] M_xi for
      // xi = h*XH + xl, il = xl / 5, j = xl % 5 (the same for both halves);
      // the rows (AT2) are applied once, after the loop
#pragma unroll
      for (int q = 0; q < XG; ++q) {
        const int xl = g * XG + q, il = xl / 5, j = xl % 5;
        const f32x4 mv = acc[q];
#pragma unroll
        for (int ox = 0; ox < 3; ++ox) {
          const float cf = wino_at3(ox, j);
          if (cf == 1.f) yp[il * 3 + ox] += mv;
          else if (cf == -1.f) yp[il * 3 + ox] -= mv;
          else if (cf != 0.f) yp[il * 3 + ox] += cf * mv;
        }
      }
    }
  }
  // rows: Y[oy][ox] = sum_i AT2[oy][i] Z[i][ox] over this half's i = 2h, 2h+1
  // (AT2 = [[1,1,1,0],[0,1,-1,1]]): h = 0: Y0 = Z0 + Z1, Y1 = Z1;
  // h = 1: Y0 = Z2, Y1 = Z3 - Z2.  yp[0..2] / yp[3..5] become Y[0] / Y[1].
  if (active) {
#pragma unroll
    for (int ox = 0; ox < 3; ++ox) {
      const f32x4 z0 = yp[ox], z1 = yp[3 + ox];
      if (h == 0) { yp[ox] = z0 + z1; yp[3 + ox] = z1; }
      else { yp[ox] = z0; yp[3 + ox] = z1 - z0; }
    }
  }
  __builtin_amdgcn_s_setprio(0);
  if (st) { st->wave_add(8 + wave, __builtin_amdgcn_s_memtime() - t_loop); st->lap(6); }

  // epilogue constants (the bias was loaded before the GEMM, its latency
  // hidden there)
  float hw[NH > 0 ? NH : 1][4];
  if (active) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = m * 16 + kq * 4 + r;
#pragma unroll
      for (int hh = 0; hh < NH; ++hh) hw[hh][r] = head_w[hh * COUT + co];
    }
  }
  __syncthreads();                            // V is dead: red may overwrite it
  // wave (m, h) hands its partial of output row oy = 1 - h to its partner
  // (the other xi half of the same cout tile)
  // (rows picked by a wave-uniform select, not a dynamic register index)
  f32x4 ymine[3], ygive[3];
#pragma unroll
  for (int ox = 0; ox < 3; ++ox) {
    ymine[ox] = h == 0 ? yp[ox] : yp[3 + ox];
    ygive[ox] = h == 0 ? yp[3 + ox] : yp[ox];
  }
  // (one ds_write_b128 / ds_read_b128 per output column: [m][h][ox][lane] f32x4)
  f32x4* red4 = reinterpret_cast<f32x4*>(red);
  if (active) {
#pragma unroll
    for (int ox = 0; ox < 3; ++ox) red4[((ml * 2 + h) * 3 + ox) * 64 + lane] = ygive[ox];
  }
  __syncthreads();
  if (st) st->lap(7);
  const int c0 = strip * W::SCELLS;          // first cell of this strip
  if constexpr (YM && NH == 0 && W::NSTRIP == 1) {
    // The pre-activation Y of a parent conv, cell-major [CELLS][COUT]: lane
    // (t, kq) holds couts m*16 + 4kq .. +3 of its cells (2ty + h, 3tx + ox),
    // one float4 of Y each -- stored straight from the registers, no staging
    // (the LDS copy ylds overlays red: written after every wave's red reads)
    f32x4 yv[3];
    int cl[3];
    bool ok[3];
    const int ty = t / W::TX, tx = t - ty * W::TX, y = 2 * ty + h;
#pragma unroll
    for (int ox = 0; ox < 3; ++ox) {
      const int x = 3 * tx + ox;
      ok[ox] = active && t < W::T && y < G::N && x < G::N;
      cl[ox] = y * G::N + x;
      if (active) {
        const f32x4 other = red4[((ml * 2 + (1 - h)) * 3 + ox) * 64 + lane];
        const f32x4 mine = ymine[ox];
#pragma unroll
        for (int r = 0; r < 4; ++r) yv[ox][r] = (h == 0 ? mine[r] + other[r] : other[r] + mine[r]) + bb[r];   // (xi half 0) + (xi half 1)
        if (ok[ox]) reinterpret_cast<f32x4*>(out + (size_t)cl[ox] * COUT)[m * 4 + kq] = yv[ox];
      }
    }
    if (ylds) {
      __syncthreads();
#pragma unroll
      for (int ox = 0; ox < 3; ++ox)
        if (ok[ox]) reinterpret_cast<f32x4*>(ylds + (size_t)cl[ox] * COUT)[m * 4 + kq] = yv[ox];
    }
    return;                                   // (the caller synchronises before reading Y)
  }
  if (active) {
    const int oy = h;
    const int ty = t / W::TX, tx = t - ty * W::TX;
    const int y = strip * W::SROWS + 2 * ty + oy;
    float hsum[NH > 0 ? NH : 1][3];
#pragma unroll
    for (int hh = 0; hh < (NH > 0 ? NH : 1); ++hh)
#pragma unroll
      for (int ox = 0; ox < 3; ++ox) hsum[hh][ox] = 0.f;
#pragma unroll
    for (int ox = 0; ox < 3; ++ox) {
      const int x = 3 * tx + ox;
      const bool valid = t < W::T && y < G::N && x < G::N;
      const int cell = y * G::N + x;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float other = red4[((ml * 2 + (1 - h)) * 3 + ox) * 64 + lane][r];
        const float mine = ymine[ox][r];
        // fixed order: (xi half 0) + (xi half 1)
        float v = (h == 0 ? mine + other : other + mine) + bb[r];
        if (!YM) v = v > 0.f ? v : 0.f;           // YM: pre-activation conv + bias
        v = valid ? v : 0.f;
        const int co = m * 16 + kq * 4 + r;
        outs[co * OS + (valid ? cell - c0 : W::OCELLS)] = v;   // staged (off-board lanes: junk cell)
#pragma unroll
        for (int hh = 0; hh < NH; ++hh) hsum[hh][ox] = __builtin_fmaf(hw[hh][r], v, hsum[hh][ox]);
      }
    }
    if constexpr (NH > 0) {
#pragma unroll
      for (int hh = 0; hh < NH; ++hh)
#pragma unroll
        for (int ox = 0; ox < 3; ++ox) {
          float v = hsum[hh][ox];
          v = swap_add<false>(v);               // + lane ^ 16
          v = swap_add<true>(v);                // + lane ^ 32
          const int x = 3 * tx + ox;
          if (kq == 0 && t < W::T && y < G::N && x < G::N) hp[(m * 3 + hh) * W::HS + y * G::N + x - c0] = v;
        }
    }
  }
  // pad cells of the staged rows are 0 (the pooled layout keeps them 0)
  const bool last = strip == W::NSTRIP - 1;
  if (last)
    for (int i = tid_local(); i < COUT * (G::CS - G::CELLS); i += G::THREADS) {
      const int co = i / (G::CS - G::CELLS);
      outs[co * OS + G::CELLS - c0 + (i - co * (G::CS - G::CELLS))] = 0.f;
    }
  __syncthreads();
  if constexpr (W::NSTRIP > 1 && NH > 0) {
    // strip boards: this strip's head sums over the cout tiles, in a fixed
    // order, into the board-wide hfin [3][CS] (hp is reused by the next strip)
    constexpr int SC = W::SCELLS;
    for (int i = tid_local(); i < NH * SC; i += G::THREADS) {
      const int hh = i / SC, lc = i - hh * SC;
      if (c0 + lc < G::CELLS) {
        float v = hp[hh * W::HS + lc];
#pragma unroll
        for (int mm = 1; mm < MT; ++mm) v += hp[(mm * 3 + hh) * W::HS + lc];
        hfin[hh * G::CS + c0 + lc] = v;
      }
    }
  }
  // whole-row stores (the tile-ordered epilogue would scatter 4-byte writes)
  if constexpr (YM) {
    // cell-major [CELLS][COUT] (the factored expansion reads a cell's channels
    // as contiguous float4s): float4 of 4 couts per (cell, cout quad)
    constexpr int Q = COUT / 4;
    const int n = min(c0 + W::SCELLS, G::CELLS) - c0;
    for (int i = tid_local(); i < n * Q; i += G::THREADS) {
      const int j = i / Q, q = i - j * Q;
      const f32x4 v = {outs[(4 * q) * OS + j], outs[(4 * q + 1) * OS + j], outs[(4 * q + 2) * OS + j],
                       outs[(4 * q + 3) * OS + j]};
      reinterpret_cast<f32x4*>(out + (size_t)(c0 + j) * COUT)[q] = v;
      // (ylds: the same Y also into LDS -- the expansion's copy, over the
      // exchange buffer, dead by now -- instead of reading it back from HBM)
      if (ylds) reinterpret_cast<f32x4*>(ylds + (size_t)(c0 + j) * COUT)[q] = v;
    }
  } else if (out != nullptr) {
    if (out_stride == G::CS && out_cells == G::CS) {
      const int Q = ((last ? G::CS : c0 + W::SCELLS) - c0) / 4;   // float4 of this strip's row span
      for (int i = tid_local(); i < COUT * Q; i += G::THREADS) {
        const int co = i / Q, q = i - co * Q;
        const f32x4 v = *reinterpret_cast<const f32x4*>(outs + co * OS + q * 4);
        f32x4* dst = reinterpret_cast<f32x4*>(out + (size_t)co * G::CS + c0) + q;
        __builtin_nontemporal_store(v, dst);
      }
    } else {
      const int n = min(c0 + W::SCELLS, out_cells) - c0;
      for (int i = tid_local(); i < COUT * n; i += G::THREADS) {
        const int co = i / n, j = i - co * n;
        out[(size_t)co * out_stride + c0 + j] = outs[co * OS + j];
      }
    }
  }
  // no barrier: a caller that reads ``out`` (or hfin) back synchronises first
}

// wino_conv of a rebuilt input on one-strip boards (9x9 parent convs), the
// second channel slab (the GEMM's second K half) scattered and transformed
// between the first half's MFMA groups instead of before the GEMM: its LDS
// and VALU work issues under the matrix cores' time.  The same operations as
// wino_input_rebuilt + wino_conv, so the same bits.
template <class G>
struct RebuiltHook {
  static constexpr bool DEFERS = true;
  // first-half steps (of KP / 2 * XI / 2 / kWinoXG = 15 at 9x9) after which
  // the scatter, the barrier before the transform and the transform run
  // (measured, same call: (2, 7, 10) 81.4-81.6 M sims/s, (2, 6, 9) 81.3,
  // (4, 10, 12) 81.3-81.4, (1, 5, 7) 81.0, (0, 3, 4) 80.4-80.7)
  static constexpr int kScatter = 2, kBarrier = 7, kTransform = 10;
  RebuiltInput<G, G::C> in;
  __device__ __forceinline__ void operator()(int s) {
    if (s == kScatter) in.scatter(1);
    else if (s == kBarrier) __syncthreads();
    else if (s == kTransform) in.transform(1);
  }
  __device__ __forceinline__ void finish() { __syncthreads(); }
};
template <class G>
__device__ __forceinline__ void wino_conv_rebuilt(float* V, float* raw, float* red, float* hp, float* outs,
                                                  float* hfin, const float* __restrict__ ypar,
                                                  const float* __restrict__ ea, const float* __restrict__ upk,
                                                  const float* __restrict__ bias, float* __restrict__ out,
                                                  Stamp* st, float* ylds, const float* ysrc_lds, int strip = 0,
                                                  int m0 = 0, int nm = G::C / 16) {
  static_assert(RebuiltInput<G, G::C>::SLABS == 2, "two slabs");
  RebuiltInput<G, G::C> in(V, raw, ypar, ea, strip, ysrc_lds);
  in.begin();
  in.slab(0);
  if (st) st->lap(1);
  wino_conv<G, G::C, G::C, 0, true, RebuiltHook<G>>(V, red, hp, outs, hfin, upk, bias, out, G::CS, G::CS, nullptr,
                                                     strip, st, ylds, m0, nm, RebuiltHook<G>{in});
}

}  // namespace mzgo

// mzgo_capi.hip -- the C ABI of include/mzgo.h: engine lifetime, device
// memory, weight packing and dispatch to the per-(N, C) kernel tables.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/mzgo.h"
#include "mzgo_dispatch.hpp"
#include "mzgo_tower_host.hpp"

namespace mzgo {
extern const KernelSet kernels_n5_c96, kernels_n6_c96, kernels_n9_c96, kernels_n19_c96, kernels_n6_c128,
    kernels_n6_c64;

// the trainer's conv layers (mzgo_train.hip)
size_t conv_bwd_workspace_bytes(int B, int Cin, int Cout);
hipError_t conv_forward(const float* x, const int64_t* action, const float* emb, const float* w, const float* bias,
                        int B, int Cin, int Cout, int N, float* y, hipStream_t s);
hipError_t conv_backward(const float* g, const float* out, const float* x, const int64_t* action, const float* emb,
                         const float* w, int B, int Cin, int Cout, int N, float* gx, float* gw, float* gb,
                         void* workspace, hipStream_t s);

const KernelSet* find_kernels(int N, int C) {
  static const KernelSet* all[] = {&kernels_n5_c96, &kernels_n6_c96, &kernels_n9_c96, &kernels_n19_c96,
                                   &kernels_n6_c128, &kernels_n6_c64};
  for (const KernelSet* k : all)
    if (k->N == N && k->C == C) return k;
  return nullptr;
}
}  // namespace mzgo

using namespace mzgo;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) return fail(MZGO_EHIP, "%s: %s", #expr, hipGetErrorString(e_));    \
  } while (0)

namespace {

// Reference state_dict keys (self_play.py:63-128) and their shapes.
struct Spec {
  std::string key;
  std::vector<int64_t> shape;
};

std::vector<Spec> specs(int C, int A) {
  return {
      {"representation.conv1.weight", {64, 6, 3, 3}}, {"representation.conv1.bias", {64}},
      {"representation.conv2.weight", {64, 64, 3, 3}}, {"representation.conv2.bias", {64}},
      {"representation.conv3.weight", {C, 64, 3, 3}}, {"representation.conv3.bias", {C}},
      {"dynamics.action_embedding.weight", {A, C}},
      {"dynamics.conv.weight", {C, C, 3, 3}}, {"dynamics.conv.bias", {C}},
      {"dynamics.reward_conv.weight", {1, C, 1, 1}}, {"dynamics.reward_conv.bias", {1}},
      {"dynamics.fc_reward_hidden.weight", {16, 1}}, {"dynamics.fc_reward_hidden.bias", {16}},
      {"dynamics.fc_reward_output.weight", {1, 16}}, {"dynamics.fc_reward_output.bias", {1}},
      {"prediction.pass_logit", {1}},
      {"prediction.value_conv.weight", {1, C, 1, 1}}, {"prediction.value_conv.bias", {1}},
      {"prediction.value_fc.weight", {1, 1}}, {"prediction.value_fc.bias", {1}},
      {"prediction.policy_conv.weight", {1, C, 1, 1}}, {"prediction.policy_conv.bias", {1}},
  };
}

// conv weight W[cout][cin][3][3] -> MFMA A-fragment order of mzgo_conv.hpp:
// packed[((s * NCOG + cog) * 64 + lane) * MGP + mi] with k-step s = tap*CQ + c4,
// cout = (cog*MG + mi)*16 + (lane & 15), cin = c4*4 + (lane >> 4).
// With cog_major the layout is packed[(frag * 64 + lane) * MGP + mi] with
// frag = ((cog * ksplit + half) * 9 + tap) * (CQ / ksplit) + c4 % (CQ / ksplit):
// one contiguous stream per (cout group, k-half) for the per-wave DMA rings
// of conv3x3_ring (ksplit = Geo::KSPLIT); otherwise frag = s * NCOG + cog
// (conv3x3_direct).
std::vector<float> pack_conv(const float* W, int COUT, int CIN, bool cog_major, int ksplit = 1) {
  const int CINP = (CIN + 3) / 4 * 4, CQ = CINP / 4, KS = 9 * CQ, CQH = CQ / ksplit;
  const int MT = COUT / 16;
  const int MG = (MT % 3 == 0) ? 3 : ((MT % 4 == 0 && MT >= 8) ? 4 : 2);
  const int MGP = MG == 3 ? 4 : MG, NCOG = MT / MG;
  std::vector<float> out((size_t)KS * NCOG * 64 * MGP, 0.f);
  for (int s = 0; s < KS; ++s) {
    const int t = s / CQ, c4 = s % CQ, ky = t / 3, kx = t % 3;
    for (int cog = 0; cog < NCOG; ++cog)
      for (int lane = 0; lane < 64; ++lane)
        for (int mi = 0; mi < MG; ++mi) {
          const int cout = (cog * MG + mi) * 16 + (lane & 15);
          const int cin = c4 * 4 + (lane >> 4);
          const float v = cin < CIN ? W[(((size_t)cout * CIN + cin) * 3 + ky) * 3 + kx] : 0.f;
          // cog-major streams are further ordered [half][tap][c4 within the half]
          const int half = c4 / CQH, c4h = c4 % CQH;
          const size_t frag = cog_major ? (((size_t)cog * ksplit + half) * 9 + t) * CQH + c4h
                                        : (size_t)s * NCOG + cog;
          out[(frag * 64 + lane) * MGP + mi] = v;
        }
  }
  return out;
}

// conv weight W[cout][cin][3][3] -> Winograd U for mzgo_wino.hpp (9x9):
// U_xi[cout][cin] = (G2 g G3^T)[i][j], g = W[cout][cin], xi = i*5 + j, with
// G2 of F(2,3) (points 0, 1, -1, inf) on kernel rows and G3 of F(3,3)
// (points 0, 1, -1, -2, inf) on kernel columns, computed in double and
// rounded once.  Packed as packed[(((m*2 + h)*L + pos)*64 + lane)*4 + e]
// = U_xi[16m + (lane & 15)][hh*CIN/2 + 4*(4*s4 + e) + (lane >> 4)] for
// xi = h*10 + xl, k-position k = hh*S4 + s4 (S4 = CIN/32), and
// pos = ((xl/XG)*KP + k)*XG + xl%XG (kWinoXG, KP = CIN/16): one contiguous
// float4 stream per (cout tile m, xi half h) wave, in the order wino_conv
// consumes it.
// khalf (one-strip boards, wino_conv's KHALF loop): consumption order is
// K half, xi group, k-position within the half, xi within the group -- the
// GEMM runs the first half of CIN for every xi before the second, so the
// rebuilt input's second channel slab is transformed under the first half's
// MFMAs (wino_conv_rebuilt)
std::vector<float> pack_wino(const float* W, int COUT, int CIN, bool khalf) {
  static const double G2[4][3] = {{1, 0, 0}, {0.5, 0.5, 0.5}, {0.5, -0.5, 0.5}, {0, 0, 1}};
  static const double G3[5][3] = {{0.5, 0, 0},
                                  {1.0 / 6, 1.0 / 6, 1.0 / 6},
                                  {0.5, -0.5, 0.5},
                                  {1.0 / 6, -1.0 / 3, 2.0 / 3},
                                  {0, 0, 1}};
  const int MT = COUT / 16, CH = CIN / 2, S4 = CH / 16, KP = CIN / 16, L = 10 * KP;
  std::vector<float> out((size_t)MT * 2 * L * 64 * 4, 0.f);
  for (int m = 0; m < MT; ++m)
    for (int h = 0; h < 2; ++h)
      for (int xl = 0; xl < 10; ++xl)
        for (int k = 0; k < KP; ++k)
          for (int lane = 0; lane < 64; ++lane)
            for (int e = 0; e < 4; ++e) {
              const int xi = h * 10 + xl, i = xi / 5, j = xi % 5;
              const int hh = k / S4, s4 = k % S4;
              const int co = 16 * m + (lane & 15), ci = hh * CH + 4 * (4 * s4 + e) + (lane >> 4);
              const float* g = W + ((size_t)co * CIN + ci) * 9;
              double u = 0.0;
              for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) u += G2[i][a] * (double)g[a * 3 + b] * G3[j][b];
              const int KH = KP / 2, kh = k / KH, NG = 10 / kWinoXG;
              const int pos = khalf ? (((kh * NG + xl / kWinoXG) * KH + k % KH) * kWinoXG + xl % kWinoXG)
                                    : (((xl / kWinoXG) * KP + k) * kWinoXG + xl % kWinoXG);   // consumption order
              out[((((size_t)m * 2 + h) * L + pos) * 64 + lane) * 4 + e] = (float)u;
            }
  return out;
}

// The action-tap table of the factored expansion (mzgo_expand.hpp):
// E[a][r][co] = sum over the taps (ky, kx) on the board for a cell of region
// r = ry*3 + rx (ry, rx in {first, interior, last} row / column) of
// sum_ci W[co][ci][ky][kx] * emb[a][ci], so that conv3x3(x + emb[a]) =
// conv3x3(x) + E[a][region] under zero padding.  f64 sums, rounded once.
std::vector<float> action_taps(const float* W, const float* emb, int C, int A) {
  std::vector<float> out((size_t)A * 9 * C);
  std::vector<double> u((size_t)9 * C);
  for (int a = 0; a < A; ++a) {
    const float* e = emb + (size_t)a * C;
    for (int co = 0; co < C; ++co)
      for (int t = 0; t < 9; ++t) {
        double s = 0.0;
        for (int ci = 0; ci < C; ++ci) s += (double)W[((size_t)co * C + ci) * 9 + t] * (double)e[ci];
        u[(size_t)t * C + co] = s;
      }
    for (int r = 0; r < 9; ++r) {
      const int ry = r / 3, rx = r % 3;
      for (int co = 0; co < C; ++co) {
        double s = 0.0;
        for (int ky = 0; ky < 3; ++ky) {
          if ((ry == 0 && ky == 0) || (ry == 2 && ky == 2)) continue;   // row y-1 / y+1 off the board
          for (int kx = 0; kx < 3; ++kx) {
            if ((rx == 0 && kx == 0) || (rx == 2 && kx == 2)) continue;
            s += u[(size_t)(ky * 3 + kx) * C + co];
          }
        }
        out[((size_t)a * 9 + r) * C + co] = (float)s;
      }
    }
  }
  return out;
}

}  // namespace

// CUs of the current device (one self-play workgroup fills a CU's LDS)
static int device_cus() {
  static int ncu[64];                  // per device ordinal (0: not read yet)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (ncu[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    ncu[dev] = n;
  }
  return ncu[dev];
}

struct mzgo_engine {
  mzgo_config cfg;
  const KernelSet* ks = nullptr;
  int N = 0, C = 0, A = 0, CELLS = 0, CS = 0, G = 0, S = 0, M = 0;
  int TS = 0;                   // search-tree slots: G, or the CU count when larger (move-parallel epoch)
  std::map<std::string, std::vector<float>> sd;  // host copies of the state_dict
  std::vector<Spec> spec;
  bool dirty = true;
  float* d_w = nullptr;
  size_t d_w_bytes = 0;
  NetParams np{};
  EngineArrays E{};
  int* d_err = nullptr;
  float* d_scr = nullptr;      // initial_inference scratch (strip boards), grown on demand
  size_t scr_floats = 0;
  std::vector<void*> allocs;
  // move-parallel launch timing (mzgo_selfplay_set_timing): per launch pair,
  // events before the boards launch, between it and k_search_queue, after it
  bool timing = false;
  std::vector<hipEvent_t> tev;
  int tn = 0;                   // launch pairs recorded since the last read
  int64_t bytes = 0;
  int epoch = 0;
  const double* noise = nullptr;
  double* noise_out = nullptr;  // test hook: roots' normalised Dirichlet samples [G][M][A]
  TowerHost* tower = nullptr;   // residual-tower network (mzgo_config.tower, BASELINE config 5)

  template <class T>
  int alloc(T** p, size_t n) {
    void* v = nullptr;
    hipError_t e = hipMalloc(&v, n * sizeof(T) + 256);
    if (e != hipSuccess) return fail(MZGO_EHIP, "hipMalloc(%zu): %s", n * sizeof(T), hipGetErrorString(e));
    allocs.push_back(v);
    bytes += (int64_t)(n * sizeof(T));
    *p = reinterpret_cast<T*>(v);
    return MZGO_OK;
  }
  ~mzgo_engine() {
    if (tower) {
      for (hipEvent_t ev : tower->evs) (void)hipEventDestroy(ev);
      tower->free_chains();
      for (void* p : {tower->d_wb, (void*)tower->d_wf, (void*)tower->ib, (void*)tower->ob, (void*)tower->s0,
                      (void*)tower->s1, (void*)tower->shp, (void*)tower->sact})
        if (p) (void)hipFree(p);
      if (tower->h_total) (void)hipHostFree(tower->h_total);
      tower->free_batch();
      delete tower;
    }
    for (hipEvent_t ev : tev) (void)hipEventDestroy(ev);
    for (void* p : allocs) (void)hipFree(p);
    if (d_w) (void)hipFree(d_w);
    if (d_scr) (void)hipFree(d_scr);
  }

  // pack + upload the network if any tensor changed since the last upload
  int sync_weights() {
    if (C == 0) return fail(MZGO_EINVAL, "board-only engine (latent_dim 0) has no network");
    if (!dirty) return MZGO_OK;
    for (const Spec& s : spec)
      if (!sd.count(s.key)) return fail(MZGO_ENOWEIGHTS, "missing weight '%s'", s.key.c_str());
    if (tower) {
      HIPCHK(tower->upload(sd, &action_taps));
      dirty = false;
      return MZGO_OK;
    }
    std::vector<std::vector<float>> parts;
    parts.push_back(pack_conv(sd["representation.conv1.weight"].data(), 64, 6, false));
    parts.push_back(sd["representation.conv1.bias"]);
    // k-range split of the ring conv: 2 when the board runs 8 waves (Geo::KSPLIT)
    const int ct = (N * N + 15) / 16, ng = ct >= 3 ? 3 : ct, ncg = (ct + ng - 1) / ng;
    const int ksplit = ncg <= 2 ? 2 : 1;
    const bool wino = N == 9 || N == 19;           // Geo::WINO
    auto latent = [&](const char* key, int cout, int cin) {
      return wino ? pack_wino(sd[key].data(), cout, cin, true) : pack_conv(sd[key].data(), cout, cin, true, ksplit);
    };
    parts.push_back(latent("representation.conv2.weight", 64, 64));
    parts.push_back(sd["representation.conv2.bias"]);
    parts.push_back(latent("representation.conv3.weight", C, 64));
    parts.push_back(sd["representation.conv3.bias"]);
    parts.push_back(latent("dynamics.conv.weight", C, C));
    parts.push_back(sd["dynamics.conv.bias"]);
    parts.push_back(sd["dynamics.action_embedding.weight"]);
    std::vector<float> hw;
    for (const char* k : {"dynamics.reward_conv.weight", "prediction.value_conv.weight",
                          "prediction.policy_conv.weight"})
      hw.insert(hw.end(), sd[k].begin(), sd[k].end());
    parts.push_back(hw);
    parts.push_back(action_taps(sd["dynamics.conv.weight"].data(), sd["dynamics.action_embedding.weight"].data(), C, A));
    const char* scal[] = {"dynamics.reward_conv.bias", "dynamics.fc_reward_hidden.weight",
                          "dynamics.fc_reward_hidden.bias", "dynamics.fc_reward_output.weight",
                          "dynamics.fc_reward_output.bias", "prediction.value_conv.bias",
                          "prediction.value_fc.weight", "prediction.value_fc.bias",
                          "prediction.policy_conv.bias", "prediction.pass_logit"};
    for (const char* k : scal) parts.push_back(sd[k]);
    std::vector<size_t> off;
    size_t total = 0;
    for (auto& p : parts) { off.push_back(total); total += (p.size() + 63) / 64 * 64; }
    std::vector<float> blob(total, 0.f);
    for (size_t i = 0; i < parts.size(); ++i) std::memcpy(blob.data() + off[i], parts[i].data(), parts[i].size() * 4);
    if (total * 4 > d_w_bytes) {
      if (d_w) (void)hipFree(d_w);
      d_w = nullptr;
      HIPCHK(hipMalloc(&d_w, total * 4));
      d_w_bytes = total * 4;
    }
    HIPCHK(hipMemcpy(d_w, blob.data(), total * 4, hipMemcpyHostToDevice));
    const float* b = d_w;
    np.w_conv1 = b + off[0]; np.b_conv1 = b + off[1];
    np.w_conv2 = b + off[2]; np.b_conv2 = b + off[3];
    np.w_conv3 = b + off[4]; np.b_conv3 = b + off[5];
    np.w_dyn = b + off[6]; np.b_dyn = b + off[7];
    np.emb = b + off[8]; np.head_w = b + off[9]; np.etab = b + off[10];
    np.hs.reward_b = b + off[11]; np.hs.fc1_w = b + off[12]; np.hs.fc1_b = b + off[13];
    np.hs.fc2_w = b + off[14]; np.hs.fc2_b = b + off[15]; np.hs.value_b = b + off[16];
    np.hs.vfc_w = b + off[17]; np.hs.vfc_b = b + off[18]; np.hs.policy_b = b + off[19];
    np.hs.pass_logit = b + off[20];
    dirty = false;
    return MZGO_OK;
  }

  // drop-in inference scratch of the tower engine for B boards (zero borders)
  int tower_scratch(int B) {
    TowerHost& t = *tower;
    if (B <= t.scap) return MZGO_OK;
    for (void* p : {(void*)t.ib, (void*)t.ob, (void*)t.s0, (void*)t.s1, (void*)t.shp, (void*)t.sact})
      if (p) HIPCHK(hipFree(p));
    t.ib = t.ob = t.s0 = t.s1 = nullptr; t.shp = nullptr; t.sact = nullptr; t.scap = 0;
    const size_t n = (size_t)B * t.slot();
    for (bf16** q : {&t.ib, &t.ob, &t.s0, &t.s1}) {
      HIPCHK(hipMalloc((void**)q, n * sizeof(bf16)));
      HIPCHK(hipMemset(*q, 0, n * sizeof(bf16)));
    }
    HIPCHK(hipMalloc((void**)&t.shp, (size_t)B * t.CC * 3 * t.CS * sizeof(float)));
    HIPCHK(hipMalloc((void**)&t.sact, (size_t)B * sizeof(int)));
    t.scap = B;
    return MZGO_OK;
  }

  SearchParams search_params() const {
    SearchParams sp;
    sp.c_puct = cfg.c_puct; sp.discount = cfg.discount;
    sp.dirichlet_alpha = cfg.dirichlet_alpha; sp.dirichlet_epsilon = cfg.dirichlet_epsilon;
    sp.pass_epsilon = cfg.pass_epsilon; sp.num_simulations = S; sp.compat = cfg.compat;
    sp.variant = cfg.search_variant;
    sp.factored = cfg.direct_dynamics ? 0 : 1;
    sp.seed = cfg.seed;
    sp.helpers = 0;
    sp.net = 0;
    sp.tail = 0;
    const char* lz = getenv("MZGO_LAZY_ROWS");        // (=0: eager rows in self-play too, an A/B switch)
    sp.lazy_rows = lz && atoi(lz) == 0 ? 0 : 1;
    return sp;
  }
};

extern "C" {

const char* mzgo_last_error(void) { return g_err.c_str(); }

void mzgo_default_config(mzgo_config* c, int N) {
  std::memset(c, 0, sizeof *c);
  c->board_size = N;
  c->latent_dim = 96;
  c->num_games = 1;
  c->num_simulations = 128;
  c->max_moves = N * N;
  c->compat = 0;
  c->temperature_moves = 15;
  c->c_puct = 2.5;
  c->discount = 0.99;
  c->dirichlet_alpha = 0.15;
  c->dirichlet_epsilon = 0.02;
  c->pass_epsilon = 0.01;
  c->temperature = 1.0;
  c->komi = 0.0;
  c->seed = 1234;
}

int mzgo_engine_create(const mzgo_config* cfg, mzgo_engine** out) {
  if (!cfg || !out) return fail(MZGO_EINVAL, "null argument");
  *out = nullptr;
  const int N = cfg->board_size, C = cfg->latent_dim;
  const int TW = cfg->tower, RB = cfg->res_blocks;
  if (TW != 0 && TW != 1) return fail(MZGO_EINVAL, "tower must be 0 (reference network) or 1 (residual tower)");
  if (TW && RB < 0) return fail(MZGO_EINVAL, "res_blocks must be >= 0");
  const TowerSet* tset = nullptr;
  if (TW) {
    // the residual-tower network (BASELINE config 5): board kernels of the
    // N x N build, the tower's own conv / tree kernels
    tset = find_tower(N);
    if (!tset) return fail(MZGO_EINVAL, "unsupported board_size %d for the tower network (built: 5, 9, 19)", N);
    if (C < 64 || C % 64 != 0 || C > 1024)
      return fail(MZGO_EINVAL, "the tower network needs latent_dim a multiple of 64 in [64, 1024], got %d", C);
  }
  const KernelSet* ks = find_kernels(N, (C == 0 || TW) ? 96 : C);
  if (!ks) return fail(MZGO_EINVAL, "unsupported board_size %d / latent_dim %d (built: N in {5,6,9,19} with C=96; N=6 with C=128 or 64)", N, C);
  if (cfg->num_games < 1) return fail(MZGO_EINVAL, "num_games must be >= 1");
  if (C != 0 && cfg->num_simulations < 1) return fail(MZGO_EINVAL, "num_simulations must be >= 1");
  if (cfg->compat != 0 && cfg->compat != 1) return fail(MZGO_EINVAL, "compat must be 0 or 1");
  if (cfg->direct_dynamics != 0 && cfg->direct_dynamics != 1)
    return fail(MZGO_EINVAL, "direct_dynamics must be 0 (factored expansion) or 1 (a conv per simulation)");
  if (cfg->search_variant != 0 && cfg->search_variant != 1)
    return fail(MZGO_EINVAL, "search_variant must be 0 (self_play.py) or 1 (main.py)");
  HIPCHK(hipSetDevice(cfg->device));
  auto* e = new mzgo_engine();
  e->cfg = *cfg;
  e->ks = ks;
  e->N = N; e->C = C; e->A = N * N + 1; e->CELLS = N * N; e->CS = (N * N + 15) / 16 * 16;
  e->G = cfg->num_games;
  e->S = C == 0 ? 0 : cfg->num_simulations;
  e->M = cfg->max_moves > 0 ? cfg->max_moves : N * N;
  e->cfg.max_moves = e->M;
  if (TW) {
    e->spec.clear();
    for (auto& kv : TowerHost::specs(C, e->A, RB)) e->spec.push_back(Spec{kv.first, kv.second});
  } else {
    e->spec = specs(C, e->A);
  }
  EngineArrays& E = e->E;
  E.S = e->S;
  E.max_moves = e->M;
  // Search-tree slots.  Boards whose game-per-workgroup launch takes helper
  // workgroups (19x19: fewer games than CUs, 3 helpers each) get a tree per
  // CU when the move-parallel epoch can run (compat "reference", self_play.py
  // search): its queue runs one search per CU (k_search_queue).
  // MZGO_MOVE_PARALLEL=0 at creation keeps G.
  e->TS = e->G;
  if (C != 0 && !TW && ks->shared_batches && cfg->compat == 0 && cfg->search_variant == 0) {
    const char* v = getenv("MZGO_MOVE_PARALLEL");
    if (!(v && atoi(v) == 0)) e->TS = std::max(e->G, device_cus());
  }
  const size_t G = e->G, TSL = e->TS, n1 = (size_t)e->S + 1, A = e->A, CELLS = e->CELLS, M = e->M;
  int rc = MZGO_OK;
  auto chk = [&](int r) { if (r != MZGO_OK && rc == MZGO_OK) rc = r; };
  if (C != 0 && !TW) {
    // S+1 node slots + one scratch latent per game
    chk(e->alloc(&E.pool, TSL * (n1 + 1) * (size_t)C * e->CS));
    // pad cells (>= N*N) of pooled latents are read as zeros and never written
    if (rc == MZGO_OK && hipMemset(E.pool, 0, TSL * (n1 + 1) * (size_t)C * e->CS * sizeof(float)) != hipSuccess)
      chk(fail(MZGO_EHIP, "hipMemset(pool) failed"));
  }
  if (TW) {
    TowerHost* t = e->tower = new TowerHost();
    t->ts = tset;
    t->N = N; t->C = C; t->CC = C / 64; t->blocks = RB; t->G = e->G; t->S = e->S; t->A = e->A;
    t->P = (N + 2) * (N + 2); t->CS = e->CS;
    TowerArrays& T = t->TA;
    T.C = C; T.co_chunks = C / 64;
    const size_t slot = (size_t)t->slot();
    // batched simulation steps (MZGO_TOWER_BATCH=1): up to min(A, S) pending
    // entries per game (the root's children), so up to G x that many boards
    // per step; their buffers are allocated on first use (ensure_batch)
    t->bq_cap = (int)std::min<size_t>(A, n1 - 1);
    t->maxb = (int)(G * (size_t)t->bq_cap);
    T.bq_cap = t->bq_cap;
    // node latents (bf16, zero borders: the conv's padding is never written);
    // the tower's two scratch activations per board of a one-leaf step
    chk(e->alloc(&T.pool, G * n1 * slot));
    chk(e->alloc(&t->t0, G * slot));
    chk(e->alloc(&t->t1, G * slot));
    chk(e->alloc(&T.rep_in, G * (size_t)t->P * 64));
    if (rc == MZGO_OK) {
      for (auto pr : {std::make_pair((void*)T.pool, G * n1 * slot), std::make_pair((void*)t->t0, G * slot),
                      std::make_pair((void*)t->t1, G * slot), std::make_pair((void*)T.rep_in, G * (size_t)t->P * 64)})
        if (hipMemset(pr.first, 0, pr.second * sizeof(bf16)) != hipSuccess) chk(fail(MZGO_EHIP, "hipMemset(tower) failed"));
    }
    T.slot = (long long)slot;
    chk(e->alloc(&T.hpart, G * (size_t)t->CC * 3 * e->CS));
    chk(e->alloc(&T.bq_n, G));
    chk(e->alloc(&T.bq_nid0, G));
    chk(e->alloc(&T.nbg, G));
    chk(e->alloc(&T.b_total, 1));
    if (rc == MZGO_OK && (hipMemset(T.bq_n, 0, G * sizeof(int)) != hipSuccess ||
                          hipHostMalloc(&t->h_total, sizeof(int), hipHostMallocDefault) != hipSuccess))
      chk(fail(MZGO_EHIP, "tower batch setup failed"));
    chk(e->alloc(&T.rootmask, G * A));
    chk(e->alloc(&T.passp, G));
    chk(e->alloc(&T.key, G));
    chk(e->alloc(&T.playing, G));
    chk(e->alloc(&T.evalact, G));
    chk(e->alloc(&T.in_idx, G));
    chk(e->alloc(&T.out_idx, G));
    chk(e->alloc(&T.root_idx, G));
    chk(e->alloc(&T.act, G));
    chk(e->alloc(&T.job, G * 3));
    chk(e->alloc(&T.simc, G));
    if (rc == MZGO_OK) {
      std::vector<int> ri(G);
      for (size_t g = 0; g < G; ++g) ri[g] = (int)(g * n1);
      if (hipMemcpy(T.root_idx, ri.data(), G * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
          hipMemset(T.playing, 0, G * sizeof(int)) != hipSuccess || hipMemset(T.evalact, 0, G * sizeof(int)) != hipSuccess)
        chk(fail(MZGO_EHIP, "tower index setup failed"));
    }
  }
  if (C != 0) {
    chk(e->alloc(&E.prior, TSL * n1 * A));
    chk(e->alloc(&E.child, TSL * n1 * A));
    chk(e->alloc(&E.visits, TSL * n1));
    chk(e->alloc(&E.wsum, TSL * n1));
    chk(e->alloc(&E.root_prior, TSL * A));
    chk(e->alloc(&E.path, TSL * (n1 + 1)));
    chk(e->alloc(&E.nodes, TSL));
    chk(e->alloc(&E.nact, TSL * n1));
    chk(e->alloc(&E.jobs, TSL * job_bytes(A)));
    chk(e->alloc(&E.mpq, 2 * (size_t)G + 1));
    chk(e->alloc(&E.rec_stones, G * M * CELLS));
    chk(e->alloc(&E.rec_invd, G * M * CELLS));
    chk(e->alloc(&E.rec_flags, G * M));
    chk(e->alloc(&E.rec_action, G * M));
    chk(e->alloc(&E.rec_value, G * M));
    chk(e->alloc(&E.rec_policy, G * M * A));
    chk(e->alloc(&E.rec_reward, G * M));
  }
  chk(e->alloc(&E.stones, G * CELLS));
  chk(e->alloc(&E.invd, G * CELLS));
  chk(e->alloc(&E.meta, G * 4));
  chk(e->alloc(&E.game_len, G));
  chk(e->alloc(&E.final_reward, G));
  chk(e->alloc(&E.status, G));
  chk(e->alloc(&E.counters, kCounters));
  chk(e->alloc(&e->d_err, 1));
#ifdef MZGO_STAMPS
  chk(e->alloc(&E.stamps, TSL * kStampPhases));
  if (E.stamps) (void)hipMemset(E.stamps, 0, TSL * kStampPhases * 8);
#endif
  if (rc != MZGO_OK) { delete e; return rc; }
  if (hipMemset(E.counters, 0, kCounters * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(e->d_err, 0, sizeof(int)) != hipSuccess) {
    delete e;
    return fail(MZGO_EHIP, "hipMemset failed");
  }
  hipError_t he = ks->board_reset(E, e->G, nullptr);
  if (he == hipSuccess) he = hipDeviceSynchronize();
  if (he != hipSuccess) { delete e; return fail(MZGO_EHIP, "board reset: %s", hipGetErrorString(he)); }
  *out = e;
  return MZGO_OK;
}

void mzgo_engine_destroy(mzgo_engine* e) { delete e; }

int64_t mzgo_engine_device_bytes(const mzgo_engine* e) { return e ? e->bytes + (int64_t)e->d_w_bytes : 0; }

int mzgo_set_weights(mzgo_engine* e, const char* key, const float* data, const int64_t* shape, int ndim) {
  if (!e || !key || !data || (!shape && ndim > 0)) return fail(MZGO_EINVAL, "null argument");
  for (const Spec& s : e->spec) {
    if (s.key != key) continue;
    if ((int)s.shape.size() != ndim) return fail(MZGO_EINVAL, "'%s': expected %zu dims, got %d", key, s.shape.size(), ndim);
    size_t n = 1;
    for (int i = 0; i < ndim; ++i) {
      if (shape[i] != s.shape[i])
        return fail(MZGO_EINVAL, "'%s': dim %d is %lld, expected %lld", key, i, (long long)shape[i], (long long)s.shape[i]);
      n *= (size_t)shape[i];
    }
    e->sd[key].assign(data, data + n);
    e->dirty = true;
    return MZGO_OK;
  }
  return fail(MZGO_EINVAL, "unexpected key '%s' in state_dict", key);
}

int mzgo_weights_ready(const mzgo_engine* e) {
  if (!e || e->C == 0) return 0;
  for (const Spec& s : e->spec)
    if (!e->sd.count(s.key)) return 0;
  return 1;
}

int mzgo_initial_inference(mzgo_engine* e, const float* obs, int B, float* latent, float* value,
                           float* logits, void* stream) {
  if (!e || !obs || !latent || !value || !logits || B < 1) return fail(MZGO_EINVAL, "bad argument");
  int rc = e->sync_weights();
  if (rc) return rc;
  if (e->tower) {
    if ((rc = e->tower_scratch(B))) return rc;
    TowerHost& t = *e->tower;
    hipStream_t s = (hipStream_t)stream;
    TowerArrays Tb = t.TA;
    Tb.hpart = t.shp;
    HIPCHK(t.ts->tin(obs, t.ib, B, t.C, 1, t.slot(), s));
    HIPCHK(t.tower(t.rep, t.ib, nullptr, t.slot(), t.ob, nullptr, t.slot(), nullptr, nullptr, B, t.s0, t.s1, t.shp, s));
    HIPCHK(t.ts->tout(t.ob, latent, B, t.C, s));
    HIPCHK(t.ts->theads(Tb, B, 0, nullptr, value, logits, s));
    return MZGO_OK;
  }
  float* scr = nullptr;
  if (e->ks->rep_scratch) {
    const size_t need = (size_t)B * e->ks->rep_scratch;
    if (need > e->scr_floats) {
      if (e->d_scr) HIPCHK(hipFree(e->d_scr));   // synchronising: no launch still reads it
      e->d_scr = nullptr;
      e->scr_floats = 0;
      HIPCHK(hipMalloc(&e->d_scr, need * sizeof(float)));
      e->scr_floats = need;
    }
    scr = e->d_scr;
  }
  HIPCHK(e->ks->initial_inference(e->np, obs, B, latent, value, logits, scr, (hipStream_t)stream));
  return MZGO_OK;
}

int mzgo_recurrent_inference(mzgo_engine* e, const float* latent, const int64_t* action, int B,
                             float* next_latent, float* reward, float* value, float* logits, void* stream) {
  if (!e || !latent || !action || !next_latent || !reward || !value || !logits || B < 1)
    return fail(MZGO_EINVAL, "bad argument");
  int rc = e->sync_weights();
  if (rc) return rc;
  if (e->tower) {
    if ((rc = e->tower_scratch(B))) return rc;
    TowerHost& t = *e->tower;
    hipStream_t s = (hipStream_t)stream;
    TowerArrays Tb = t.TA;
    Tb.hpart = t.shp;
    HIPCHK(launch_tact(action, t.sact, B, e->A, e->d_err, s));
    HIPCHK(t.ts->tin(latent, t.ib, B, t.C, 0, t.slot(), s));
    HIPCHK(t.tower(t.dyn, t.ib, nullptr, t.slot(), t.ob, nullptr, t.slot(), t.sact, nullptr, B, t.s0, t.s1, t.shp, s));
    HIPCHK(t.ts->tout(t.ob, next_latent, B, t.C, s));
    HIPCHK(t.ts->theads(Tb, B, 1, reward, value, logits, s));
    return MZGO_OK;
  }
  HIPCHK(e->ks->recurrent_inference(e->np, latent, action, B, next_latent, reward, value, logits,
                                    e->d_err, (hipStream_t)stream));
  return MZGO_OK;
}

// Tower engines: a k_tconv_chain wait that expired makes that launch's
// results wrong; it is reported (MZGO_EHIP) and cleared by the first API
// call that synchronises afterwards -- every call of the tower path does
// (self-play moves, search, inference checks, tree / record / counter reads).
static int check_chain(mzgo_engine* e, hipStream_t s) {
  if (!e->tower) return MZGO_OK;
  bool bad = false;
  HIPCHK(e->tower->chain_error(s, bad));
  if (bad) return fail(MZGO_EHIP, "k_tconv_chain: a workgroup's wait for its board expired (results of the call are wrong)");
  return MZGO_OK;
}

int mzgo_check_inference_errors(mzgo_engine* e, void* stream) {
  if (!e) return fail(MZGO_EINVAL, "null engine");
  if (int rc = check_chain(e, (hipStream_t)stream)) return rc;
  int h = 0;
  HIPCHK(hipMemcpyAsync(&h, e->d_err, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  if (h) {
    HIPCHK(hipMemsetAsync(e->d_err, 0, sizeof(int), (hipStream_t)stream));
    return fail(MZGO_EINVAL, "index out of range in self (action outside [0, %d))", e->A);
  }
  return MZGO_OK;
}

int mzgo_search(mzgo_engine* e, const float* root_obs, const double* noise, int G, int move_index,
                int32_t* visits, double* value, void* stream) {
  if (!e || !root_obs || G < 1 || G > e->G) return fail(MZGO_EINVAL, "bad argument (G=%d, engine has %d slots)", G, e ? e->G : 0);
  int rc = e->sync_weights();
  if (rc) return rc;
  if (e->tower) {
    TowerHost& t = *e->tower;
    hipStream_t s = (hipStream_t)stream;
    const SearchParams sp = e->search_params();
    HIPCHK(hipMemsetAsync(t.TA.playing, 0, e->G * sizeof(int), s));
    HIPCHK(t.ts->obs_search(t.TA, sp, root_obs, e->cfg.game_base, move_index, G, s));
    HIPCHK(t.root_phase(sp, e->E, noise, e->A, 0, s));
    HIPCHK(t.simulations(sp, e->E, s));
    HIPCHK(t.ts->search_out(t.TA, sp, e->E, G, visits, value, s));
    return check_chain(e, s);
  }
  SearchParams sp = e->search_params();
  sp.lazy_rows = 0;                                   // every row of an exported tree formed
  HIPCHK(e->ks->search(e->np, sp, e->E, root_obs, noise, G, e->cfg.game_base, move_index, visits, value,
                       (hipStream_t)stream));
  return MZGO_OK;
}

int mzgo_tree_export(mzgo_engine* e, int g, int32_t* n_nodes, int32_t* child, int32_t* visits,
                     double* value_sum, float* prior, double* root_prior, void* stream) {
  if (!e || e->C == 0 || g < 0 || g >= e->G) return fail(MZGO_EINVAL, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  const size_t n1 = (size_t)e->S + 1, A = e->A;
  if (e->tower) {
    // rows a select never reached still hold logits + the kRawRow sentinel
    // after a self-play move (lazy child priors): settle them as the search
    // API does (k_tsearch_out; idempotent, the values a later select would form)
    TowerHost& t = *e->tower;
    HIPCHK(t.ts->search_out(t.TA, e->search_params(), e->E, e->G, nullptr, nullptr, s));
    if (int rc = check_chain(e, s)) return rc;
  }
  int nn = 0;
  HIPCHK(hipMemcpyAsync(&nn, e->E.nodes + g, sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (n_nodes) *n_nodes = nn;
  if (child) HIPCHK(hipMemcpyAsync(child, e->E.child + g * n1 * A, nn * A * 4, hipMemcpyDeviceToHost, s));
  if (visits) HIPCHK(hipMemcpyAsync(visits, e->E.visits + g * n1, nn * 4, hipMemcpyDeviceToHost, s));
  if (value_sum) HIPCHK(hipMemcpyAsync(value_sum, e->E.wsum + g * n1, nn * 8, hipMemcpyDeviceToHost, s));
  if (prior) HIPCHK(hipMemcpyAsync(prior, e->E.prior + g * n1 * A, nn * A * 4, hipMemcpyDeviceToHost, s));
  if (root_prior) HIPCHK(hipMemcpyAsync(root_prior, e->E.root_prior + g * A, A * 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return MZGO_OK;
}

int mzgo_board_reset(mzgo_engine* e, void* stream) {
  if (!e) return fail(MZGO_EINVAL, "null engine");
  HIPCHK(e->ks->board_reset(e->E, e->G, (hipStream_t)stream));
  return MZGO_OK;
}

int mzgo_board_step(mzgo_engine* e, const int32_t* actions, int32_t* status, double* winner, void* stream) {
  if (!e || !actions) return fail(MZGO_EINVAL, "bad argument");
  HIPCHK(e->ks->board_step(e->E, e->G, actions, status, winner, e->cfg.komi, (hipStream_t)stream));
  return MZGO_OK;
}

int mzgo_board_planes(mzgo_engine* e, double* planes, void* stream) {
  if (!e || !planes) return fail(MZGO_EINVAL, "bad argument");
  HIPCHK(e->ks->board_planes(e->E, e->G, planes, (hipStream_t)stream));
  return MZGO_OK;
}

int mzgo_board_set(mzgo_engine* e, int g, const int8_t* stones, const uint8_t* invd, const int32_t* meta,
                   void* stream) {
  if (!e || g < 0 || g >= e->G || !stones || !invd || !meta) return fail(MZGO_EINVAL, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(hipMemcpyAsync(e->E.stones + (size_t)g * e->CELLS, stones, e->CELLS, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(e->E.invd + (size_t)g * e->CELLS, invd, e->CELLS, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(e->E.meta + (size_t)g * 4, meta, 16, hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  return MZGO_OK;
}

int mzgo_selfplay_reset(mzgo_engine* e, int epoch, void* stream) {
  if (!e || e->C == 0) return fail(MZGO_EINVAL, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  e->epoch = epoch;
  HIPCHK(e->ks->board_reset(e->E, e->G, s));
  return MZGO_OK;
}

// k_selfplay_move; boards whose batch expansions stream Y from L2 (19x19) get
// helper workgroups, 3 per game by default (MZGO_HELPERS_PER_GAME), with the
// job slots zeroed before the launch (batch_expand_shared)

// The epoch tail (whole-game launches): a workgroup whose game has ended
// stays resident and serves running games.  Only when every workgroup of the
// launch is resident at once (one per CU): otherwise ended workgroups would
// hold CUs that games not yet dispatched are waiting for.  MZGO_TAIL_HELPERS=0
// turns it off, =2 forces it on past that bound (a test of the kernel's own
// guards: helpers never join a game whose workgroup has not started).  The
// bound is per launch: engines launched concurrently on several streams (bench.py
// --refill) share the CUs, so their launches are not all resident even when
// each fits -- the started guard keeps that correct, but ended workgroups then
// hold CUs the other engines' games need, and --refill sets MZGO_TAIL_HELPERS=0.
static bool tail_enabled(int workgroups) {
  const char* v = getenv("MZGO_TAIL_HELPERS");
  const int mode = v ? atoi(v) : 1;
  if (mode == 0) return false;
  return mode == 2 || workgroups <= device_cus();
}

// The move-parallel epoch (k_search_queue): multi-move launches under compat
// "reference" play the boards first and then run every recorded move's search
// from one queue, one workgroup per CU (no helper workgroups: at 19x19 every
// CU runs its own search instead of a game's 4 workgroups sharing one); the
// records are the same as the game-per-workgroup launch's.
// MZGO_MOVE_PARALLEL=0 keeps the game-per-workgroup launch (its epoch tail:
// tail_help / join_running_game).
static bool move_parallel(const mzgo_engine* e, const SearchParams& sp, const PlayParams& pp) {
  const char* v = getenv("MZGO_MOVE_PARALLEL");
  if (v && atoi(v) == 0) return false;
  return pp.moves > 1 && !pp.arena && sp.compat == 0 && sp.variant == 0;
}

static int launch_selfplay(mzgo_engine* e, const NetParams& np_b, const PlayParams& pp, hipStream_t s) {
  SearchParams sp = e->search_params();
  if (move_parallel(e, sp, pp)) {
    hipEvent_t* ev = nullptr;
    if (e->timing) {
      while ((int)e->tev.size() < 3 * (e->tn + 1)) {
        hipEvent_t x;
        HIPCHK(hipEventCreate(&x));
        e->tev.push_back(x);
      }
      ev = &e->tev[3 * e->tn++];
    }
    HIPCHK(hipMemsetAsync(e->E.mpq + 2 * e->G, 0, sizeof(int), s));
    if (ev) HIPCHK(hipEventRecord(ev[0], s));
    HIPCHK(e->ks->selfplay_boards(sp, pp, e->E, e->G, s));
    if (ev) HIPCHK(hipEventRecord(ev[1], s));
    const int ncu = device_cus();
    int wg = ncu > 0 && ncu < e->TS ? ncu : e->TS;           // one tree slot per workgroup
    // 19x19: MZGO_QUEUE_HELPERS=h gives every searching workgroup h helpers
    // (wg / (1 + h) searches at once, each tree slot's jobs shared)
    if (e->ks->shared_batches) {
      const char* v = getenv("MZGO_QUEUE_HELPERS");
      const int h = v ? atoi(v) : 0;
      if (h > 0 && wg / (1 + h) >= 1) {
        const int leaders = wg / (1 + h);
        sp.helpers = h * leaders;
        wg = leaders * (1 + h);
        HIPCHK(hipMemsetAsync(e->E.jobs, 0, (size_t)leaders * job_bytes(e->A), s));
      }
    }
    HIPCHK(e->ks->search_queue(e->np, sp, pp, e->E, e->G, wg, s));
    if (ev) HIPCHK(hipEventRecord(ev[2], s));
    return MZGO_OK;
  }
  if (e->ks->shared_batches) {
    int per = 3;
    if (const char* v = getenv("MZGO_HELPERS_PER_GAME")) per = atoi(v);
    sp.helpers = per > 0 ? per * e->G : 0;
    HIPCHK(hipMemsetAsync(e->E.jobs, 0, (size_t)e->G * job_bytes(e->A), s));
    // the epoch tail: helpers (and workgroups) of ended games join running games
    if (sp.helpers > 0 && sp.factored && pp.moves > 1 && tail_enabled(e->G + sp.helpers)) sp.tail = 1;
  } else if (e->ks->tail_convs && sp.factored && pp.moves > 1 && tail_enabled(e->G)) {
    // the epoch tail (one-strip Winograd boards): a workgroup whose game has
    // ended serves running games' parent convs (records the same either way)
    sp.tail = 1;
    HIPCHK(hipMemsetAsync(e->E.jobs, 0, (size_t)e->G * job_bytes(e->A), s));
  }
  HIPCHK(e->ks->selfplay_move(e->np, np_b, sp, pp, e->E, e->G, s));
  return MZGO_OK;
}

int mzgo_selfplay_move(mzgo_engine* e, void* stream) { return mzgo_selfplay_moves(e, 1, stream); }

int mzgo_selfplay_set_timing(mzgo_engine* e, int on) {
  if (!e) return fail(MZGO_EINVAL, "bad argument");
  e->timing = on != 0;
  e->tn = 0;
  return MZGO_OK;
}

int mzgo_selfplay_launch_times(mzgo_engine* e, float* boards_ms, float* queue_ms, int cap, int* n_host) {
  if (!e || !n_host || cap < 0 || (cap > 0 && (!boards_ms || !queue_ms))) return fail(MZGO_EINVAL, "bad argument");
  const int n = e->tn < cap ? e->tn : cap;
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipEventSynchronize(e->tev[3 * i + 2]));
    HIPCHK(hipEventElapsedTime(&boards_ms[i], e->tev[3 * i], e->tev[3 * i + 1]));
    HIPCHK(hipEventElapsedTime(&queue_ms[i], e->tev[3 * i + 1], e->tev[3 * i + 2]));
  }
  *n_host = e->tn;
  e->tn = 0;
  return MZGO_OK;
}

int mzgo_selfplay_moves(mzgo_engine* e, int moves, void* stream) {
  if (!e || e->C == 0 || moves < 1) return fail(MZGO_EINVAL, "bad argument");
  int rc = e->sync_weights();
  if (rc) return rc;
  PlayParams pp;
  pp.temperature = e->cfg.temperature;
  pp.temperature_moves = e->cfg.temperature_moves;
  pp.komi = e->cfg.komi;
  pp.game_base = e->cfg.game_base;
  pp.epoch = e->epoch;
  pp.noise = e->noise;
  pp.noise_out = e->noise_out;
  pp.arena = 0;
  pp.moves = moves;
  if (e->tower) {
    // one move of every game: observation + representation tower + root,
    // S x (select, dynamics tower, expand), action choice + board step
    TowerHost& t = *e->tower;
    hipStream_t s = (hipStream_t)stream;
    const SearchParams sp = e->search_params();
    std::vector<int> st(e->G);
    for (int k = 0; k < moves; ++k) {
      // a tower move is ~43 launches per simulation, so once every game has
      // ended the remaining moves are not enqueued at all: every 4 moves the
      // host reads the slots' status (one small copy per ~4 x S towers)
      if (k > 0 && k % 4 == 0) {
        HIPCHK(hipMemcpyAsync(st.data(), e->E.status, e->G * sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (int rc = check_chain(e, s)) return rc;
        bool any = false;
        for (int v : st) any |= v == 0;
        if (!any) break;
      }
      HIPCHK(t.ts->obs(t.TA, sp, pp, e->E, e->G, s));
      HIPCHK(t.root_phase(sp, e->E, e->noise, (long long)e->M * e->A, 1, s));
      HIPCHK(t.simulations(sp, e->E, s));
      HIPCHK(t.ts->choose(t.TA, sp, pp, e->E, e->G, s));
    }
    // (a tower move is ~1.5 s of device work: one synchronisation per call
    // reports an expired chain wait of this call, MZGO_EHIP, and clears it)
    return check_chain(e, s);
  }
  return launch_selfplay(e, e->np, pp, (hipStream_t)stream);
}

int mzgo_arena_move(mzgo_engine* e, mzgo_engine* opponent, void* stream) {
  return mzgo_arena_moves(e, opponent, 1, stream);
}

int mzgo_arena_moves(mzgo_engine* e, mzgo_engine* opponent, int moves, void* stream) {
  if (!e || !opponent || e->C == 0 || moves < 1) return fail(MZGO_EINVAL, "bad argument");
  if (e->tower || opponent->tower) return fail(MZGO_EINVAL, "the arena runs the reference network only (tower 0)");
  if (opponent->N != e->N || opponent->C != e->C)
    return fail(MZGO_EINVAL, "arena engines differ in board size / latent_dim (%d/%d vs %d/%d)", e->N, e->C,
                opponent->N, opponent->C);
  int rc = e->sync_weights();
  if (rc) return rc;
  rc = opponent->sync_weights();
  if (rc) return rc;
  PlayParams pp;
  pp.temperature = e->cfg.temperature;
  pp.temperature_moves = e->cfg.temperature_moves;
  pp.komi = e->cfg.komi;
  pp.game_base = e->cfg.game_base;
  pp.epoch = e->epoch;
  pp.noise = e->noise;
  pp.noise_out = e->noise_out;
  pp.arena = 1;
  pp.moves = moves;
  return launch_selfplay(e, opponent->np, pp, (hipStream_t)stream);
}

int mzgo_dyn_conv_backward_workspace(int B, int C, int64_t* bytes_host) {
  if (B < 1 || C < 16 || C % 16 || !bytes_host) return fail(MZGO_EINVAL, "bad argument (B=%d, C=%d)", B, C);
  *bytes_host = (int64_t)conv_bwd_workspace_bytes(B, C, C);
  return MZGO_OK;
}

int mzgo_dyn_conv_backward(const float* grad_out, const float* out, const float* latent, const int64_t* action,
                           const float* emb, const float* weight, int B, int C, int N, float* grad_latent,
                           float* grad_weight, float* grad_bias, void* workspace, int64_t workspace_bytes,
                           void* stream) {
  if (!grad_out || !out || !latent || !action || !emb || !weight || !grad_latent || !grad_weight || !grad_bias ||
      !workspace || B < 1 || C < 16 || C % 16 || N < 2 || N > 19)
    return fail(MZGO_EINVAL, "bad argument (B=%d, C=%d, N=%d)", B, C, N);
  if (workspace_bytes < (int64_t)conv_bwd_workspace_bytes(B, C, C))
    return fail(MZGO_EINVAL, "workspace too small: %lld < %lld bytes", (long long)workspace_bytes,
                (long long)conv_bwd_workspace_bytes(B, C, C));
  HIPCHK(conv_backward(grad_out, out, latent, action, emb, weight, B, C, C, N, grad_latent, grad_weight, grad_bias,
                       workspace, (hipStream_t)stream));
  return MZGO_OK;
}

int mzgo_conv3x3_relu_forward(const float* x, const int64_t* action, const float* emb, const float* weight,
                              const float* bias, int B, int Cin, int Cout, int N, float* out, void* stream) {
  if (!x || !weight || !bias || !out || (emb && !action) || B < 1 || Cin < 1 || Cout < 1 || N < 2 || N > 19)
    return fail(MZGO_EINVAL, "bad argument (B=%d, Cin=%d, Cout=%d, N=%d)", B, Cin, Cout, N);
  HIPCHK(conv_forward(x, action, emb, weight, bias, B, Cin, Cout, N, out, (hipStream_t)stream));
  return MZGO_OK;
}

int mzgo_conv3x3_backward_workspace(int B, int Cin, int Cout, int64_t* bytes_host) {
  if (B < 1 || Cin < 1 || Cout < 1 || !bytes_host)
    return fail(MZGO_EINVAL, "bad argument (B=%d, Cin=%d, Cout=%d)", B, Cin, Cout);
  *bytes_host = (int64_t)conv_bwd_workspace_bytes(B, Cin, Cout);
  return MZGO_OK;
}

int mzgo_conv3x3_backward(const float* grad_out, const float* out, const float* x, const int64_t* action,
                          const float* emb, const float* weight, int B, int Cin, int Cout, int N, float* grad_x,
                          float* grad_weight, float* grad_bias, void* workspace, int64_t workspace_bytes,
                          void* stream) {
  if (!grad_out || !out || !x || (emb && !action) || !weight || !grad_weight || !grad_bias || !workspace || B < 1 ||
      Cin < 1 || Cout < 1 || N < 2 || N > 19)
    return fail(MZGO_EINVAL, "bad argument (B=%d, Cin=%d, Cout=%d, N=%d)", B, Cin, Cout, N);
  if (workspace_bytes < (int64_t)conv_bwd_workspace_bytes(B, Cin, Cout))
    return fail(MZGO_EINVAL, "workspace too small: %lld < %lld bytes", (long long)workspace_bytes,
                (long long)conv_bwd_workspace_bytes(B, Cin, Cout));
  HIPCHK(conv_backward(grad_out, out, x, action, emb, weight, B, Cin, Cout, N, grad_x, grad_weight, grad_bias,
                       workspace, (hipStream_t)stream));
  return MZGO_OK;
}

int mzgo_tower_timing(mzgo_engine* e, int enable, double* tower_ms, int64_t* towers) {
  if (!e || !e->tower) return fail(MZGO_EINVAL, "not a tower engine");
  TowerHost& t = *e->tower;
  HIPCHK(t.harvest());
  if (tower_ms) *tower_ms = t.tower_ms;
  if (towers) *towers = t.towers_timed;
  t.tower_ms = 0.0;
  t.towers_timed = 0;
  t.timing = enable != 0;
  return MZGO_OK;
}

int mzgo_selfplay_inject_noise(mzgo_engine* e, const double* noise) {
  if (!e) return fail(MZGO_EINVAL, "null engine");
  e->noise = noise;
  return MZGO_OK;
}

int mzgo_selfplay_record_noise(mzgo_engine* e, double* dst) {
  if (!e) return fail(MZGO_EINVAL, "null engine");
  if (e->tower) return fail(MZGO_EINVAL, "the noise record covers the reference-network engine (tower 0)");
  e->noise_out = dst;
  return MZGO_OK;
}

int mzgo_tower_record_nodes(mzgo_engine* e, float* dst) {
  if (!e || !e->tower) return fail(MZGO_EINVAL, "not a tower engine");
  e->tower->TA.node_out = dst;
  return MZGO_OK;
}

int mzgo_selfplay_counters(mzgo_engine* e, uint64_t* out, void* stream) {
  if (!e || !out) return fail(MZGO_EINVAL, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  unsigned long long c[kCounters] = {};
  std::vector<int> st(e->G);
  HIPCHK(hipMemcpyAsync(c, e->E.counters, sizeof c, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(st.data(), e->E.status, e->G * sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (int rc = check_chain(e, s)) return rc;
  int playing = 0;
  for (int v : st) playing += v == 0;
  out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = (uint64_t)playing; out[4] = c[3]; out[5] = c[4];
  out[6] = c[5]; out[7] = c[6]; out[8] = c[7];
  if (c[8] != 0) {                   // a mzgo_stream_wait_started gate gave up (bounded wait)
    const unsigned long long zero = 0;
    HIPCHK(hipMemcpyAsync(e->E.counters + 8, &zero, sizeof zero, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    return fail(MZGO_EHIP, "mzgo_stream_wait_started: %llu gate(s) gave up before the target count", c[8]);
  }
  return MZGO_OK;
}

int mzgo_records_export(mzgo_engine* e, int g, int32_t* length, int32_t* status, int8_t* stones,
                        uint8_t* invd, uint8_t* flags, int32_t* action, double* value, double* policy,
                        double* reward, double* final_reward, void* stream) {
  if (!e || e->C == 0 || g < 0 || g >= e->G) return fail(MZGO_EINVAL, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  int meta[4], st = 0;
  HIPCHK(hipMemcpyAsync(meta, e->E.meta + (size_t)g * 4, 16, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(&st, e->E.status + g, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (int rc = check_chain(e, s)) return rc;
  const int L = meta[3];
  if (length) *length = L;
  if (status) *status = st;
  const size_t M = e->M, CELLS = e->CELLS, A = e->A, base = (size_t)g * M;
  if (L > 0) {
    if (stones) HIPCHK(hipMemcpyAsync(stones, e->E.rec_stones + base * CELLS, L * CELLS, hipMemcpyDeviceToHost, s));
    if (invd) HIPCHK(hipMemcpyAsync(invd, e->E.rec_invd + base * CELLS, L * CELLS, hipMemcpyDeviceToHost, s));
    if (flags) HIPCHK(hipMemcpyAsync(flags, e->E.rec_flags + base, L, hipMemcpyDeviceToHost, s));
    if (action) HIPCHK(hipMemcpyAsync(action, e->E.rec_action + base, L * 4, hipMemcpyDeviceToHost, s));
    if (value) HIPCHK(hipMemcpyAsync(value, e->E.rec_value + base, L * 8, hipMemcpyDeviceToHost, s));
    if (policy) HIPCHK(hipMemcpyAsync(policy, e->E.rec_policy + base * A, L * A * 8, hipMemcpyDeviceToHost, s));
    if (reward) HIPCHK(hipMemcpyAsync(reward, e->E.rec_reward + base, L * 8, hipMemcpyDeviceToHost, s));
  }
  if (final_reward) HIPCHK(hipMemcpyAsync(final_reward, e->E.final_reward + g, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return MZGO_OK;
}

#ifdef MZGO_STAMPS
// Diagnostic build only: copy (and zero) the per-slot phase cycle sums.
int mzgo_debug_stamps(mzgo_engine* e, unsigned long long* host) {
  if (!e || !e->E.stamps) return fail(MZGO_EINVAL, "no stamps");
  const size_t n = (size_t)e->TS * kStampPhases;     // every tree slot's row (TS >= G)
  HIPCHK(hipMemcpy(host, e->E.stamps, n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemset(e->E.stamps, 0, n * 8));
  return MZGO_OK;
}
#endif

// A gate for a collective (mzgo_stream_wait_started, a diagnostic entry
// point): one wave, no LDS and a handful of registers, so it sits beside a
// self-play workgroup on any CU; it returns once *count >= target, or after
// a bounded ~seconds wait, which it records in *expired (reported by the next
// mzgo_selfplay_counters call)
__global__ void __launch_bounds__(64) k_wait_count(const unsigned long long* count, unsigned long long target,
                                                  unsigned long long* expired) {
  if (threadIdx.x != 0) return;
  for (long long spins = 0; spins < (1ll << 26); ++spins) {
    if (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return;
    __builtin_amdgcn_s_sleep(16);
  }
  atomicAdd(expired, 1ull);
}

int mzgo_stream_wait_started(mzgo_engine* e, uint64_t target, void* stream) {
  if (!e || e->C == 0) return fail(MZGO_EINVAL, "bad argument");
  // tower engines run a move as many small launches and never count
  // workgroups_started: the gate would only time out
  if (e->tower) return fail(MZGO_EINVAL, "mzgo_stream_wait_started: not for tower engines");
  hipLaunchKernelGGL(k_wait_count, dim3(1), dim3(64), 0, (hipStream_t)stream, e->E.counters + 6,
                     (unsigned long long)target, e->E.counters + 8);
  HIPCHK(hipGetLastError());
  return MZGO_OK;
}

// Packed records of all G slots, for the multi-GPU gather (layout in mzgo.h).
int mzgo_records_pack(mzgo_engine* e, uint8_t* dst, int64_t capacity, int64_t* bytes_needed, void* stream) {
  if (!e || e->C == 0) return fail(MZGO_EINVAL, "bad argument");
  const size_t G = e->G, M = e->M, CELLS = e->CELLS, A = e->A;
  const size_t sizes[] = {G * M * CELLS, G * M * CELLS, G * M, G * M * 4, G * M * 8, G * M * A * 8,
                          G * M * 8, G * 4 * 4, G * 4, G * 8};
  const void* srcs[] = {e->E.rec_stones, e->E.rec_invd, e->E.rec_flags, e->E.rec_action, e->E.rec_value,
                        e->E.rec_policy, e->E.rec_reward, e->E.meta, e->E.status, e->E.final_reward};
  size_t total = 0;
  for (size_t s : sizes) total += (s + 15) / 16 * 16;
  if (bytes_needed) *bytes_needed = (int64_t)total;
  if (!dst) return MZGO_OK;
  if (capacity < (int64_t)total) return fail(MZGO_EINVAL, "records_pack: buffer of %lld bytes, need %zu", (long long)capacity, total);
  size_t off = 0;
  for (int i = 0; i < 10; ++i) {
    HIPCHK(hipMemcpyAsync(dst + off, srcs[i], sizes[i], hipMemcpyDeviceToDevice, (hipStream_t)stream));
    off += (sizes[i] + 15) / 16 * 16;
  }
  return MZGO_OK;
}

}  // extern "C"

// mzgo_tower_host.hpp -- host side of the residual-tower engine (BASELINE
// config 5): the state_dict of mzgo/resnet.py's ResMuZeroNet, weight packing,
// device buffers and the launch sequences of a move / a search / the
// drop-in inference calls.  Included by mzgo_capi.hip (the engine owns one
// TowerHost when mzgo_config.tower is 1).
#pragma once
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <type_traits>
#include <vector>

#include "mzgo_tower_dispatch.hpp"

namespace mzgo {

// f32 -> bf16 bits, round to nearest even (the device's v_cvt_pk_bf16_f32)
inline uint16_t bf16_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
inline float bf16_round(float f) {
  uint32_t u = (uint32_t)bf16_bits(f) << 16;
  float r;
  std::memcpy(&r, &u, 4);
  return r;
}

// conv weight W[cout][cin][3][3] (f32) -> bf16 tiles [co chunk][ci chunk][tap][64 cout][64 cin],
// the 16-byte pieces of row r at position piece ^ ((r >> 1) & 7) (mzgo_tower.hpp)
inline std::vector<uint16_t> pack_tconv(const float* W, int COUT, int CIN) {
  const int CO = COUT / 64, CI = (CIN + 63) / 64;
  std::vector<uint16_t> out((size_t)CO * CI * 9 * 64 * 64, 0);
  for (int cg = 0; cg < CO; ++cg)
    for (int cc = 0; cc < CI; ++cc)
      for (int t = 0; t < 9; ++t)
        for (int r = 0; r < 64; ++r)
          for (int k = 0; k < 64; ++k) {
            const int co = cg * 64 + r, ci = cc * 64 + k;
            const float v = ci < CIN ? W[((size_t)co * CIN + ci) * 9 + t] : 0.f;
            const size_t tile = (((size_t)cg * CI + cc) * 9 + t) * 64 * 64;
            out[tile + (size_t)r * 64 + (((k >> 3) ^ ((r >> 1) & 7)) << 3) + (k & 7)] = bf16_bits(v);
          }
  return out;
}

struct TowerHost {
  int N = 0, C = 0, CC = 0, blocks = 0, G = 0, S = 0, A = 0, P = 0, CS = 0;
  const TowerSet* ts = nullptr;
  // device buffers (owned by the engine's allocation list)
  TowerArrays TA{};
  bf16* t0 = nullptr; bf16* t1 = nullptr;
  // drop-in inference scratch, grown on demand
  bf16* ib = nullptr; bf16* ob = nullptr; bf16* s0 = nullptr; bf16* s1 = nullptr;
  float* shp = nullptr; int* sact = nullptr;
  int scap = 0;
  // weights
  void* d_wb = nullptr; size_t d_wb_bytes = 0;        // bf16 conv tiles
  float* d_wf = nullptr; size_t d_wf_bytes = 0;       // f32: biases, E table, heads, scalars
  struct Conv { const bf16* w; const float* b; int cin_chunks; };
  std::vector<Conv> rep, dyn;                         // conv_in then (conv1, conv2) per block
  const float* etab = nullptr;
  HeadScalars hs{};

  // optional timing of the dynamics towers (bench.py --config 5): one event
  // pair around every kTimeEvery-th simulation step's tower (one leaf per
  // game), or around every batched step's tower, on the launch stream (an
  // event record between two kernels costs a ~3 us dispatch gap: around every
  // one-leaf tower that was 0.5 % of the simulation time)
  static constexpr int kTimeEvery = 16;
  bool timing = false;
  std::vector<hipEvent_t> evs;
  std::vector<long long> ev_boards;   // boards of the tower behind each event pair
  size_t ev_used = 0;
  long long towers_timed = 0;         // board-towers: boards summed over the timed towers
  double tower_ms = 0.0;

  // batched simulation steps (k_tbatch, mzgo_tower.hpp; MZGO_TOWER_BATCH=1):
  // per game up to bq_cap pending entries (the root's children: min(A, S); a
  // non-root leaf's speculative batch: MZGO_TOWER_SPEC, default kSpecCap), so
  // up to G * bq_cap boards per step.  The default keeps one leaf per game
  // per step (k_tselect / k_texpand).  kSpecCap = 1: on the
  // config-5 network the next simulations' root children are predicted for
  // ~7-8 of 16, so speculative entries would cost more
  // towers than larger batches save with the current conv kernel.
  static constexpr int kSpecCap = 1;
  int bq_cap = 0, maxb = 0;
  int* h_total = nullptr;             // pinned: the step's board count
  long long steps_run = 0;
  // the batched steps' buffers (maxb boards), allocated on first use: the
  // tower's two scratch activations and head partials per board, the
  // pending entries and the step's board list
  bf16* bt0 = nullptr; bf16* bt1 = nullptr; float* bhp = nullptr;
  std::vector<void*> batch_allocs;
  hipError_t ensure_batch(hipStream_t s) {
    if (bt0) return hipSuccess;
    hipError_t e;
    const size_t MB = (size_t)maxb;
    auto get = [&](auto** p, size_t n) {
      void* v = nullptr;
      hipError_t r = hipMalloc(&v, n * sizeof(**p) + 256);
      if (r == hipSuccess) { batch_allocs.push_back(v); *p = reinterpret_cast<std::remove_pointer_t<decltype(p)>>(v); }
      return r;
    };
    if ((e = get(&bt0, MB * slot())) != hipSuccess || (e = get(&bt1, MB * slot())) != hipSuccess ||
        (e = get(&bhp, MB * CC * 3 * CS)) != hipSuccess || (e = get(&TA.bq_leaf, MB)) != hipSuccess ||
        (e = get(&TA.bq_act, MB)) != hipSuccess || (e = get(&TA.bq_rv, 2 * MB)) != hipSuccess ||
        (e = get(&TA.b_in, MB)) != hipSuccess || (e = get(&TA.b_out, MB)) != hipSuccess ||
        (e = get(&TA.b_act, MB)) != hipSuccess || (e = get(&TA.b_game, MB)) != hipSuccess ||
        (e = get(&TA.b_ent, MB)) != hipSuccess)
      return e;
    // zero borders of the scratch activations (the conv's padding is never written)
    if ((e = hipMemsetAsync(bt0, 0, MB * slot() * sizeof(bf16), s)) != hipSuccess) return e;
    return hipMemsetAsync(bt1, 0, MB * slot() * sizeof(bf16), s);
  }
  void free_batch() {
    for (void* p : batch_allocs) (void)hipFree(p);
    batch_allocs.clear();
    bt0 = bt1 = nullptr;
    bhp = nullptr;
  }

  long long slot() const { return (long long)CC * P * 64; }

  // k_tconv_chain: a tower's convs in one launch when all of its nb x CC
  // workgroups (one per CU) are resident at once; MZGO_TCONV_CHAIN=0 keeps
  // one k_tconv_ks launch per conv.  The layer tables live on the device,
  // one per distinct tower call (the dynamics tower's is the same every
  // simulation); the per-(board, cout chunk) flags count layers done.
  int ncu = -1;
  unsigned* cflags = nullptr; int cflags_n = 0;
  unsigned long long* cxcc = nullptr;
  int* cerr = nullptr;
  unsigned cseq = 0;
  // The layer tables: a ring of kChainSlots device slots, each filled from
  // its own pinned staging copy by an async upload on the launch stream.
  // Stream order puts an upload after every earlier launch on the stream
  // (those reading the slot's previous table) and before the launch that
  // reads it; the event behind the upload guards the staging copy (a host
  // wait only if a slot comes round again before its last upload ran).  A
  // call whose table is in a slot already (the dynamics tower's, every
  // simulation) uploads nothing.  A slot last used on another stream is
  // reused after that stream drains (calls of one engine on several streams).
  static constexpr int kChainSlots = 16;
  struct ChainBuf {
    std::vector<TConvArgs> host;       // the table in the slot (empty: none)
    TConvArgs* dev = nullptr;          // device slot, `cap` entries
    TConvArgs* pin = nullptr;          // pinned staging, `cap` entries
    int cap = 0;
    hipEvent_t done = nullptr;         // recorded behind the slot's last upload
    hipStream_t stream = nullptr;      // of the slot's last launch
  };
  std::vector<ChainBuf> chains;
  int chain_next = 0;
  bool chain_ok(int nb) {
    const char* env = getenv("MZGO_TCONV_CHAIN");                // (read per tower: tests switch it)
    if ((env && atoi(env) == 0) || !ts->chain) return false;
    if (ncu < 0) {
      int dev = 0;
      ncu = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        ncu = 0;
    }
    return nb * CC <= ncu;
  }
  hipError_t launch_chain(const std::vector<TConvArgs>& L, int nb, hipStream_t s) {
    hipError_t e;
    if (cflags_n < nb * CC) {
      if (cflags) (void)hipFree(cflags);
      if (cxcc) (void)hipFree(cxcc);
      cflags = nullptr;
      cxcc = nullptr;
      if ((e = hipMalloc(&cflags, (size_t)nb * CC * sizeof(unsigned))) != hipSuccess) return e;
      if ((e = hipMemset(cflags, 0, (size_t)nb * CC * sizeof(unsigned))) != hipSuccess) return e;
      if ((e = hipMalloc(&cxcc, (size_t)nb * CC * sizeof(unsigned long long))) != hipSuccess) return e;
      if ((e = hipMemset(cxcc, 0xFF, (size_t)nb * CC * sizeof(unsigned long long))) != hipSuccess) return e;
      cflags_n = nb * CC;
      cseq = 0;
    }
    if (!cerr) {
      if ((e = hipMalloc(&cerr, sizeof(int))) != hipSuccess) return e;
      if ((e = hipMemset(cerr, 0, sizeof(int))) != hipSuccess) return e;
    }
    if (chains.empty()) chains.resize(kChainSlots);
    ChainBuf* slot = nullptr;
    for (ChainBuf& c : chains)
      if (c.host.size() == L.size() && std::memcmp(c.host.data(), L.data(), L.size() * sizeof(TConvArgs)) == 0)
        slot = &c;
    if (!slot) {
      slot = &chains[chain_next];
      chain_next = (chain_next + 1) % kChainSlots;
      ChainBuf& c = *slot;
      // the staging copy of the slot's last upload: free once that upload ran
      if (c.done && (e = hipEventSynchronize(c.done)) != hipSuccess) return e;
      if (c.dev && c.stream != s && (e = hipStreamSynchronize(c.stream)) != hipSuccess) return e;
      c.host.clear();
      if (c.cap < (int)L.size()) {
        // (a larger slot: launches still reading the old one come first)
        if (c.dev && (e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (c.dev) (void)hipFree(c.dev);
        if (c.pin) (void)hipHostFree(c.pin);
        c.dev = nullptr;
        c.pin = nullptr;
        c.cap = 0;
        const int cap = (int)L.size() < 64 ? 64 : (int)L.size();
        if ((e = hipMalloc(&c.dev, cap * sizeof(TConvArgs))) != hipSuccess) return e;
        if ((e = hipHostMalloc(&c.pin, cap * sizeof(TConvArgs), hipHostMallocDefault)) != hipSuccess) return e;
        c.cap = cap;
      }
      if (!c.done && (e = hipEventCreateWithFlags(&c.done, hipEventDisableTiming)) != hipSuccess) return e;
      std::memcpy(c.pin, L.data(), L.size() * sizeof(TConvArgs));
      if ((e = hipMemcpyAsync(c.dev, c.pin, L.size() * sizeof(TConvArgs), hipMemcpyHostToDevice, s)) != hipSuccess)
        return e;
      if ((e = hipEventRecord(c.done, s)) != hipSuccess) return e;
      c.host = L;
    }
    // a slot found by its contents may have been uploaded on another stream:
    // this launch reads it only after that upload
    if (slot->stream && slot->stream != s && slot->done && (e = hipStreamWaitEvent(s, slot->done, 0)) != hipSuccess)
      return e;
    const TConvArgs* dev = slot->dev;
    slot->stream = s;
    // MZGO_TCONV_CHAIN_SPIN: the waits' bound (test hook: a negative bound
    // makes every wait expire, which every API call must then report)
    long long spin_max = 1ll << 24;
    if (const char* v = getenv("MZGO_TCONV_CHAIN_SPIN")) spin_max = atoll(v);
    const TConvChain ch{dev, (int)L.size(), cflags, cxcc, cseq, cerr, spin_max};
    cseq += (unsigned)L.size();
    return ts->chain(ch, nb * CC, s);
  }
  // a chain wait expired (results of those launches are wrong): read (and
  // cleared, once reported) at every host synchronisation point of the
  // tower engine's API calls (mzgo_check_chain)
  hipError_t chain_error(hipStream_t s, bool& bad) {
    bad = false;
    if (!cerr) return hipSuccess;
    int v = 0;
    hipError_t e = hipMemcpyAsync(&v, cerr, sizeof(int), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    bad = v != 0;
    if (bad && e == hipSuccess) e = hipMemsetAsync(cerr, 0, sizeof(int), s);
    if (bad && e == hipSuccess) e = hipStreamSynchronize(s);
    return e;
  }
  void free_chains() {
    for (ChainBuf& c : chains) {
      if (c.done) (void)hipEventSynchronize(c.done);
      if (c.dev) (void)hipFree(c.dev);
      if (c.pin) (void)hipHostFree(c.pin);
      if (c.done) (void)hipEventDestroy(c.done);
    }
    chains.clear();
    if (cflags) (void)hipFree(cflags);
    if (cxcc) (void)hipFree(cxcc);
    if (cerr) (void)hipFree(cerr);
    cflags = nullptr;
    cxcc = nullptr;
    cerr = nullptr;
  }

  // boards: of the tower that starts at this mark (its end mark passes 0)
  hipError_t mark(hipStream_t s, long long boards = 0) {
    if (!timing) return hipSuccess;
    if (ev_used == evs.size()) {
      hipEvent_t e;
      hipError_t r = hipEventCreate(&e);
      if (r != hipSuccess) return r;
      evs.push_back(e);
      ev_boards.push_back(0);
    }
    ev_boards[ev_used] = boards;
    return hipEventRecord(evs[ev_used++], s);
  }
  // sum the recorded spans (synchronises) and recycle the events
  hipError_t harvest() {
    for (size_t i = 0; i + 1 < ev_used; i += 2) {
      hipError_t r = hipEventSynchronize(evs[i + 1]);
      if (r != hipSuccess) return r;
      float ms = 0.f;
      if ((r = hipEventElapsedTime(&ms, evs[i], evs[i + 1])) != hipSuccess) return r;
      tower_ms += ms;
      towers_timed += ev_boards[i];
    }
    ev_used = 0;
    return hipSuccess;
  }

  static std::vector<std::pair<std::string, std::vector<int64_t>>> specs(int C, int A, int blocks) {
    std::vector<std::pair<std::string, std::vector<int64_t>>> s;
    auto conv = [&](const std::string& k, int64_t co, int64_t ci) {
      s.push_back({k + ".weight", {co, ci, 3, 3}});
      s.push_back({k + ".bias", {co}});
    };
    conv("representation.conv_in", C, 6);
    for (int i = 0; i < blocks; ++i) {
      conv("representation.blocks." + std::to_string(i) + ".conv1", C, C);
      conv("representation.blocks." + std::to_string(i) + ".conv2", C, C);
    }
    s.push_back({"dynamics.action_embedding.weight", {A, C}});
    conv("dynamics.conv_in", C, C);
    for (int i = 0; i < blocks; ++i) {
      conv("dynamics.blocks." + std::to_string(i) + ".conv1", C, C);
      conv("dynamics.blocks." + std::to_string(i) + ".conv2", C, C);
    }
    s.push_back({"dynamics.reward_conv.weight", {1, C, 1, 1}});
    s.push_back({"dynamics.reward_conv.bias", {1}});
    s.push_back({"dynamics.fc_reward_hidden.weight", {16, 1}});
    s.push_back({"dynamics.fc_reward_hidden.bias", {16}});
    s.push_back({"dynamics.fc_reward_output.weight", {1, 16}});
    s.push_back({"dynamics.fc_reward_output.bias", {1}});
    s.push_back({"prediction.pass_logit", {1}});
    s.push_back({"prediction.value_conv.weight", {1, C, 1, 1}});
    s.push_back({"prediction.value_conv.bias", {1}});
    s.push_back({"prediction.value_fc.weight", {1, 1}});
    s.push_back({"prediction.value_fc.bias", {1}});
    s.push_back({"prediction.policy_conv.weight", {1, C, 1, 1}});
    s.push_back({"prediction.policy_conv.bias", {1}});
    return s;
  }

  // pack + upload (host f32 state_dict -> device).  The dynamics' first conv
  // adds the action embedding through the region table of mzgo_expand.hpp
  // (conv(x + emb[a]) = conv(x) + E[a][region] under zero padding), built from
  // the bf16-rounded weights the MFMA uses: the GEMM never sees emb.
  hipError_t upload(std::map<std::string, std::vector<float>>& sd,
                    std::vector<float> (*taps)(const float*, const float*, int, int)) {
    std::vector<uint16_t> wb;
    std::vector<size_t> woff;
    std::vector<std::string> order;
    auto addw = [&](const std::string& k, int cin) {
      woff.push_back(wb.size());
      order.push_back(k);
      std::vector<uint16_t> p = pack_tconv(sd[k + ".weight"].data(), C, cin);
      wb.insert(wb.end(), p.begin(), p.end());
    };
    addw("representation.conv_in", 6);
    for (int i = 0; i < blocks; ++i) {
      addw("representation.blocks." + std::to_string(i) + ".conv1", C);
      addw("representation.blocks." + std::to_string(i) + ".conv2", C);
    }
    addw("dynamics.conv_in", C);
    for (int i = 0; i < blocks; ++i) {
      addw("dynamics.blocks." + std::to_string(i) + ".conv1", C);
      addw("dynamics.blocks." + std::to_string(i) + ".conv2", C);
    }
    std::vector<float> wf;
    auto addf = [&](const std::vector<float>& v) {
      const size_t o = wf.size();
      wf.insert(wf.end(), v.begin(), v.end());
      wf.resize((wf.size() + 63) / 64 * 64, 0.f);
      return o;
    };
    std::vector<size_t> boff;
    for (const std::string& k : order) boff.push_back(addf(sd[k + ".bias"]));
    std::vector<float> wr = sd["dynamics.conv_in.weight"];
    for (float& x : wr) x = bf16_round(x);
    const size_t eoff = addf(taps(wr.data(), sd["dynamics.action_embedding.weight"].data(), C, A));
    std::vector<float> hw;
    for (const char* k : {"dynamics.reward_conv.weight", "prediction.value_conv.weight",
                          "prediction.policy_conv.weight"})
      hw.insert(hw.end(), sd[k].begin(), sd[k].end());
    const size_t hoff = addf(hw);
    const char* scal[] = {"dynamics.reward_conv.bias", "dynamics.fc_reward_hidden.weight",
                          "dynamics.fc_reward_hidden.bias", "dynamics.fc_reward_output.weight",
                          "dynamics.fc_reward_output.bias", "prediction.value_conv.bias",
                          "prediction.value_fc.weight", "prediction.value_fc.bias",
                          "prediction.policy_conv.bias", "prediction.pass_logit"};
    std::vector<size_t> soff;
    for (const char* k : scal) soff.push_back(addf(sd[k]));
    hipError_t e;
    if (wb.size() * 2 > d_wb_bytes) {
      if (d_wb) (void)hipFree(d_wb);
      d_wb = nullptr;
      if ((e = hipMalloc(&d_wb, wb.size() * 2)) != hipSuccess) return e;
      d_wb_bytes = wb.size() * 2;
    }
    if (wf.size() * 4 > d_wf_bytes) {
      if (d_wf) (void)hipFree(d_wf);
      d_wf = nullptr;
      if ((e = hipMalloc(&d_wf, wf.size() * 4)) != hipSuccess) return e;
      d_wf_bytes = wf.size() * 4;
    }
    if ((e = hipMemcpy(d_wb, wb.data(), wb.size() * 2, hipMemcpyHostToDevice)) != hipSuccess) return e;
    if ((e = hipMemcpy(d_wf, wf.data(), wf.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) return e;
    const bf16* bw = reinterpret_cast<const bf16*>(d_wb);
    rep.clear();
    dyn.clear();
    const int nrep = 1 + 2 * blocks;
    for (size_t i = 0; i < order.size(); ++i) {
      Conv c{bw + woff[i], d_wf + boff[i], (i == 0) ? 1 : CC};
      if ((int)i < nrep) rep.push_back(c); else dyn.push_back(c);
    }
    etab = d_wf + eoff;
    TA.headw = d_wf + hoff;
    const float* f = d_wf;
    hs.reward_b = f + soff[0]; hs.fc1_w = f + soff[1]; hs.fc1_b = f + soff[2]; hs.fc2_w = f + soff[3];
    hs.fc2_b = f + soff[4]; hs.value_b = f + soff[5]; hs.vfc_w = f + soff[6]; hs.vfc_b = f + soff[7];
    hs.policy_b = f + soff[8]; hs.pass_logit = f + soff[9];
    TA.hs = hs;
    return hipSuccess;
  }

  // One tower over nb boards: conv_in (in -> t0, or straight to out without
  // blocks), then per block conv1 (t0 -> t1) and conv2 (t1 + t0 -> t0; the
  // last block's into out) with the fused heads on the final conv.
  hipError_t tower(const std::vector<Conv>& L, const bf16* in, const int* in_idx, long long in_stride, bf16* out,
                   const int* out_idx, long long out_stride, const int* act, const int* active, int nb, bf16* a0,
                   bf16* a1, float* hpart, hipStream_t s) {
    TConvArgs c{};
    c.nboards = nb;
    c.co_chunks = CC;
    c.active = active;
    const long long sl = slot();
    std::vector<TConvArgs> layers;
    auto run = [&](const Conv& cv, const bf16* src, const int* sidx, long long sstr, bf16* dst, const int* didx,
                   long long dstr, const bf16* res, bool heads, const float* et) {
      c.in = src; c.in_idx = sidx; c.in_stride = sstr;
      c.out = dst; c.out_idx = didx; c.out_stride = dstr;
      c.res = res; c.res_idx = nullptr; c.res_stride = sl;
      c.w = cv.w; c.bias = cv.b; c.ci_chunks = cv.cin_chunks;
      c.etab = et; c.act = et ? act : nullptr;
      c.headw = heads ? TA.headw : nullptr; c.hpart = hpart;
      layers.push_back(c);
    };
    const int nb_ = (int)(L.size() - 1) / 2;
    const float* et = act ? etab : nullptr;
    if (nb_ == 0) {
      run(L[0], in, in_idx, in_stride, out, out_idx, out_stride, nullptr, true, et);
    } else {
      run(L[0], in, in_idx, in_stride, a0, nullptr, sl, nullptr, false, et);
      for (int k = 0; k < nb_; ++k) {
        const bool lastb = k == nb_ - 1;
        run(L[1 + 2 * k], a0, nullptr, sl, a1, nullptr, sl, nullptr, false, nullptr);
        run(L[2 + 2 * k], a1, nullptr, sl, lastb ? out : a0, lastb ? out_idx : nullptr, lastb ? out_stride : sl, a0,
            lastb, nullptr);
      }
    }
    if (layers.size() > 1 && chain_ok(nb)) return launch_chain(layers, nb, s);
    for (const TConvArgs& l : layers) {
      hipError_t e = ts->conv(l, s);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }

  // representation tower + root priors for the slots marked playing
  hipError_t root_phase(const SearchParams& sp, const EngineArrays& E, const double* noise, long long nstride,
                        int per_move, hipStream_t s) {
    hipError_t e;
    if ((e = tower(rep, TA.rep_in, nullptr, (long long)P * 64, TA.pool, TA.root_idx, slot(), nullptr, TA.playing, G,
                   t0, t1, TA.hpart, s)) != hipSuccess)
      return e;
    return ts->root(TA, sp, E, noise, nstride, per_move, G, s);
  }

  // S simulations of every game
  hipError_t simulations(const SearchParams& sp, const EngineArrays& E, hipStream_t s) {
    // batched steps only on request (MZGO_TOWER_BATCH=1, read per call):
    // measured on config 5 they do not pay with this conv kernel (DESIGN.md
    // §4b: 64.0 k sims/s with the root batch and one leaf per step after it,
    // 64.7 k one leaf per step throughout, 50.6 k / 38.1 k with 4 / 8
    // speculative entries, same call)
    const char* env = getenv("MZGO_TOWER_BATCH");
    if (!env || atoi(env) == 0) return simulations_one_leaf(sp, E, s);
    int spec = kSpecCap;
    if (const char* v = getenv("MZGO_TOWER_SPEC")) spec = atoi(v);
    spec = spec < 1 ? 1 : (spec > bq_cap ? bq_cap : spec);
    hipError_t e;
    if ((e = ensure_batch(s)) != hipSuccess) return e;
    TowerArrays TB = TA;                                  // the step kernels' view: per-board head partials
    TB.hpart = bhp;
    // one step: commit what the previous step evaluated, form the next batch
    // per game (k_tbatch), the step's board list (k_tboards); then the tower
    // over all of them and their heads.  The host reads the board count (the
    // grid of the next launches): one small synchronising copy per step.
    for (;;) {
      if ((e = ts->batch(TB, sp, E, G, bq_cap, spec, s)) != hipSuccess) return e;
      if ((e = hipMemcpyAsync(h_total, TA.b_total, sizeof(int), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
      if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
      const int nb = *h_total;
      if (nb <= 0) break;
      if (nb > maxb) return hipErrorInvalidValue;          // (cannot happen: bq_cap entries per game)
      ++steps_run;
      if ((e = mark(s, nb)) != hipSuccess) return e;
      if ((e = tower(dyn, TA.pool, TA.b_in, slot(), TA.pool, TA.b_out, slot(), TA.b_act, nullptr, nb, bt0, bt1,
                     bhp, s)) != hipSuccess)
        return e;
      if ((e = mark(s)) != hipSuccess) return e;
      if ((e = ts->bexpand(TB, sp, E, nb, s)) != hipSuccess) return e;
    }
    if (timing) return harvest();
    return hipSuccess;
  }

  // one leaf per game per step: select (all games) -> dynamics tower (all
  // leaves) -> expand + backup, S times
  hipError_t simulations_one_leaf(const SearchParams& sp, const EngineArrays& E, hipStream_t s) {
    hipError_t e;
    for (int i = 0; i < S; ++i) {
      const bool tm = i % kTimeEvery == 0;
      if ((e = ts->select(TA, sp, E, G, s)) != hipSuccess) return e;
      if (tm && (e = mark(s, G)) != hipSuccess) return e;
      if ((e = tower(dyn, TA.pool, TA.in_idx, slot(), TA.pool, TA.out_idx, slot(), TA.act, TA.evalact, G, t0, t1,
                     TA.hpart, s)) != hipSuccess)
        return e;
      if (tm && (e = mark(s)) != hipSuccess) return e;
      if ((e = ts->expand(TA, sp, E, G, s)) != hipSuccess) return e;
    }
    if (timing) return harvest();
    return hipSuccess;
  }
};

}  // namespace mzgo

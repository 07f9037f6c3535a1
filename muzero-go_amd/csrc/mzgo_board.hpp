// mzgo_board.hpp -- GymGo board rules as bit-exact integer device code.
//
// One workgroup steps one board held in LDS.  Groups are found
// by min-label propagation with pointer jumping (label = smallest cell index
// of the 4-connected component, as scipy.ndimage.label's components), and
// liberties are counted as distinct empty neighbour points per group.
//
// Restates upstream GymGo (not in the reference snapshot; SURVEY.md
// Appendix B, oracle/gogame.py): gogame.next_state (pass / double pass,
// placement, capture, simple ko), state_utils.compute_invalid_moves (suicide
// rule from the opponent's perspective) and gogame.areas / winning (area
// scoring).  Reference call sites: self_play.py:479 (env.step), :502/:513
// (env.winner), :152/:363 (the INVD plane).
#pragma once
#include "mzgo_common.hpp"

namespace mzgo {

// Board state of one game as the engine keeps it (global memory, per slot).
struct BoardMeta {
  int turn;      // 0 = black to move, 1 = white
  int passed;    // previous move was a pass (PASS plane)
  int done;      // game ended by double pass (DONE plane)
  int moves;     // moves played
};

// LDS working set for one board step.  stone/invd persist across the move;
// label/libs/gsize are scratch that may alias the conv staging buffer.
template <class G>
struct BoardLds {
  int8_t* stone;   // [CELLS] 0 empty, 1 black, 2 white
  uint8_t* invd;   // [CELLS] INVD plane for the side to move
  int* label;      // [CELLS]
  int* libs;       // [CELLS]
  int* gsize;      // [CELLS]
  int* killed;     // [4]
  int* misc;       // [8] 0: nkilled, 1: boxed, 2: ko point, 3/4: area reduction
};

// Who steps a board (the board functions' team parameter T): the whole
// workgroup.  (One wave alone was tried for self-play's end of move: the
// label propagation ran slower without the other waves' lanes.)
template <class G>
struct BoardWG {
  static constexpr int SIZE = G::THREADS;
  __device__ static int id() { return tid_local(); }
  __device__ static void sync() { __syncthreads(); }
  __device__ static bool any(int v) { return __syncthreads_or(v) != 0; }
  __device__ static bool leader() { return tid_local() == 0; }
};
template <class G>
__device__ __forceinline__ bool nbr(int c, int d, int& n) {
  const int r = c / G::N, col = c - r * G::N;
  switch (d) {
    case 0: if (r == 0) return false; n = c - G::N; return true;
    case 1: if (r == G::N - 1) return false; n = c + G::N; return true;
    case 2: if (col == 0) return false; n = c - 1; return true;
    default: if (col == G::N - 1) return false; n = c + 1; return true;
  }
}

// label[c] = min cell index of c's 4-connected component of cells whose
// class(c) is equal; -1 where class(c) == 0.
template <class G, class T, class ClassFn>
__device__ __forceinline__ void label_components(int* label, ClassFn cls) {
  for (int c = T::id(); c < G::CELLS; c += T::SIZE) label[c] = cls(c) ? c : -1;
  T::sync();
  for (int it = 0; it < G::CELLS + 2; ++it) {
    int changed = 0;
    for (int c = T::id(); c < G::CELLS; c += T::SIZE) {
      const int k = cls(c);
      if (!k) continue;
      int m = label[c];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        int n;
        if (nbr<G>(c, d, n) && cls(n) == k) { int ln = label[n]; m = ln < m ? ln : m; }
      }
      int j = label[m];
      m = j < m ? j : m;
      if (m < label[c]) { label[c] = m; changed = 1; }
    }
    if (!T::any(changed)) break;
  }
}

// libs[g] = #distinct empty points adjacent to group g; gsize[g] = #stones
template <class G, class T>
__device__ __forceinline__ void count_liberties(BoardLds<G>& b, bool sizes) {
  for (int c = T::id(); c < G::CELLS; c += T::SIZE) { b.libs[c] = 0; if (sizes) b.gsize[c] = 0; }
  T::sync();
  for (int c = T::id(); c < G::CELLS; c += T::SIZE) {
    if (b.stone[c]) {
      if (sizes) atomicAdd(&b.gsize[b.label[c]], 1);
      continue;
    }
    int seen[4];
    int ns = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      int n;
      if (nbr<G>(c, d, n) && b.stone[n]) {
        int l = b.label[n];
        bool dup = false;
        for (int i = 0; i < ns; ++i) dup |= seen[i] == l;
        if (!dup) { seen[ns++] = l; atomicAdd(&b.libs[l], 1); }
      }
    }
  }
  T::sync();
}

// INVD plane for the opponent of ``mover`` (state_utils.compute_invalid_moves)
template <class G, class T>
__device__ __forceinline__ void compute_invalid(BoardLds<G>& b, int mover, int ko) {
  for (int c = T::id(); c < G::CELLS; c += T::SIZE) {
    uint8_t inv;
    if (b.stone[c]) {
      inv = 1;
    } else {
      bool boxed = true, maybe_bad = false, surely_ok = false;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        int n;
        if (!nbr<G>(c, d, n)) continue;          // off-board counts as occupied
        const int s = b.stone[n];
        if (!s) { boxed = false; continue; }
        const int lib = b.libs[b.label[n]];
        if (s - 1 == mover) { maybe_bad |= lib > 1; surely_ok |= lib == 1; }
        else                { maybe_bad |= lib == 1; surely_ok |= lib > 1; }
      }
      inv = (boxed && maybe_bad && !surely_ok) ? 1 : 0;
    }
    b.invd[c] = inv;
  }
  T::sync();
  if (ko >= 0 && T::leader()) b.invd[ko] = 1;
  T::sync();
}

enum : int { BOARD_OK = 0, BOARD_ERR_DONE = 1, BOARD_ERR_INVALID = 2, BOARD_ERR_RANGE = 3 };

// gogame.next_state(state, action, canonical=False) on the LDS board.
// Returns a BOARD_* status (uniform across the workgroup).
template <class G, class T = BoardWG<G>>
__device__ __forceinline__ int board_step(BoardLds<G>& b, BoardMeta& m, int action) {
  if (m.done) return BOARD_ERR_DONE;                 // GoEnv.step: assert not self.done
  if (action < 0 || action > G::CELLS) return BOARD_ERR_RANGE;
  const int player = m.turn;
  int ko = -1;
  if (action == G::CELLS) {                          // pass
    if (m.passed) m.done = 1;
    m.passed = 1;
    label_components<G, T>(b.label, [&](int c) { return (int)b.stone[c]; });
    count_liberties<G, T>(b, false);
  } else {
    if (b.invd[action]) return BOARD_ERR_INVALID;    // assert INVD == 0
    m.passed = 0;
    if (T::leader()) {
      b.stone[action] = (int8_t)(player + 1);
      bool boxed = true;
      for (int d = 0; d < 4; ++d) {
        int n;
        if (nbr<G>(action, d, n)) boxed &= b.stone[n] == 2 - player;   // opponent stone
      }
      b.misc[1] = boxed;
    }
    T::sync();
    label_components<G, T>(b.label, [&](int c) { return (int)b.stone[c]; });
    count_liberties<G, T>(b, true);
    // opponent groups adjacent to the new stone with no liberty die
    if (T::leader()) {
      int nk = 0;
      for (int d = 0; d < 4; ++d) {
        int n;
        if (!nbr<G>(action, d, n) || b.stone[n] != 2 - player) continue;
        const int l = b.label[n];
        bool dup = false;
        for (int i = 0; i < nk; ++i) dup |= b.killed[i] == l;
        if (!dup && b.libs[l] == 0) b.killed[nk++] = l;
      }
      b.misc[0] = nk;
      b.misc[2] = (nk == 1 && b.misc[1] && b.gsize[b.killed[0]] == 1) ? b.killed[0] : -1;
    }
    T::sync();
    const int nk = b.misc[0];
    ko = b.misc[2];
    if (nk > 0) {
      for (int c = T::id(); c < G::CELLS; c += T::SIZE) {
        if (b.stone[c] == 2 - player) {
          const int l = b.label[c];
          bool dead = false;
          for (int i = 0; i < nk; ++i) dead |= b.killed[i] == l;
          if (dead) b.stone[c] = 0;
        }
      }
      T::sync();
      count_liberties<G, T>(b, false);                   // labels of survivors still hold
    }
  }
  compute_invalid<G, T>(b, player, ko);
  m.turn = 1 - m.turn;
  m.moves += 1;
  return BOARD_OK;
}

// gogame.winning: sign(black_area - white_area - komi), area (Tromp-Taylor).
template <class G, class T = BoardWG<G>>
__device__ __forceinline__ double board_winning(BoardLds<G>& b, double komi) {
  label_components<G, T>(b.label, [&](int c) { return b.stone[c] == 0 ? 1 : 0; });
  for (int c = T::id(); c < G::CELLS; c += T::SIZE) { b.libs[c] = 0; b.gsize[c] = 0; }
  T::sync();
  for (int c = T::id(); c < G::CELLS; c += T::SIZE) {
    if (b.stone[c]) continue;
    int f = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      int n;
      if (nbr<G>(c, d, n) && b.stone[n]) f |= b.stone[n];   // 1 black, 2 white
    }
    if (f) atomicOr(&b.libs[b.label[c]], f);
    atomicAdd(&b.gsize[b.label[c]], 1);
  }
  T::sync();
  int black = 0, white = 0;
  for (int c = T::id(); c < G::CELLS; c += T::SIZE) {
    if (b.stone[c] == 1) black++;
    else if (b.stone[c] == 2) white++;
    else if (b.label[c] == c) {
      if (b.libs[c] == 1) black += b.gsize[c];
      else if (b.libs[c] == 2) white += b.gsize[c];
    }
  }
  // block reduction of (black, white) through LDS
  if (T::leader()) { b.misc[3] = 0; b.misc[4] = 0; }
  T::sync();
  atomicAdd(&b.misc[3], black);
  atomicAdd(&b.misc[4], white);
  T::sync();
  const double diff = (double)b.misc[3] - (double)b.misc[4] - komi;
  T::sync();
  return diff > 0 ? 1.0 : (diff < 0 ? -1.0 : 0.0);
}

}  // namespace mzgo

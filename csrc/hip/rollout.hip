// Fast-rollout playouts on the GPU: one wavefront plays one game to the end.
//
// The policy is the same linear softmax as the native one (csrc/mcts/rollout.hpp): per candidate
// move, 7 binary features + a 3x3 pattern weight; candidates are empty points that are not an
// own single-point eye and are legal (no suicide, not the ko point). Sampling uses the Gumbel-max
// trick (argmax of logit + Gumbel noise == a draw from the softmax over the legal candidates,
// i.e. the same distribution the CPU rejection sampler draws from), so a move costs one wave-wide
// max reduction.
//
// Latency design (a playout is ~430 strictly sequential moves, so per-move latency is the cost):
//   * board state per wave in LDS: one byte per point ("cell": colour in bits 0-1, the liberty
//     count of its group clamped to 3 in bits 2-3 — every feature only distinguishes 1 / 2 / 3+),
//     a group label per stone and a liberty counter per label;
//   * everything in a candidate's logit except the last-move terms is a function of its 3x3
//     neighbourhood of cells, so it is cached per point for both players to move ("base") and
//     recomputed only where a cell of that neighbourhood changed in the last move (the placed
//     stone, captured stones, groups whose clamped liberty count moved) — a handful of points per
//     move instead of all 361; the 256 KB pattern table is only read for those;
//   * per move every lane then just reads its points' cached bases, adds the last-move features
//     and Gumbel noise, and one wave-wide argmax picks the move;
//   * neighbour indices are computed (p +- 1, p +- S with edge tests; the board size is a template
//     constant for 19x19 / 13x13 / 9x9) instead of read from an LDS table: fewer LDS instructions
//     per move and 6 KB less LDS per block (5 -> 6 blocks per CU).
// A move: place, remove captured groups (opponent neighbours whose count was 1), relabel the
// merged own groups to the new stone, recount liberties (each empty point adds 1 to each distinct
// neighbouring label, LDS atomics), refresh the cells and mark changed neighbourhoods dirty.
// Rules match the native engine in light mode: simple ko (reference rule Q15), no superko, end
// of game after two passes with WHITE to move (Q3), area score with single-point eyeish
// empties and komi, minus passes (Q12).
#include "common.h"

using namespace rag;

namespace {

// games (waves) per block: 4 (256 threads, 26 KB LDS) or 1 (64 threads, 6.5 KB LDS, so a
// block fits next to two 76 KB conv blocks on a CU while the search's nets run): RAG_ROLLOUT_GPB

constexpr uint8_t kOff = 3;  // colour code of an off-board neighbour

template <int PM>
struct alignas(16) GameLds {
  float base[2][PM];  // cached logit w/o last-move terms; [0] black to move, [1] white
  int lib[PM];
  int16_t lab[PM];
  uint8_t cell[PM];
  uint8_t chg[PM];
  uint8_t dirty[PM];
  int16_t list[PM];  // compacted dirty points (refresh)
};

template <int PM, int GPB>
struct BlockLds {
  GameLds<PM> g[GPB];
};

// ring slot k of the 3x3 neighbourhood, clockwise from north ((x, y+1) first)
__device__ constexpr int kDx[8] = {0, 1, 1, 1, 0, -1, -1, -1};
__device__ constexpr int kDy[8] = {1, 1, 0, -1, -1, -1, 0, 1};

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

struct LaneRng {
  uint32_t s;
  __device__ float uniform() {  // (0, 1)
    s = s * 1664525u + 1013904223u;
    return ((hash32(s) >> 8) + 0.5f) * (1.0f / 16777216.0f);
  }
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void wave_argmax(float& key, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float k2 = __shfl_xor(key, o, 64);
    const int i2 = __shfl_xor(idx, o, 64);
    if (k2 > key || (k2 == key && i2 < idx)) {
      key = k2;
      idx = i2;
    }
  }
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int SC, int NPL, int PM>
struct Game {
  int S_rt;
  GameLds<PM>* L;
  int lane;

  __device__ __forceinline__ int S() const { return SC > 0 ? SC : S_rt; }
  __device__ __forceinline__ int P() const { return S() * S(); }
  // neighbour in ring slot k of p (-1 off board); orthogonal neighbours are ring slots 0 (N),
  // 2 (E), 4 (S), 6 (W), diagonals 1, 3, 5, 7
  __device__ __forceinline__ int ring(int p, int k) const {
    const int s = S();
    const int x = p / s, y = p - x * s;
    const int ax = x + kDx[k], ay = y + kDy[k];
    return (ax < 0 || ay < 0 || ax >= s || ay >= s) ? -1 : p + kDx[k] * s + kDy[k];
  }
  __device__ __forceinline__ int orth(int p, int i) const { return ring(p, 2 * i); }

  __device__ void init_labels() {
    const int P_ = P();
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P_) L->lab[p] = (L->cell[p] & 3) ? (int16_t)p : (int16_t)-1;
    }
    wave_sync();
    for (int it = 0; it < 4 * PM; ++it) {
      int changed = 0;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int p = lane + 64 * k;
        if (p >= P_) continue;
        const int c = L->cell[p] & 3;
        if (!c) continue;
        int m = L->lab[L->lab[p]];
        for (int i = 0; i < 4; ++i) {
          const int q = orth(p, i);
          if (q >= 0 && (L->cell[q] & 3) == c) m = min(m, (int)L->lab[q]);
        }
        if (m < L->lab[p]) {
          L->lab[p] = (int16_t)m;
          changed = 1;
        }
      }
      wave_sync();
      if (!__any(changed)) break;
    }
  }

  // liberty counters per label, then the clamped count into every stone's cell (flagging the
  // cells that changed). Every LDS load of a phase is issued for all of the lane's points before
  // the phase's first LDS write (uint8 cells alias everything, so the compiler cannot reorder
  // loads across a store): a few LDS round trips per move instead of a dependent chain per
  // neighbour.
  __device__ void recount_libs() {
    const int P_ = P();
    int nb[NPL][4];
    uint8_t cp[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      const bool in = p < P_;
      cp[k] = in ? L->cell[p] : (uint8_t)0;
#pragma unroll
      for (int i = 0; i < 4; ++i) nb[k][i] = in ? orth(p, i) : -1;
    }
    uint8_t cq[NPL][4];
#pragma unroll
    for (int k = 0; k < NPL; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) cq[k][i] = nb[k][i] >= 0 ? (uint8_t)(L->cell[nb[k][i]] & 3) : 0;
    int lq[NPL][4], lp[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      const bool empty = p < P_ && !(cp[k] & 3);
#pragma unroll
      for (int i = 0; i < 4; ++i) lq[k][i] = (empty && cq[k][i]) ? (int)L->lab[nb[k][i]] : -1;
      lp[k] = (p < P_ && (cp[k] & 3)) ? (int)L->lab[p] : -1;
    }
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P_) L->lib[p] = 0;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int l = lq[k][i];
        bool dup = l < 0;
#pragma unroll
        for (int j = 0; j < i; ++j) dup |= lq[k][j] == l;
        if (!dup) atomicAdd(&L->lib[l], 1);
      }
    }
    wave_sync();
    int lv[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) lv[k] = lp[k] >= 0 ? L->lib[lp[k]] : 0;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      if (lp[k] < 0) continue;
      const int p = lane + 64 * k;
      const uint8_t nc = (uint8_t)((cp[k] & 3) | (min(lv[k], 3) << 2));
      if (nc != cp[k]) {
        L->cell[p] = nc;
        L->chg[p] = 1;
      }
    }
    wave_sync();
  }

  // base logit (everything but the last-move terms) for both players from the packed 3x3
  // neighbourhood r (cells of ring slots 0..7, one byte each) and the two pattern weights
  __device__ __forceinline__ void base_from(int p, uint64_t r8, float patb, float patw,
                                            const float* __restrict__ w) {
    const int s = S();
    const int x = p / s, y = p - (p / s) * s;
    const bool edge = x == 0 || y == 0 || x == s - 1 || y == s - 1;
#pragma unroll
    for (int own = 1; own <= 2; ++own) {
      const int opp = 3 - own;
      int nnb = 0, own_nb = 0, empty_nb = 0, own_libs = 0;
      bool capture = false, own_atari = false, own_multi = false;
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        const int rk = (int)((r8 >> (8 * k)) & 0xff);
        const int c = rk & 3;
        if (c == kOff) continue;
        ++nnb;
        const int lc = rk >> 2;
        if (c == 0) {
          ++empty_nb;
        } else if (c == own) {
          ++own_nb;
          if (lc == 1) own_atari = true;
          else own_multi = true;
          own_libs += lc - 1;
        } else if (lc == 1) {
          capture = true;
        }
      }
      float v;
      bool cand = true;
      if (own_nb == nnb) {  // own single-point eye
        int bad = 0;
#pragma unroll
        for (int k = 1; k < 8; k += 2) bad += (int)((r8 >> (8 * k)) & 3) == opp;
        if (nnb < 4 ? bad == 0 : bad <= 1) cand = false;
      }
      if (empty_nb == 0 && !own_multi && !capture) cand = false;  // suicide
      if (cand) {
        v = own == 1 ? patb : patw;
        if (edge) v += w[6];
        if (capture) v += w[2];
        if (own_atari && (empty_nb >= 2 || capture)) v += w[1];
        if (!capture && empty_nb + own_libs <= 1) v += w[3];
      } else {
        v = -INFINITY;
      }
      L->base[own - 1][p] = v;
    }
  }

  // pattern indices (2 bits per ring slot) of a packed neighbourhood, black and white to move
  __device__ __forceinline__ void pattern_idx(uint64_t r8, int& pb, int& pw) const {
    pb = 0;
    pw = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = (int)((r8 >> (8 * k)) & 3);
      pb |= c << (2 * k);
      pw |= ((c == 1 || c == 2) ? 3 - c : c) << (2 * k);
    }
  }

  // gather the packed 3x3 neighbourhood of p (off-board slots = kOff)
  __device__ __forceinline__ uint64_t gather(int p) const {
    int q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) q[k] = ring(p, k);
    uint64_t r8 = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      r8 |= (uint64_t)(q[k] < 0 ? kOff : L->cell[q[k]]) << (8 * k);
    return r8;
  }

  __device__ void compute_base(int p, const float* __restrict__ w,
                               const float* __restrict__ pattern) {
    if (L->cell[p] & 3) {
      L->base[0][p] = -INFINITY;
      L->base[1][p] = -INFINITY;
      return;
    }
    const uint64_t r8 = gather(p);
    int pb, pw;
    pattern_idx(r8, pb, pw);
    base_from(p, r8, pattern ? pattern[pb] : 0.f, pattern ? pattern[pw] : 0.f, w);
  }

  // mark the 3x3 neighbourhoods of changed cells dirty, recompute their bases, clear the flags.
  // The dirty points (typically 10-40 of 361) are compacted into a list with a ballot per lane
  // slot, so the base recompute (8-cell gather, two pattern loads, ~150 instructions of
  // base_from) runs once per lane per 64 dirty points instead of once per lane slot with most
  // lanes masked off; one global round trip per 64 dirty points.
  __device__ void refresh(const float* __restrict__ w, const float* __restrict__ pattern) {
    const int P_ = P();
    uint8_t ch[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      ch[k] = p < P_ ? L->chg[p] : (uint8_t)0;
    }
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      if (!ch[k]) continue;
      const int p = lane + 64 * k;
      int q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = ring(p, j);
      L->dirty[p] = 1;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (q[j] >= 0) L->dirty[q[j]] = 1;
    }
    wave_sync();
    uint8_t d[NPL];
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      d[k] = p < P_ ? L->dirty[p] : (uint8_t)0;
    }
    int n = 0;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      const uint64_t m = __ballot(d[k] != 0);
      const int slot =
          n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (d[k]) {
        L->list[slot] = (int16_t)p;
        L->dirty[p] = 0;
      }
      if (ch[k]) L->chg[p] = 0;
      n += __popcll(m);
    }
    wave_sync();
    for (int r = 0; r < n; r += 64) {
      const int i = r + lane;
      if (i < n) {
        const int p = L->list[i];
        if (L->cell[p] & 3) {
          L->base[0][p] = -INFINITY;
          L->base[1][p] = -INFINITY;
        } else {
          const uint64_t r8 = gather(p);
          float pb = 0.f, pw = 0.f;
          if (pattern) {
            int ib, iw;
            pattern_idx(r8, ib, iw);
            pb = pattern[ib];
            pw = pattern[iw];
          }
          base_from(p, r8, pb, pw, w);
        }
      }
    }
    wave_sync();
  }
};

// Sliced playouts (rag_rollouts_sliced): a game's whole state — its LDS image, the scalars and
// every lane's generator — is parked in HBM between launches of at most `slice` moves, so no
// launch keeps a CU's LDS for a whole ~5 ms playout (conv blocks of the search's networks, which
// need ~150 KB of a CU's LDS, could not start on any CU holding a rollout wave: their launches
// overlapping a resident rollout kernel took 1.1 ms instead of 0.1, profiles/
// mcts_rollout_interference_r5.txt). The moves played are the unsliced kernel's bit for bit.
template <int PM>
struct ParkedGame {
  GameLds<PM> lds;
  int32_t sc[16];    // cur, ko, l1, l2, pb, pw, nm, end, moves, done
  uint32_t rng[64];  // per lane
};

// meta: [cur, ko, last1, last2, passes_b, passes_w, nmoves, end]
// park: null (one launch plays the whole game) or the game's parked state; first: initialise
// from colors / meta (else resume from park); slice: moves this launch may play
template <int SC, int NPL, int PM, int GPB>
__device__ __forceinline__ void rollout_body(
    BlockLds<PM, GPB>& sh, const int8_t* __restrict__ colors, const int32_t* __restrict__ meta,
    int n_pos, int R, int S_rt, float komi, int limit, const float* __restrict__ w,
    const float* __restrict__ pattern, uint32_t seed, int8_t* __restrict__ winner,
    int16_t* __restrict__ length, float* __restrict__ dbg_logits,
    ParkedGame<PM>* __restrict__ park = nullptr, int first = 1, int slice = 1 << 30) {
  const int S = SC > 0 ? SC : S_rt;
  const int P = S * S;
  const int wv = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int game = blockIdx.x * GPB + wv;
  if (game >= n_pos * R) return;  // whole wave exits together
  const int pos = game / R;
  ParkedGame<PM>* pk = park ? park + game : nullptr;
  if (pk && !first && pk->sc[9]) return;  // finished in an earlier slice
  GameLds<PM>& L = sh.g[wv];
  Game<SC, NPL, PM> g{S_rt, &L, lane};
  float wl[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) wl[i] = w[i];
  int px[NPL], py[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int p = lane + 64 * k;
    px[k] = p / S;
    py[k] = p - px[k] * S;
  }
  int cur, ko, l1, l2, pb, pw, nm, moves = 0;
  bool end;
  LaneRng rng;
  if (pk && !first) {
    // resume: the LDS image back in 16-byte pieces, the scalars, this lane's generator
    constexpr int kPieces = (int)(sizeof(GameLds<PM>) / 16);
    static_assert(sizeof(GameLds<PM>) % 16 == 0, "parked LDS image in 16-byte pieces");
    const uint4* src = reinterpret_cast<const uint4*>(&pk->lds);
    uint4* dst = reinterpret_cast<uint4*>(&L);
    for (int i = lane; i < kPieces; i += 64) dst[i] = src[i];
    cur = pk->sc[0];
    ko = pk->sc[1];
    l1 = pk->sc[2];
    l2 = pk->sc[3];
    pb = pk->sc[4];
    pw = pk->sc[5];
    nm = pk->sc[6];
    end = pk->sc[7] != 0;
    moves = pk->sc[8];
    rng.s = pk->rng[lane];
    wave_sync();
  } else {
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P) {
        const int c = colors[(size_t)pos * P + p];
        L.cell[p] = (uint8_t)(c > 0 ? 1 : (c < 0 ? 2 : 0));
        L.chg[p] = 0;
        L.dirty[p] = 0;
      }
    }
    wave_sync();
    g.init_labels();
    g.recount_libs();
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P) {
        g.compute_base(p, wl, pattern);
        L.chg[p] = 0;
      }
    }
    wave_sync();
    const int32_t* m = meta + pos * 8;
    cur = m[0];
    ko = m[1];
    l1 = m[2];
    l2 = m[3];
    pb = m[4];
    pw = m[5];
    nm = m[6];
    end = m[7] != 0;
    rng.s = hash32(seed ^ hash32(game * 0x9E3779B9u + lane * 0x85EBCA6Bu + 1u));
  }

  // logit of lane point k = cached base + last-move terms
  // (branch-free: selects instead of early returns; adding 0 to a finite logit and anything to
  // -inf leave it unchanged, so the values equal the branchy form bit for bit)
  auto full_logit = [&](int k, int own_idx, int l1x, int l1y, int l2x, int l2y) -> float {
    const int p = lane + 64 * k;  // < PM: the base read is in bounds even for p >= P
    float v = (p < P && p != ko) ? L.base[own_idx][p] : -INFINITY;
    const int d1x = abs(px[k] - l1x), d1y = abs(py[k] - l1y);
    v += (d1x <= 1 && d1y <= 1) ? wl[0] : (d1x + d1y <= 2 ? wl[4] : 0.f);
    v += (abs(px[k] - l2x) <= 1 && abs(py[k] - l2y) <= 1) ? wl[5] : 0.f;
    return v;
  };

  if (dbg_logits) {  // debug: logits of the initial position only
    const int l1x = l1 >= 0 ? l1 / S : -100, l1y = l1 >= 0 ? l1 % S : -100;
    const int l2x = l2 >= 0 ? l2 / S : -100, l2y = l2 >= 0 ? l2 % S : -100;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P)
        dbg_logits[(size_t)game * P + p] = full_logit(k, cur > 0 ? 0 : 1, l1x, l1y, l2x, l2y);
    }
    return;
  }

  const int stop = moves + slice < limit ? moves + slice : limit;
  while (!end && moves < stop) {
    const int own = cur > 0 ? 1 : 2;
    const int l1x = l1 >= 0 ? l1 / S : -100, l1y = l1 >= 0 ? l1 - (l1 / S) * S : -100;
    const int l2x = l2 >= 0 ? l2 / S : -100, l2y = l2 >= 0 ? l2 - (l2 / S) * S : -100;
    float key = -INFINITY;
    int idx = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const float lg = full_logit(k, own - 1, l1x, l1y, l2x, l2y);
      // the lane's generator advances only on candidates (as the branchy form did)
      const bool cand = lg != -INFINITY;
      const uint32_t s1 = rng.s * 1664525u + 1013904223u;
      rng.s = cand ? s1 : rng.s;
      const float u = ((hash32(s1) >> 8) + 0.5f) * (1.0f / 16777216.0f);
      const float kk = cand ? lg - __logf(-__logf(u)) : -INFINITY;
      const bool better = kk > key;
      key = better ? kk : key;
      idx = better ? lane + 64 * k : idx;
    }
    wave_argmax(key, idx);
    const int mv = key == -INFINITY ? -1 : idx;  // -1 = pass
    ko = -1;
    if (mv >= 0) {
      // wave-uniform bookkeeping (every lane reads the same LDS words)
      int nq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) nq[i] = g.orth(mv, i);
      uint8_t cq4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) cq4[i] = nq[i] >= 0 ? L.cell[nq[i]] : (uint8_t)0;
      int lq4[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) lq4[i] = (cq4[i] & 3) ? (int)L.lab[nq[i]] : -1;
      // one slot per neighbour (-1 = none): membership tests need no de-duplication, and fixed
      // slots keep the arrays in registers (a running count index would put them in scratch)
      int cap_l[4], own_l[4];
      int cap_pt = -1;
      bool any_own = false;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = cq4[i] & 3;
        own_l[i] = c == own ? lq4[i] : -1;
        const bool cap = c && c != own && (cq4[i] >> 2) == 1;
        cap_l[i] = cap ? lq4[i] : -1;
        if (cap) cap_pt = nq[i];  // only used when exactly one stone is captured
        any_own |= c == own;
      }
      wave_sync();
      int removed = 0;
      uint8_t cc[NPL];
      int lc[NPL];
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int p = lane + 64 * k;
        cc[k] = p < P ? (uint8_t)(L.cell[p] & 3) : (uint8_t)0;
        lc[k] = cc[k] ? (int)L.lab[p] : -1;
      }
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int c = cc[k];
        if (!c) continue;
        const int p = lane + 64 * k;
        const int l = lc[k];
        if (c != own) {
          bool hit = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) hit |= cap_l[j] == l;
          if (hit) {
            L.cell[p] = 0;
            L.lab[p] = -1;
            L.chg[p] = 1;
            ++removed;
          }
        } else {
          bool hit = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) hit |= own_l[j] == l;
          if (hit) L.lab[p] = (int16_t)mv;
        }
      }
      if (lane == 0) {
        L.cell[mv] = (uint8_t)own;
        L.lab[mv] = (int16_t)mv;
        L.chg[mv] = 1;
      }
      wave_sync();
      g.recount_libs();
      removed = wave_sum_i(removed);
      // ko: one stone captured by a lone stone that is left with a single liberty
      if (removed == 1 && !any_own && L.lib[mv] == 1) ko = cap_pt;
      g.refresh(wl, pattern);
    } else {
      if (cur == 1) ++pb;
      else ++pw;
    }
    l2 = l1;
    l1 = mv;
    ++nm;
    cur = -cur;
    if (nm > 1 && l1 == -1 && l2 == -1 && cur == -1) end = true;
    ++moves;
  }
  if (pk && !end && moves < limit) {  // park the game until the next slice
    constexpr int kPieces = (int)(sizeof(GameLds<PM>) / 16);
    wave_sync();
    const uint4* src = reinterpret_cast<const uint4*>(&L);
    uint4* dst = reinterpret_cast<uint4*>(&pk->lds);
    for (int i = lane; i < kPieces; i += 64) dst[i] = src[i];
    pk->rng[lane] = rng.s;
    if (lane == 0) {
      const int32_t v[10] = {cur, ko, l1, l2, pb, pw, nm, (int32_t)end, moves, 0};
#pragma unroll
      for (int i = 0; i < 10; ++i) pk->sc[i] = v[i];
    }
    return;
  }
  if (pk && lane == 0) pk->sc[9] = 1;
  // area score: stones + single-point eyeish empties
  int sb = 0, sw = 0;
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int p = lane + 64 * k;
    if (p >= P) continue;
    const int c = L.cell[p] & 3;
    if (c == 1) {
      ++sb;
    } else if (c == 2) {
      ++sw;
    } else {
      bool allb = true, allw = true;
      for (int i = 0; i < 4; ++i) {
        const int q = g.orth(p, i);
        if (q < 0) continue;
        const int cq = L.cell[q] & 3;
        allb &= cq == 1;
        allw &= cq == 2;
      }
      if (allb) ++sb;
      else if (allw) ++sw;
    }
  }
  sb = wave_sum_i(sb);
  sw = wave_sum_i(sw);
  if (lane == 0) {
    const float black = (float)(sb - pb), white = (float)sw + komi - (float)pw;
    winner[game] = black > white ? 1 : (white > black ? -1 : 0);
    if (length) length[game] = (int16_t)moves;
  }
}

#define RAG_RO_ARGS                                                                              \
  const int8_t *__restrict__ colors, const int32_t *__restrict__ meta, int n_pos, int R, int S_rt, \
      float komi, int limit, const float *__restrict__ w, const float *__restrict__ pattern,       \
      uint32_t seed, int8_t *__restrict__ winner, int16_t *__restrict__ length,                    \
      float *__restrict__ dbg_logits, void *__restrict__ park, int first, int slice
#define RAG_RO_FWD                                                                              \
  colors, meta, n_pos, R, S_rt, komi, limit, w, pattern, seed, winner, length, dbg_logits,        \
      reinterpret_cast<ParkedGame<PM>*>(park), first, slice

// The same playout body at two register budgets: the compiler's choice (146 VGPRs for 19x19,
// 3 waves per SIMD) and a cap at 128 VGPRs (4 waves per SIMD, a few spills outside the move
// loop). RAG_ROLLOUT_WPE=3|4 picks one (default measured: see docs/KERNELS.md).
template <int SC, int NPL, int PM, int GPB>
__global__ void __launch_bounds__(64 * GPB) rollout_kernel(RAG_RO_ARGS) {
  __shared__ BlockLds<PM, GPB> sh;
  rollout_body<SC, NPL, PM, GPB>(sh, RAG_RO_FWD);
}

template <int SC, int NPL, int PM, int GPB>
__global__ void __launch_bounds__(64 * GPB) __attribute__((amdgpu_waves_per_eu(4)))
rollout_kernel_w4(RAG_RO_ARGS) {
  __shared__ BlockLds<PM, GPB> sh;
  rollout_body<SC, NPL, PM, GPB>(sh, RAG_RO_FWD);
}

int rollout_wpe() {
  static const int v = [] {
    const char* e = getenv("RAG_ROLLOUT_WPE");
    return e ? atoi(e) : 4;
  }();
  return v;
}

int rollout_gpb() {
  static int v = [] {
    const char* e = getenv("RAG_ROLLOUT_GPB");
    return e && atoi(e) == 4 ? 4 : 1;
  }();
  return v;
}

template <int SC, int NPL, int PM, int GPB>
void launch_gpb(hipStream_t st, const int8_t* c, const int32_t* meta, int n_pos, int R, int S,
                float komi, int limit, const float* w, const float* pattern, unsigned seed,
                void* winner, void* length, float* dbg, void* park, int slice) {
  const dim3 grid((n_pos * R + GPB - 1) / GPB);
  // unsliced: one launch; sliced: ceil(limit / slice) launches on the same stream, the first
  // initialising from the inputs, every later one resuming the parked games
  const int nl = park ? (limit + slice - 1) / slice : 1;
  for (int l = 0; l < nl; ++l) {
    const int first = l == 0, sl = park ? slice : (1 << 30);
    if (rollout_wpe() == 4)
      rollout_kernel_w4<SC, NPL, PM, GPB><<<grid, 64 * GPB, 0, st>>>(
          c, meta, n_pos, R, S, komi, limit, w, pattern, seed, (int8_t*)winner,
          (int16_t*)length, dbg, park, first, sl);
    else
      rollout_kernel<SC, NPL, PM, GPB><<<grid, 64 * GPB, 0, st>>>(
          c, meta, n_pos, R, S, komi, limit, w, pattern, seed, (int8_t*)winner,
          (int16_t*)length, dbg, park, first, sl);
  }
}

template <int SC, int NPL, int PM>
void launch(hipStream_t st, const int8_t* c, const int32_t* meta, int n_pos, int R, int S,
            float komi, int limit, const float* w, const float* pattern, unsigned seed,
            void* winner, void* length, float* dbg, void* park, int slice) {
  if (rollout_gpb() == 4)
    launch_gpb<SC, NPL, PM, 4>(st, c, meta, n_pos, R, S, komi, limit, w, pattern, seed, winner,
                               length, dbg, park, slice);
  else
    launch_gpb<SC, NPL, PM, 1>(st, c, meta, n_pos, R, S, komi, limit, w, pattern, seed, winner,
                               length, dbg, park, slice);
}

}  // namespace

// colors [n_pos][S*S] int8, meta [n_pos][8] int32, weights [7], pattern [65536] (or null);
// winner [n_pos*R] int8 (+1 black, -1 white, 0 draw), length [n_pos*R] int16 (optional).
// dbg_logits (optional, [n_pos*R][S*S]) switches to "initial logits only" mode.
// park: null (one launch per playout) or rag_rollout_park_bytes(S) x n_pos x R bytes of device
// memory (sliced: launches of at most `slice` moves, identical results)
RAG_API long rag_rollout_park_bytes(int S) {
  if (S == 19) return (long)sizeof(ParkedGame<384>);
  if (S == 13) return (long)sizeof(ParkedGame<192>);
  if (S == 9) return (long)sizeof(ParkedGame<128>);
  return S * S <= 384 ? (long)sizeof(ParkedGame<384>) : (long)sizeof(ParkedGame<640>);
}

RAG_API int rag_rollouts(const void* colors, const int32_t* meta, int n_pos, int R, int S,
                         float komi, int limit, const float* w, const float* pattern,
                         unsigned seed, void* winner, void* length, float* dbg_logits,
                         hipStream_t stream, void* park, int slice) {
  if (S < 2 || S > 25 || n_pos <= 0 || R <= 0) return -1;
  if (park && (slice <= 0 || dbg_logits)) return -1;
  const int8_t* c = (const int8_t*)colors;
#define RAG_RO(SC, NPL, PM)                                                                     \
  launch<SC, NPL, PM>(stream, c, meta, n_pos, R, S, komi, limit, w, pattern, seed, winner, length, \
                      dbg_logits, park, slice)
  if (S == 19) RAG_RO(19, 6, 384);
  else if (S == 13) RAG_RO(13, 3, 192);
  else if (S == 9) RAG_RO(9, 2, 128);
  else if (S * S <= 384) RAG_RO(0, 6, 384);
  else RAG_RO(0, 10, 640);
#undef RAG_RO
  return (int)hipGetLastError();
}

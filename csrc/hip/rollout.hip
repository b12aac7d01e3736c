// Fast-rollout playouts on the GPU: one wavefront plays one game to the end.
//
// The policy is the same linear softmax as the native one (csrc/mcts/rollout.hpp): per candidate
// move, 7 binary features + a 3x3 pattern weight; candidates are empty points that are not an
// own single-point eye and are legal (no suicide, not the ko point). Sampling uses the Gumbel-max
// trick (argmax of logit + Gumbel noise == a draw from the softmax over the legal candidates,
// i.e. the same distribution the CPU rejection sampler draws from), so a move costs one wave-wide
// max reduction.
//
// Board state lives in LDS, one slice per wave: colour per point, a group label per stone (the
// index of a representative stone) and a liberty count per label. Each lane owns the points
// p = lane + 64*k. A move: place the stone, remove captured groups (opponent neighbours whose
// count was 1), relabel the merged own groups to the new stone, then recount every liberty from
// scratch (each empty point adds 1 to each distinct neighbouring label with LDS atomics).
// Rules match the native engine in light mode: simple ko (reference rule Q15), no superko, end
// of game after two passes with WHITE to move (Q3), area score with single-point eyeish
// empties and komi, minus passes (Q12).
#include "common.h"

using namespace rag;

namespace {

constexpr int kWaves = 4;  // games per 256-thread block

struct Shared {
  int8_t col[kWaves][640];
  int16_t lab[kWaves][640];
  int lib[kWaves][640];
};

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

// wave-wide argmax of (key, idx); ties -> smaller idx
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

template <int NPL>
struct Game {
  int S, P;
  int8_t* col;
  int16_t* lab;
  int* lib;
  int lane;

  __device__ int nb(int p, int k) const {  // orthogonal neighbour k (engine order) or -1
    const int x = p / S, y = p - (p / S) * S;
    switch (k) {
      case 0: return x > 0 ? p - S : -1;
      case 1: return x < S - 1 ? p + S : -1;
      case 2: return y > 0 ? p - 1 : -1;
      default: return y < S - 1 ? p + 1 : -1;
    }
  }

  __device__ void recount_libs() {
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P) lib[p] = 0;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p >= P || col[p] != 0) continue;
      int seen[4];
      int ns = 0;
      for (int i = 0; i < 4; ++i) {
        const int q = nb(p, i);
        if (q < 0 || col[q] == 0) continue;
        const int l = lab[q];
        bool dup = false;
        for (int j = 0; j < ns; ++j) dup |= seen[j] == l;
        if (!dup) {
          seen[ns++] = l;
          atomicAdd(&lib[l], 1);
        }
      }
    }
    wave_sync();
  }

  __device__ void init_labels() {
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P) lab[p] = col[p] ? (int16_t)p : (int16_t)-1;
    }
    wave_sync();
    // min-label propagation with pointer jumping until stable
    for (int it = 0; it < 4 * 640; ++it) {
      int changed = 0;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int p = lane + 64 * k;
        if (p >= P || col[p] == 0) continue;
        int m = lab[lab[p]];
        for (int i = 0; i < 4; ++i) {
          const int q = nb(p, i);
          if (q >= 0 && col[q] == col[p]) m = min(m, (int)lab[q]);
        }
        if (m < lab[p]) {
          lab[p] = (int16_t)m;
          changed = 1;
        }
      }
      wave_sync();
      if (!__any(changed)) break;
    }
  }
};

// logits of all candidates for player c (-inf for non-candidates); returns per-lane keys
template <int NPL>
__device__ __forceinline__ float cand_logit(const Game<NPL>& g, int p, int c, int ko, int l1,
                                            int l2, const float* __restrict__ w,
                                            const float* __restrict__ pattern) {
  const int S = g.S;
  if (g.col[p] != 0 || p == ko) return -INFINITY;
  const int x = p / S, y = p - (p / S) * S;
  int nnb = 0, own_nb = 0;
  int empty_nb = 0, own_libs = 0;
  bool capture = false, own_atari = false, own_multi = false;
  for (int i = 0; i < 4; ++i) {
    const int q = g.nb(p, i);
    if (q < 0) continue;
    ++nnb;
    const int cq = g.col[q];
    if (cq == 0) {
      ++empty_nb;
    } else if (cq == c) {
      ++own_nb;
      const int lc = g.lib[g.lab[q]];
      if (lc == 1) own_atari = true;
      else own_multi = true;
      own_libs += lc - 1;
    } else if (g.lib[g.lab[q]] == 1) {
      capture = true;
    }
  }
  // own single-point eye (all orthogonal neighbours own; <=1 opponent diagonal in the centre,
  // none on the edge)
  if (own_nb == nnb) {
    int bad = 0;
    const int dx[4] = {-1, 1, 1, -1}, dy[4] = {-1, 1, -1, 1};
    for (int i = 0; i < 4; ++i) {
      const int ax = x + dx[i], ay = y + dy[i];
      if (ax < 0 || ay < 0 || ax >= S || ay >= S) continue;
      bad += g.col[ax * S + ay] == -c;
    }
    if (nnb < 4 ? bad == 0 : bad <= 1) return -INFINITY;
  }
  // suicide
  if (empty_nb == 0 && !own_multi && !capture) return -INFINITY;
  float s = 0.f;
  if (l1 >= 0) {
    const int d1x = abs(x - l1 / S), d1y = abs(y - l1 % S);
    if (d1x <= 1 && d1y <= 1) s += w[0];
    else if (d1x + d1y <= 2) s += w[4];
  }
  if (l2 >= 0 && abs(x - l2 / S) <= 1 && abs(y - l2 % S) <= 1) s += w[5];
  if (x == 0 || y == 0 || x == S - 1 || y == S - 1) s += w[6];
  if (capture) s += w[2];
  if (own_atari && (empty_nb >= 2 || capture)) s += w[1];
  if (!capture && empty_nb + own_libs <= 1) s += w[3];
  const int rdx[8] = {0, 1, 1, 1, 0, -1, -1, -1}, rdy[8] = {1, 1, 0, -1, -1, -1, 0, 1};
  int pidx = 0;
  for (int k = 0; k < 8; ++k) {
    const int ax = x + rdx[k], ay = y + rdy[k];
    int code = 3;
    if (ax >= 0 && ay >= 0 && ax < S && ay < S) {
      const int cq = g.col[ax * S + ay];
      code = cq == 0 ? 0 : (cq == c ? 1 : 2);
    }
    pidx |= code << (2 * k);
  }
  return pattern ? s + pattern[pidx] : s;
}

// meta: [cur, ko, last1, last2, passes_b, passes_w, nmoves, end]
template <int NPL>
__global__ void __launch_bounds__(256)
rollout_kernel(const int8_t* __restrict__ colors, const int32_t* __restrict__ meta, int n_pos,
               int R, int S, float komi, int limit, const float* __restrict__ w,
               const float* __restrict__ pattern, uint32_t seed, int8_t* __restrict__ winner,
               int16_t* __restrict__ length, float* __restrict__ dbg_logits) {
  __shared__ Shared sh;
  const int wv = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int game = blockIdx.x * kWaves + wv;
  if (game >= n_pos * R) return;  // whole wave exits together
  const int pos = game / R;
  Game<NPL> g;
  g.S = S;
  g.P = S * S;
  g.col = sh.col[wv];
  g.lab = sh.lab[wv];
  g.lib = sh.lib[wv];
  g.lane = lane;
  const int P = g.P;
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int p = lane + 64 * k;
    if (p < P) g.col[p] = colors[(size_t)pos * P + p];
  }
  wave_sync();
  g.init_labels();
  g.recount_libs();
  const int32_t* m = meta + pos * 8;
  int cur = m[0], ko = m[1], l1 = m[2], l2 = m[3], pb = m[4], pw = m[5], nm = m[6];
  bool end = m[7] != 0;
  LaneRng rng{hash32(seed ^ hash32(game * 0x9E3779B9u + lane * 0x85EBCA6Bu + 1u))};

  if (dbg_logits) {  // debug: logits of the initial position only
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P) dbg_logits[(size_t)game * P + p] = cand_logit(g, p, cur, ko, l1, l2, w, pattern);
    }
    return;
  }

  int moves = 0;
  while (!end && moves < limit) {
    float key = -INFINITY;
    int idx = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < NPL; ++k) {
      const int p = lane + 64 * k;
      if (p >= P) continue;
      const float lg = cand_logit(g, p, cur, ko, l1, l2, w, pattern);
      if (lg == -INFINITY) continue;
      const float u = rng.uniform();
      const float kk = lg - __logf(-__logf(u));
      if (kk > key) {
        key = kk;
        idx = p;
      }
    }
    wave_argmax(key, idx);
    const int mv = key == -INFINITY ? -1 : idx;  // -1 = pass
    ko = -1;
    if (mv >= 0) {
      // wave-uniform bookkeeping from LDS (all lanes read the same words)
      int cap_l[4], own_l[4];
      int ncap = 0, nown = 0, cap_pt = -1;
      for (int i = 0; i < 4; ++i) {
        const int q = g.nb(mv, i);
        if (q < 0 || g.col[q] == 0) continue;
        const int l = g.lab[q];
        if (g.col[q] == cur) {
          bool dup = false;
          for (int j = 0; j < nown; ++j) dup |= own_l[j] == l;
          if (!dup) own_l[nown++] = l;
        } else if (g.lib[l] == 1) {
          bool dup = false;
          for (int j = 0; j < ncap; ++j) dup |= cap_l[j] == l;
          if (!dup) {
            cap_l[ncap++] = l;
            cap_pt = q;
          }
        }
      }
      wave_sync();
      int removed = 0;
#pragma unroll
      for (int k = 0; k < NPL; ++k) {
        const int p = lane + 64 * k;
        if (p >= P) continue;
        const int8_t cp = g.col[p];
        if (cp == 0) continue;
        const int l = g.lab[p];
        if (cp == -cur) {
          bool hit = false;
          for (int j = 0; j < ncap; ++j) hit |= cap_l[j] == l;
          if (hit) {
            g.col[p] = 0;
            g.lab[p] = -1;
            ++removed;
          }
        } else {
          bool hit = false;
          for (int j = 0; j < nown; ++j) hit |= own_l[j] == l;
          if (hit) g.lab[p] = (int16_t)mv;
        }
      }
      if (lane == 0) {
        g.col[mv] = (int8_t)cur;
        g.lab[mv] = (int16_t)mv;
      }
      wave_sync();
      g.recount_libs();
      removed = wave_sum_i(removed);
      // ko: one stone captured by a lone stone that is left with a single liberty
      if (removed == 1 && nown == 0 && g.lib[mv] == 1) ko = cap_pt;
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
  // area score: stones + single-point eyeish empties
  int sb = 0, sw = 0;
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int p = lane + 64 * k;
    if (p >= P) continue;
    const int cp = g.col[p];
    if (cp == 1) {
      ++sb;
    } else if (cp == -1) {
      ++sw;
    } else {
      bool allb = true, allw = true;
      for (int i = 0; i < 4; ++i) {
        const int q = g.nb(p, i);
        if (q < 0) continue;
        allb &= g.col[q] == 1;
        allw &= g.col[q] == -1;
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

}  // namespace

// colors [n_pos][S*S] int8, meta [n_pos][8] int32, weights [7], pattern [65536];
// winner [n_pos*R] int8 (+1 black, -1 white, 0 draw), length [n_pos*R] int16 (optional).
// dbg_logits (optional, [n_pos*R][S*S]) switches to "initial logits only" mode.
RAG_API int rag_rollouts(const void* colors, const int32_t* meta, int n_pos, int R, int S,
                         float komi, int limit, const float* w, const float* pattern,
                         unsigned seed, void* winner, void* length, float* dbg_logits,
                         hipStream_t stream) {
  if (S < 2 || S > 25 || n_pos <= 0 || R <= 0) return -1;
  const int games = n_pos * R;
  dim3 grid((games + kWaves - 1) / kWaves);
  const int8_t* c = (const int8_t*)colors;
  if (S * S <= 384)
    rollout_kernel<6><<<grid, 256, 0, stream>>>(c, meta, n_pos, R, S, komi, limit, w, pattern,
                                                seed, (int8_t*)winner, (int16_t*)length,
                                                dbg_logits);
  else
    rollout_kernel<10><<<grid, 256, 0, stream>>>(c, meta, n_pos, R, S, komi, limit, w, pattern,
                                                 seed, (int8_t*)winner, (int16_t*)length,
                                                 dbg_logits);
  return (int)hipGetLastError();
}

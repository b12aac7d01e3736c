// Ladder reading on the GPU: the `ladder_capture` and `ladder_escape`
// feature planes, bit-exact with the native engine's Board::is_ladder_capture / is_ladder_escape
// (csrc/engine/go_engine.cpp, itself pinned to the reference go.py:329-463 by
// tests/test_ladders.py).
//
// Two launches:
//   * ladder_prep_kernel — one wavefront per position: group labels (min-label propagation),
//     liberty counts, and the candidate moves: an empty legal point p is a capture candidate if a
//     neighbouring group of the opponent has exactly 2 liberties and an escape candidate if a
//     neighbouring own group has exactly 1 (every other point reads `false` in the reference
//     search without moving a stone). Candidates are appended to a task queue; both planes of the
//     position are zeroed.
//   * ladder_search_kernel — a persistent grid of single-wave workgroups pulling tasks from the
//     queue until it is empty (every wave reaches that exit). One wavefront reads one ladder: the
//     reference's mutual recursion as an explicit DFS over an LDS frame stack (depth <= 80 =
//     remaining_attempts). The board lives in LDS (colour + group label per point); a move is
//     applied in place and undone from the frame (captured groups and relabelled merged groups
//     are kept as 361-bit stone sets), so no board is ever copied. Every board query is one
//     wave-wide pass over the points (6 per lane) reduced with ballots: liberty counts of the
//     (at most 4) groups around a move, the prey's liberty set, and the escape set (prey
//     liberties plus the liberties of hunter groups in atari that touch the prey).
// The search is a pure boolean function of (position, move, prey, remaining), so candidate and
// option order never changes a result; options are visited in increasing point order, like the
// native search.
// Positions that enforce positional superko keep the native search (host), since their
// legality depends on the game history.
#include "common.h"

using namespace rag;

namespace {

constexpr int kPMAX = 384;
constexpr int kNW = 6;       // 64-bit words per point set
constexpr int kNPL = 6;      // points per lane
constexpr int kDepth = 81;   // frames: remaining 80 .. 1
constexpr int kMaxSteps = 1 << 21;  // safety bound on DFS steps per task (never reached in tests)

enum { K_CAP = 0, K_ESC = 1 };

// One call of the recursion whose move is (or is about to be) on the board. Neighbour data is
// slot-indexed (slot i = the i-th orthogonal neighbour of the move), so every index into the
// small per-move arrays is a compile-time constant in registers and an LDS index here.
struct Frame {
  unsigned long long iter[kNW];      // options still to visit
  unsigned long long gb[4][kNW];     // stones of the group at neighbour slot i (captured/merged)
  int16_t gl[4];                     // label of that group before the move
  int16_t cand[4];                   // candidate prey (a stone) per slot, or cand[0] = given prey
  int16_t a, pr, ko_before;
  int8_t kind, rem, ci, capm, mrgm, candm, mover;
};

struct SearchLds {
  int8_t col[kPMAX];
  int16_t lab[kPMAX];  // group label (a stone of the group), -1 on empty points
  int lib[kPMAX];      // per-label liberty counters (escape sets)
  uint8_t adj[kPMAX];  // per-label flag: hunter group touching the prey
  Frame fr[kDepth];
};

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ unsigned long long ballot(bool b) {
  return (unsigned long long)__ballot(b);
}

__device__ __forceinline__ int nbr(int p, int k, int S) {
  const int x = p / S, y = p - (p / S) * S;
  switch (k) {  // native order: (x-1,y) (x+1,y) (x,y-1) (x,y+1)
    case 0: return x > 0 ? p - S : -1;
    case 1: return x < S - 1 ? p + S : -1;
    case 2: return y > 0 ? p - 1 : -1;
    default: return y < S - 1 ? p + 1 : -1;
  }
}

__device__ __forceinline__ bool bit(const unsigned long long* s, int p) {
  return (s[p >> 6] >> (p & 63)) & 1ull;
}

// ---------------------------------------------------------------------------------- prep
__global__ void __launch_bounds__(64)
ladder_prep_kernel(const int8_t* __restrict__ colors, const int32_t* __restrict__ meta, int n_pos,
                   int S, int16_t* __restrict__ labels, int* __restrict__ queue,
                   int* __restrict__ tasks, uint8_t* __restrict__ out) {
  __shared__ int8_t col[kPMAX];
  __shared__ int16_t lab[kPMAX];
  __shared__ int lib[kPMAX];
  const int pos = blockIdx.x;
  const int lane = threadIdx.x;
  const int P = S * S;
  const int me = meta[pos * 4 + 0];
  const int ko = meta[pos * 4 + 1];
#pragma unroll
  for (int k = 0; k < kNPL; ++k) {
    const int p = lane + 64 * k;
    if (p < P) {
      col[p] = colors[(size_t)pos * P + p];
      lab[p] = col[p] ? (int16_t)p : (int16_t)-1;
      lib[p] = 0;
      out[((size_t)pos * 2 + 0) * P + p] = 0;
      out[((size_t)pos * 2 + 1) * P + p] = 0;
    }
  }
  wsync();
  for (int it = 0; it < 2 * kPMAX; ++it) {
    int changed = 0;
#pragma unroll
    for (int k = 0; k < kNPL; ++k) {
      const int p = lane + 64 * k;
      if (p >= P || col[p] == 0) continue;
      int m = lab[lab[p]];
      for (int i = 0; i < 4; ++i) {
        const int q = nbr(p, i, S);
        if (q >= 0 && col[q] == col[p]) m = min(m, (int)lab[q]);
      }
      if (m < lab[p]) {
        lab[p] = (int16_t)m;
        changed = 1;
      }
    }
    wsync();
    if (!__any(changed)) break;
  }
#pragma unroll
  for (int k = 0; k < kNPL; ++k) {
    const int p = lane + 64 * k;
    if (p >= P || col[p] != 0) continue;
    int seen[4], ns = 0;
    for (int i = 0; i < 4; ++i) {
      const int q = nbr(p, i, S);
      if (q < 0 || col[q] == 0) continue;
      const int l = lab[q];
      bool dup = false;
      for (int j = 0; j < ns; ++j) dup |= seen[j] == l;
      if (dup) continue;
      seen[ns++] = l;
      atomicAdd(&lib[l], 1);
    }
  }
  wsync();
#pragma unroll
  for (int k = 0; k < kNPL; ++k) {
    const int p = lane + 64 * k;
    if (p >= P) continue;
    labels[(size_t)pos * P + p] = lab[p];
    if (col[p] != 0 || p == ko) continue;
    bool empty_nb = false, own_multi = false, cap = false, cand_c = false, cand_e = false;
    for (int i = 0; i < 4; ++i) {
      const int q = nbr(p, i, S);
      if (q < 0) continue;
      if (col[q] == 0) {
        empty_nb = true;
        continue;
      }
      const int l = lib[lab[q]];
      if (col[q] == me) {
        own_multi |= l > 1;
        cand_e |= l == 1;
      } else {
        cap |= l == 1;
        cand_c |= l == 2;
      }
    }
    if (!(empty_nb || own_multi || cap)) continue;  // suicide: illegal, both planes false
    if (cand_c) tasks[atomicAdd(&queue[0], 1)] = (pos << 10) | (p << 1) | K_CAP;
    if (cand_e) tasks[atomicAdd(&queue[0], 1)] = (pos << 10) | (p << 1) | K_ESC;
  }
}

// ---------------------------------------------------------------------------------- search
struct Wave {
  SearchLds* L;
  int S, P, lane;
  int me, ko;  // player to move, ko point (wave-uniform)
  int nb[kNPL][4];

  // Surroundings of move a (all wave-uniform, slot i = neighbour i in native order):
  // q[i] point (-1 off board), c[i] colour, l[i] label; ownf / oppf: slot holds the first
  // occurrence of an own / opponent group; lc[i] the liberty count of slot i's group.
  struct Around {
    int q[4], c[4], l[4], lc[4];
    int ownf, oppf, empty;
  };

  __device__ __forceinline__ void around(int a, Around& r) const {
    r.ownf = r.oppf = r.empty = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = nbr(a, i, S);
      r.q[i] = q;
      r.c[i] = q >= 0 ? (int)L->col[q] : 2;
      r.l[i] = q >= 0 ? (int)L->lab[q] : -1;
      r.empty += r.c[i] == 0;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool dup = false;
#pragma unroll
      for (int j = 0; j < i; ++j) dup |= r.l[j] == r.l[i];
      const bool stone = r.c[i] == 1 || r.c[i] == -1;
      if (stone && !dup) {
        if (r.c[i] == me) r.ownf |= 1 << i;
        else r.oppf |= 1 << i;
      }
    }
    int cnt[4] = {0, 0, 0, 0};
    if (r.ownf | r.oppf) {
#pragma unroll
      for (int k = 0; k < kNPL; ++k) {
        const int p = lane + 64 * k;
        const bool emp = p < P && L->lab[p] < 0;
        int nl[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = nb[k][i];
          nl[i] = (emp && q >= 0) ? (int)L->lab[q] : -2;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int lj = ((r.ownf | r.oppf) >> j) & 1 ? r.l[j] : -3;
          const bool hit = nl[0] == lj || nl[1] == lj || nl[2] == lj || nl[3] == lj;
          cnt[j] += __popcll(ballot(hit));
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) r.lc[j] = uni(cnt[j]);
  }

  __device__ __forceinline__ bool legal(int a, const Around& r) const {
    if (L->col[a] != 0 || a == ko) return false;
    if (r.empty > 0) return true;
    bool ok = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ok |= ((r.ownf >> i) & 1) && r.lc[i] > 1;  // own group keeps a liberty
      ok |= ((r.oppf >> i) & 1) && r.lc[i] == 1;  // captures
    }
    return ok;
  }

  // stones with label l -> set (ballot), written by lane 0
  __device__ __forceinline__ void stones(int l, unsigned long long* s) const {
#pragma unroll
    for (int k = 0; k < kNPL; ++k) {
      const int p = lane + 64 * k;
      const unsigned long long b = ballot(p < P && L->lab[p] == l);
      if (lane == 0) s[k] = b;
    }
  }

  // Play `a` for the player to move (legal; `r` describes its surroundings), recording the undo
  // information in frame f. Captured opponent groups (whose only liberty was a) are removed;
  // the new stone joins the first own neighbour group's label and the other own neighbour
  // groups are relabelled to it. Ko: the native rule (the first captured group in neighbour
  // order is a single stone, and the new stone has neither an own nor an empty neighbour).
  __device__ __forceinline__ void play(int a, const Around& r, Frame& f) {
    const int c = me;
    int capm = 0, mrgm = 0, first_own = -1, first_cap = -1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (((r.oppf >> i) & 1) && r.lc[i] == 1) {
        capm |= 1 << i;
        if (first_cap < 0) first_cap = i;
      }
      if ((r.ownf >> i) & 1) {
        if (first_own < 0) first_own = i;
        else mrgm |= 1 << i;
      }
    }
    int tgt = a;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i == first_own) tgt = r.l[i];
    if (lane == 0) {
      f.a = (int16_t)a;
      f.ko_before = (int16_t)ko;
      f.mover = (int8_t)c;
      f.capm = (int8_t)capm;
      f.mrgm = (int8_t)mrgm;
#pragma unroll
      for (int i = 0; i < 4; ++i) f.gl[i] = (int16_t)r.l[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (((capm | mrgm) >> i) & 1) stones(r.l[i], f.gb[i]);
    wsync();  // the stone sets are in LDS
    int first_size = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i == first_cap)
#pragma unroll
        for (int w = 0; w < kNW; ++w) first_size += __popcll(f.gb[i][w]);
#pragma unroll
    for (int k = 0; k < kNPL; ++k) {
      const int p = lane + 64 * k;
      if (p >= P) continue;
      const int l = L->lab[p];
      if (l < 0) continue;
      bool cap = false, mrg = false;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        cap |= ((capm >> i) & 1) && l == r.l[i];
        mrg |= ((mrgm >> i) & 1) && l == r.l[i];
      }
      if (cap) {
        L->col[p] = 0;
        L->lab[p] = -1;
      } else if (mrg) {
        L->lab[p] = (int16_t)tgt;
      }
    }
    wsync();
    if (lane == 0) {
      L->col[a] = (int8_t)c;
      L->lab[a] = (int16_t)tgt;
    }
    wsync();
    int kop = -1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i == first_cap) kop = r.q[i];
    ko = (first_own < 0 && r.empty == 0 && first_cap >= 0 && first_size == 1) ? kop : -1;
    me = -c;
  }

  __device__ __forceinline__ void undo(const Frame& f) {
    const int c = uni(f.mover);
    const int a = uni(f.a);
    const int capm = uni(f.capm), mrgm = uni(f.mrgm);
    int gl[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) gl[i] = uni(f.gl[i]);
    if (capm | mrgm) {
#pragma unroll
      for (int k = 0; k < kNPL; ++k) {
        const int p = lane + 64 * k;
        if (p >= P) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (!(((capm | mrgm) >> i) & 1) || !bit(f.gb[i], p)) continue;
          if ((capm >> i) & 1) L->col[p] = (int8_t)(-c);
          L->lab[p] = (int16_t)gl[i];
        }
      }
      wsync();
    }
    if (lane == 0) {
      L->col[a] = 0;
      L->lab[a] = -1;
    }
    wsync();
    ko = uni(f.ko_before);
    me = c;
  }

  // liberty set of the group of stone pr (for an empty pr: its empty neighbours)
  __device__ __forceinline__ int libset(int pr, unsigned long long* s) const {
    const int l = L->lab[pr];
    int n = 0;
#pragma unroll
    for (int k = 0; k < kNPL; ++k) {
      const int p = lane + 64 * k;
      bool hit = false;
      if (p < P && L->lab[p] < 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = nb[k][i];
          hit |= l >= 0 ? (q >= 0 && L->lab[q] == l) : q == pr;
        }
      }
      const unsigned long long b = ballot(hit);
      n += __popcll(b);
      s[k] = b;  // private copy in every lane (the ballot is uniform)
    }
    return n;
  }

  // Escape options after the hunter's move (prey to move): the prey's liberties plus the
  // liberties of hunter groups with one liberty that touch the prey (native is_ladder_capture).
  __device__ __forceinline__ void escape_set(int pr, unsigned long long* s) {
    const int pl = L->lab[pr];
    if (pl < 0) {
      libset(pr, s);
      return;
    }
    const int hunter = -me;
#pragma unroll
    for (int k = 0; k < kNPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P) {
        L->lib[p] = 0;
        L->adj[p] = 0;
      }
    }
    wsync();
#pragma unroll
    for (int k = 0; k < kNPL; ++k) {
      const int p = lane + 64 * k;
      if (p >= P) continue;
      const int lp = L->lab[p];
      int nl[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) nl[i] = nb[k][i] >= 0 ? (int)L->lab[nb[k][i]] : -1;
      if (lp < 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          bool dup = nl[i] < 0;
#pragma unroll
          for (int j = 0; j < i; ++j) dup |= nl[j] == nl[i];
          if (!dup) atomicAdd(&L->lib[nl[i]], 1);
        }
      } else if (lp == pl) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = nb[k][i];
          if (q >= 0 && L->col[q] == hunter) L->adj[nl[i]] = 1;
        }
      }
    }
    wsync();
#pragma unroll
    for (int k = 0; k < kNPL; ++k) {
      const int p = lane + 64 * k;
      bool hit = false;
      if (p < P && L->lab[p] < 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = nb[k][i];
          if (q < 0) continue;
          const int l = L->lab[q];
          if (l < 0) continue;
          hit |= l == pl || (L->col[q] == hunter && L->adj[l] && L->lib[l] == 1);
        }
      }
      s[k] = ballot(hit);  // private copy in every lane (the ballot is uniform)
    }
  }
};

__global__ void __launch_bounds__(64)
ladder_search_kernel(const int8_t* __restrict__ colors, const int32_t* __restrict__ meta,
                     const int16_t* __restrict__ labels, int S, int* __restrict__ queue,
                     const int* __restrict__ tasks, uint8_t* __restrict__ out,
                     int* __restrict__ overflow) {
  __shared__ SearchLds sh;
  const int lane = threadIdx.x;
  const int P = S * S;
  Wave w;
  w.L = &sh;
  w.S = S;
  w.P = P;
  w.lane = lane;
#pragma unroll
  for (int k = 0; k < kNPL; ++k)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = lane + 64 * k;
      w.nb[k][i] = p < P ? nbr(p, i, S) : -1;
    }
  const int ntasks = queue[0];
  while (true) {
    int t = 0;
    if (lane == 0) t = atomicAdd(&queue[1], 1);
    t = uni(__shfl(t, 0, 64));
    if (t >= ntasks) break;  // every wave of the grid exits here once the queue is drained
    const int task = tasks[t];
    const int pos = task >> 10, p0 = (task >> 1) & 511, kind0 = task & 1;
#pragma unroll
    for (int k = 0; k < kNPL; ++k) {
      const int p = lane + 64 * k;
      if (p < P) {
        sh.col[p] = colors[(size_t)pos * P + p];
        sh.lab[p] = labels[(size_t)pos * P + p];
      }
    }
    wsync();
    w.me = meta[pos * 4 + 0];
    w.ko = meta[pos * 4 + 1];

    // explicit DFS: the reference's is_ladder_capture / is_ladder_escape recursion
    enum { ST_CALL, ST_NEXT, ST_ITER, ST_RET };
    int st = ST_CALL;
    int kind = kind0, a = p0, pr = -1, rem = 80;
    int sp = -1;
    bool ret = false;
    int steps = 0;
    Wave::Around r;
    while (true) {
      if (++steps > kMaxSteps) {  // defensive bound: report, answer false (the next task
        if (lane == 0) atomicAdd(overflow, 1);  // reloads its board, so nothing to unwind)
        ret = false;
        break;
      }
      if (st == ST_CALL) {
        w.around(a, r);
        if (!w.legal(a, r)) {
          ret = false;
          st = ST_RET;
          continue;
        }
        if (rem <= 0) {
          ret = kind == K_CAP;
          st = ST_RET;
          continue;
        }
        // candidate prey: the given one, or the groups around a (slot-indexed)
        int candm = 0;
        if (pr >= 0) {
          candm = 1;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const bool ok = kind == K_CAP ? (((r.oppf >> i) & 1) && r.lc[i] == 2)
                                          : (((r.ownf >> i) & 1) && r.lc[i] == 1);
            candm |= ok ? 1 << i : 0;
          }
        }
        ++sp;
        Frame& f = sh.fr[sp];
        if (lane == 0) {
          f.kind = (int8_t)kind;
          f.a = (int16_t)a;
          f.rem = (int8_t)rem;
          f.candm = (int8_t)candm;
          f.ci = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) f.cand[i] = (int16_t)(pr >= 0 ? pr : r.l[i]);
        }
        wsync();
        st = ST_NEXT;
        continue;
      }
      if (st == ST_RET && sp < 0) break;  // the top-level call returned
      Frame& f = sh.fr[sp];
      if (st == ST_NEXT) {
        const int candm = uni(f.candm);
        int slot = uni(f.ci);
        while (slot < 4 && !((candm >> slot) & 1)) ++slot;
        if (slot >= 4) {  // no candidate prey is captured / escapes
          --sp;
          ret = false;
          st = ST_RET;
          continue;
        }
        const int fa = uni(f.a);
        int fpr = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i == slot) fpr = uni(f.cand[i]);
        w.around(fa, r);
        w.play(fa, r, f);
        if (lane == 0) {
          f.pr = (int16_t)fpr;
          f.ci = (int8_t)(slot + 1);
        }
        unsigned long long it[kNW];
        if (uni(f.kind) == K_CAP) {
          w.escape_set(fpr, it);
        } else {
          const int lc = w.libset(fpr, it);
          if (lc >= 3 || lc == 1) {
            w.undo(f);
            if (lc >= 3) {
              --sp;
              ret = true;
              st = ST_RET;
            }
            continue;  // lc == 1: next candidate (ST_NEXT)
          }
        }
        if (lane == 0)
#pragma unroll
          for (int k = 0; k < kNW; ++k) f.iter[k] = it[k];
        wsync();
        st = ST_ITER;
        continue;
      }
      if (st == ST_ITER) {
        int x = -1;
#pragma unroll
        for (int k = kNW - 1; k >= 0; --k) {
          const unsigned long long v = f.iter[k];
          if (v) x = k * 64 + __builtin_ctzll(v);
        }
        x = uni(x);
        if (x < 0) {  // capture: no escape works; escape: no capture works -> true
          w.undo(f);
          --sp;
          ret = true;
          st = ST_RET;
          continue;
        }
        if (lane == 0) f.iter[x >> 6] &= ~(1ull << (x & 63));
        wsync();
        kind = uni(f.kind) == K_CAP ? K_ESC : K_CAP;
        a = x;
        pr = uni(f.pr);
        rem = uni(f.rem) - 1;
        st = ST_CALL;
        continue;
      }
      // ST_RET: hand `ret` to the caller frame f. Parent CAP + child ESC true (an escape
      // works) or parent ESC + child CAP true (the prey is caught): this candidate prey is
      // settled, go on with the next one; otherwise try the caller's next option.
      if (ret) {
        w.undo(f);
        st = ST_NEXT;
      } else {
        st = ST_ITER;
      }
    }
    if (lane == 0) out[((size_t)pos * 2 + kind0) * P + p0] = ret ? 1 : 0;
    wsync();
  }
}

}  // namespace

// colors [n][S*S] int8 (device), meta [n][4] int32 (player to move, ko, ...), workspace from
// rag_ladder_workspace (zeroed queue counters are part of it), out [n][2][S*S] uint8 (capture,
// escape). S*S <= 384.
static size_t label_bytes(int n_pos, int S) {  // int16 labels, padded to 256 B
  return ((size_t)n_pos * S * S * 2 + 255) & ~(size_t)255;
}

RAG_API size_t rag_ladder_workspace(int n_pos, int S) {
  const size_t P = (size_t)S * S;
  return 256 + label_bytes(n_pos, S) + (size_t)n_pos * P * 2 * 4 /*tasks*/;
}

RAG_API int rag_ladders(const void* colors, const int32_t* meta, int n_pos, int S, void* work,
                        uint8_t* out, hipStream_t stream) {
  if (S < 2 || S * S > kPMAX || n_pos <= 0 || n_pos >= (1 << 21)) return -1;
  const size_t P = (size_t)S * S;
  char* w = (char*)work;
  int* queue = (int*)w;           // [0] tasks queued, [1] next task, [2] overflow count
  int16_t* labels = (int16_t*)(w + 256);
  int* tasks = (int*)(w + 256 + label_bytes(n_pos, S));
  (void)hipMemsetAsync(queue, 0, 64, stream);
  ladder_prep_kernel<<<n_pos, 64, 0, stream>>>((const int8_t*)colors, meta, n_pos, S, labels,
                                               queue, tasks, out);
  const int grid = 4 * 256;  // 4 single-wave workgroups per CU (LDS-bound), persistent
  ladder_search_kernel<<<grid, 64, 0, stream>>>((const int8_t*)colors, meta, labels, S, queue,
                                                tasks, out, queue + 2);
  return (int)hipGetLastError();
}

// Input feature planes on the GPU: one workgroup (one lane per board
// point, ceil(S*S/64) waves) builds every plane of one position, bit-exact with the native
// extractor (csrc/engine/features.cpp, itself pinned to the reference preprocessing.py:14-205
// by tests/test_features.py).
//
// Per position (LDS, S <= 19):
//   * colours, stone ages; group labels by min-label propagation over same-coloured neighbours;
//   * per label: stone count, liberty count, and the group's stone set and liberty set as 361-bit
//     bitsets (built with LDS 64-bit atomic ORs), so "liberties after playing p" is an exact set
//     union + popcount per candidate instead of a flood fill;
//   * each lane then evaluates its point: board / ones / zeros / color / turns_since /
//     liberties / legal (suicide, ko; superko via a host-provided mask) / capture_size /
//     self_atari_size / liberties_after (captured stones adjacent to the merged group become
//     liberties: bitset dilation, only on capturing moves) / sensibleness (the recursive true-eye
//     rule, as an explicit per-lane DFS with the ancestor stack) / ladder planes (host-provided:
//     ladder reading is a deep sequential search and stays in the native engine).
// Output: uint8 [n][F][S*S] in the order of `fids`, the layout batch_features produces.
#include "common.h"

using namespace rag;

namespace {

// One point per lane: the per-position latency (label propagation, per-point capture /
// liberties-after / true-eye work) is what bounds this kernel at the 64-512-position batches of
// self-play and search, so the position is spread over up to 6 waves instead of one wave
// walking 6 points per lane (164 -> ~30 us per 128-position ply, profiles/rl_bench_r3.txt).
constexpr int kNW = 6;    // 64-bit words of a 361-point set
constexpr int kPMAX = 384;
constexpr int kEye = 192;  // compact eyeish indices (3 x 64-bit ancestor words)

// feature ids (csrc/engine/go_engine.hpp FeatureId)
enum { F_BOARD = 0, F_ONES, F_TURNS_SINCE, F_LIBERTIES, F_CAPTURE_SIZE, F_SELF_ATARI_SIZE,
       F_LIBERTIES_AFTER, F_LADDER_CAPTURE, F_LADDER_ESCAPE, F_SENSIBLENESS, F_ZEROS, F_LEGAL,
       F_COLOR };

struct FShared {
  unsigned long long libbits[kPMAX][kNW];
  unsigned long long stonebits[kPMAX][kNW];
  int lib[kPMAX];
  int gsz[kPMAX];
  // true-eye DFS of the player to move, over the eyeish points only (<= 181 on 19x19: no two
  // are orthogonally adjacent), numbered compactly: per eyeish point its four diagonals in the
  // reference order as 10-bit entries (target index | class << 8; class 0 off the board / own
  // stone, 1 bad: an opponent stone or a non-eyeish empty point, 2 an eyeish point), bit 40 =
  // four neighbours (one bad diagonal allowed), bits 41-43 the class-1 count, bits 44-47 the
  // class-2 entries
  unsigned long long einfo[kEye];
  int16_t eid[kPMAX];      // compact index of an eyeish point, -1 otherwise
  int ewave[8];            // eyeish points per wave (the prefix of the numbering)
  int16_t frs[24][kPMAX];  // the DFS frame stack of each lane (level-major)
  int16_t lab[kPMAX];
  int8_t col[kPMAX];
};

struct Pos {
  int S, P;
  const int8_t* col;
  const int16_t* lab;
  const int* lib;
  const int* gsz;
  const unsigned long long (*libbits)[kNW];
  const unsigned long long (*stonebits)[kNW];

  __device__ int nb(int p, int k) const {
    const int x = p / S, y = p - (p / S) * S;
    switch (k) {
      case 0: return x > 0 ? p - S : -1;
      case 1: return x < S - 1 ? p + S : -1;
      case 2: return y > 0 ? p - 1 : -1;
      default: return y < S - 1 ? p + 1 : -1;
    }
  }
  // reference diagonal order: (x-1,y-1),(x+1,y+1),(x+1,y-1),(x-1,y+1)
  __device__ int dg(int p, int k) const {
    const int x = p / S, y = p - (p / S) * S;
    const int dx = (k == 0 || k == 3) ? -1 : 1;
    const int dy = (k == 0 || k == 2) ? -1 : 1;
    const int ax = x + dx, ay = y + dy;
    return (ax < 0 || ay < 0 || ax >= S || ay >= S) ? -1 : ax * S + ay;
  }
  __device__ int nnb(int p) const {
    const int x = p / S, y = p - (p / S) * S;
    return (x > 0) + (x < S - 1) + (y > 0) + (y < S - 1);
  }
  __device__ bool eyeish(int p, int owner) const {
    if (col[p] != 0) return false;
    for (int k = 0; k < 4; ++k) {
      const int q = nb(p, k);
      if (q >= 0 && col[q] != owner) return false;
    }
    return true;
  }
};

// set helpers over kNW words. Word selection is unrolled (compile-time indices): a runtime index
// into a register array puts the array in scratch.
__device__ __forceinline__ void set_bit6(unsigned long long* s, int q) {
#pragma unroll
  for (int w = 0; w < kNW; ++w) s[w] |= (w == (q >> 6)) ? (1ull << (q & 63)) : 0ull;
}
__device__ __forceinline__ void clear_bit6(unsigned long long* s, int q) {
#pragma unroll
  for (int w = 0; w < kNW; ++w) s[w] &= (w == (q >> 6)) ? ~(1ull << (q & 63)) : ~0ull;
}
__device__ __forceinline__ bool get_bit6(const unsigned long long* s, int q) {
  unsigned long long v = 0ull;
#pragma unroll
  for (int w = 0; w < kNW; ++w) v = (w == (q >> 6)) ? s[w] : v;
  return (v >> (q & 63)) & 1ull;
}
__device__ __forceinline__ int popc6(const unsigned long long* s) {
  int c = 0;
#pragma unroll
  for (int k = 0; k < kNW; ++k) c += __popcll(s[k]);
  return c;
}

// Recursive true-eye rule (go.py:298-327) for the player to move, as an explicit DFS over the
// compactly numbered eyeish points: the ancestors of the top frame as a 192-bit set in registers,
// a point's four classified diagonals from one 8-byte LDS entry, the frames below the top in this
// lane's LDS column. The lanes of a wave run it in lock-step, so each iteration does one small
// action: the first forms (a private frame array indexed by the per-lane depth, divisions by S, a
// scan of the frames, nested scan / unwind loops) cost up to ~3.7k cycles per DFS step, 350 of
// the 380 us of a late-game 128-board pass (benchmarks/features_bench.py --moves 250 450).
__device__ __forceinline__ bool anc_has(const unsigned long long (&a)[3], int i) {
  const unsigned long long w = i < 64 ? a[0] : (i < 128 ? a[1] : a[2]);
  return (w >> (i & 63)) & 1ull;
}
__device__ __forceinline__ void anc_flip(unsigned long long (&a)[3], int i) {
  const unsigned long long b = 1ull << (i & 63);
  a[0] ^= i < 64 ? b : 0ull;
  a[1] ^= (i >= 64 && i < 128) ? b : 0ull;
  a[2] ^= i >= 128 ? b : 0ull;
}
__device__ bool is_eye_dfs(int ci, const unsigned long long* einfo, int16_t* stk) {
  constexpr int MAXD = 24;
  unsigned long long anc[3] = {0ull, 0ull, 0ull};
  int sp = 0, cur = ci, fi = 0;
  unsigned long long inf = einfo[cur];
  int fb = (int)((inf >> 41) & 7);  // the opponent-stone / non-eyeish diagonals, counted up front
  bool ret = false, r = true;
  // one action per iteration (push one eyeish diagonal, or hand a result to the parent): the lanes
  // of a wave stay in step, so a wave pays the longest lane's action count. The rule's result does
  // not depend on the order of the diagonals (the recursion has no side effects: the stack is
  // restored), so a frame fails as soon as its bad count exceeds the allowance and succeeds as
  // soon as its remaining eyeish diagonals could not push it over (no recursion for those)
  while (true) {
    if (ret) {
      if (sp == 0) return r;
      const int f = stk[--sp * kPMAX];
      cur = f & 255;
      fi = (f >> 8) & 7;
      fb = (f >> 11) + (r ? 0 : 1);
      anc_flip(anc, cur);
      inf = einfo[cur];
      ret = false;
    }
    const int allow = (int)((inf >> 40) & 1);
    const unsigned m = ((unsigned)(inf >> 44) & 15u) >> fi;  // eyeish diagonals not yet visited
    if (fb > allow || fb + __popc(m) <= allow) {
      r = fb <= allow;
      ret = true;
      continue;
    }
    fi += __builtin_ctz(m);  // m != 0 here
    const int t = (int)((inf >> (10 * fi)) & 255);
    ++fi;
    if (anc_has(anc, t) || sp + 1 >= MAXD) continue;  // on the stack (or deeper than the
    stk[sp++ * kPMAX] = (int16_t)(cur | (fi << 8) | (fb << 11));  // reference ever reaches)
    anc_flip(anc, cur);
    cur = t;
    inf = einfo[t];
    fi = 0;
    fb = (int)((inf >> 41) & 7);
  }
}

// No scratch and ~171 VGPRs (was 256 + 448 B/lane of scratch: runtime-indexed neighbour lists,
// bit sets and DFS frames): two waves of a block now fit on a SIMD beside one of the search's
// resident rollout waves (128 VGPRs); at 256 a block needed SIMDs free of rollout waves, and the
// 512-leaf feature passes waited behind the 5 ms rollout kernels (413 us per pass,
// profiles/mcts_kernels_r4.txt). WPE = 4 (RAG_FEATURES_WPE=4): 128 VGPRs, so a wave fits even
// beside three resident rollout waves (their 3 x 128 VGPRs), at the cost of scratch spills.
template <int WPE>
__global__ void __launch_bounds__(kPMAX, WPE)
features_kernel(const int8_t* __restrict__ colors, const int16_t* __restrict__ ages,
                const int32_t* __restrict__ meta, const uint8_t* __restrict__ extra_illegal,
                const uint8_t* __restrict__ ladders, int n_pos, int S, const int* __restrict__ fids,
                int nf, int F, uint8_t* __restrict__ out, uint8_t* __restrict__ sens) {
  __shared__ FShared sh;
  const int pos = blockIdx.x;
  const int p = threadIdx.x;
  const int P = S * S;
  const bool on = p < P;
  int8_t* col = sh.col;
  int16_t* lab = sh.lab;
  int* lib = sh.lib;
  int* gsz = sh.gsz;
  Pos g{S, P, col, lab, lib, gsz, sh.libbits, sh.stonebits};
  const int me = meta[pos * 4 + 0];
  const int ko = meta[pos * 4 + 1];

  int c = 0;
  if (on) {
    c = colors[(size_t)pos * P + p];
    col[p] = (int8_t)c;
    lab[p] = c ? (int16_t)p : (int16_t)-1;
    lib[p] = 0;
    gsz[p] = 0;
#pragma unroll
    for (int w = 0; w < kNW; ++w) {
      sh.libbits[p][w] = 0ull;
      sh.stonebits[p][w] = 0ull;
    }
  }
  __syncthreads();
  // the true-eye DFS tables (col[] of every point is in LDS now): eyeish points numbered by a
  // ballot prefix over the waves, then each one's classified diagonals
  const bool eyish = on && g.eyeish(p, me);
  {
    const unsigned long long bm = __ballot(eyish);
    if ((p & 63) == 0) sh.ewave[p >> 6] = __popcll(bm);
    __syncthreads();
    int base = 0;
    for (int k = 0; k < (p >> 6); ++k) base += sh.ewave[k];
    const int rank = __popcll(bm & ((1ull << (p & 63)) - 1ull));
    if (on) sh.eid[p] = eyish ? (int16_t)(base + rank) : (int16_t)-1;
    __syncthreads();
  }
  if (eyish) {
    unsigned long long inf = 0ull;
    int n1 = 0, m2 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int d = g.dg(p, k);
      int e = 0;
      if (d >= 0) {
        const int cd = col[d];
        if (cd == -me) e = 1 << 8;
        else if (cd == 0) e = sh.eid[d] >= 0 ? (2 << 8) | sh.eid[d] : (1 << 8);
      }
      inf |= (unsigned long long)e << (10 * k);
      n1 += (e >> 8) == 1;
      m2 |= ((e >> 8) == 2) << k;
    }
    if (g.nnb(p) == 4) inf |= 1ull << 40;
    inf |= (unsigned long long)n1 << 41 | (unsigned long long)m2 << 44;
    sh.einfo[sh.eid[p]] = inf;
  }
  // labels: min stone index of the group. Lanes of other waves may read a neighbour's label
  // while it is lowered; every value read is the index of a stone of the same group and labels
  // only decrease, so the race is benign, and an iteration in which no lane changed anything saw
  // a fixpoint.
  for (int it = 0; it < 2 * kPMAX; ++it) {
    int changed = 0;
    if (on && c != 0) {
      int m = lab[lab[p]];
      for (int i = 0; i < 4; ++i) {
        const int q = g.nb(p, i);
        if (q >= 0 && col[q] == c) m = min(m, (int)lab[q]);
      }
      if (m < lab[p]) {
        lab[p] = (int16_t)m;
        changed = 1;
      }
    }
    if (!__syncthreads_or(changed)) break;
  }
  // per-label tables
  if (on) {
    const unsigned long long bit = 1ull << (p & 63);
    if (c != 0) {
      const int l = lab[p];
      atomicAdd(&gsz[l], 1);
      atomicOr(&sh.stonebits[l][p >> 6], bit);
    } else {
      // each distinct neighbouring group gains this liberty (neighbours unrolled: static indices)
      int nl[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = g.nb(p, i);
        nl[i] = (q >= 0 && col[q] != 0) ? (int)lab[q] : -1;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        bool dup = nl[i] < 0;
#pragma unroll
        for (int j = 0; j < i; ++j) dup |= nl[j] == nl[i];
        if (dup) continue;
        atomicAdd(&lib[nl[i]], 1);
        atomicOr(&sh.libbits[nl[i]][p >> 6], bit);
      }
    }
  }
  __syncthreads();
  if (!on) return;

  // plane offsets of the requested features
  uint8_t* o = out + (size_t)pos * F * P;
  {
    // ---- legality, captures and the simulated move. Per neighbour i: its group label nlab[i]
    // and class cls[i] (0 off-board / empty, 1 own, 2 capturable opponent, 3 other opponent);
    // uniq[i]: the first neighbour of its (class, group). Unrolled, so no array leaves registers.
    int nlab[4], cls[4];
    bool uniq[4];
    int empty_nb = 0, ncap = 0;
    bool own_multi = false;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = g.nb(p, i);
      cls[i] = 0;
      nlab[i] = -1;
      if (q < 0) continue;
      const int cq = col[q];
      if (cq == 0) {
        ++empty_nb;
        continue;
      }
      const int l = lab[q];
      nlab[i] = l;
      if (cq == me) {
        cls[i] = 1;
        if (lib[l] > 1) own_multi = true;
      } else {
        cls[i] = lib[l] == 1 ? 2 : 3;
      }
    }
    int cap_size = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool u = cls[i] == 1 || cls[i] == 2;
#pragma unroll
      for (int j = 0; j < i; ++j) u &= !(cls[j] == cls[i] && nlab[j] == nlab[i]);
      uniq[i] = u;
      if (u && cls[i] == 2) {
        ++ncap;
        cap_size += gsz[nlab[i]];
      }
    }
    const bool suicide = empty_nb == 0 && !own_multi && ncap == 0;
    const bool legal = c == 0 && p != ko && !suicide &&
                       !(extra_illegal && extra_illegal[(size_t)pos * P + p]);
    int libs_after = 0, size_after = 1;
    bool need_after = false;
    for (int fi = 0; fi < nf; ++fi)
      need_after |= fids[fi] == F_SELF_ATARI_SIZE || fids[fi] == F_LIBERTIES_AFTER;
    if (legal && need_after) {
      unsigned long long ls[kNW];
#pragma unroll
      for (int w = 0; w < kNW; ++w) ls[w] = 0ull;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = g.nb(p, i);
        if (q >= 0 && col[q] == 0) set_bit6(ls, q);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!(uniq[i] && cls[i] == 1)) continue;
        size_after += gsz[nlab[i]];
#pragma unroll
        for (int w = 0; w < kNW; ++w) ls[w] |= sh.libbits[nlab[i]][w];
      }
      if (ncap > 0) {
        unsigned long long grp[kNW], cap[kNW];
#pragma unroll
        for (int w = 0; w < kNW; ++w) {
          grp[w] = 0ull;
          cap[w] = 0ull;
        }
        set_bit6(grp, p);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (!uniq[i]) continue;
#pragma unroll
          for (int w = 0; w < kNW; ++w) {
            if (cls[i] == 1) grp[w] |= sh.stonebits[nlab[i]][w];
            else cap[w] |= sh.stonebits[nlab[i]][w];
          }
        }
        // captured stones orthogonally adjacent to the merged group become liberties
#pragma unroll
        for (int w = 0; w < kNW; ++w) {
          unsigned long long m = cap[w];
          while (m) {
            const int s = w * 64 + __builtin_ctzll(m);
            m &= m - 1;
            bool adj = false;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int q = g.nb(s, i);
              adj |= q >= 0 && get_bit6(grp, q);
            }
            if (adj) ls[w] |= 1ull << (s & 63);
          }
        }
      }
      clear_bit6(ls, p);
      libs_after = popc6(ls);
    }
    // ---- write the planes (the true-eye DFS at most once per point)
    int sensible = -1;
    auto get_sensible = [&]() {
      if (sensible < 0)
        sensible = legal && !(sh.eid[p] >= 0 && is_eye_dfs(sh.eid[p], sh.einfo, &sh.frs[0][p]));
      return sensible;
    };
    if (sens) sens[(size_t)pos * P + p] = (uint8_t)get_sensible();
    int base = 0;
    for (int fi = 0; fi < nf; ++fi) {
      const int f = fids[fi];
      uint8_t* op = o + (size_t)base * P + p;
      switch (f) {
        case F_BOARD:
          op[0] = c == me;
          op[P] = c == -me;
          op[2 * P] = c == 0;
          base += 3;
          break;
        case F_ONES:
          op[0] = 1;
          base += 1;
          break;
        case F_ZEROS:
          op[0] = 0;
          base += 1;
          break;
        case F_COLOR:
          op[0] = me == 1;
          base += 1;
          break;
        case F_TURNS_SINCE: {
          const int a = ages[(size_t)pos * P + p];
          for (int t = 0; t < 8; ++t) op[t * P] = (a >= 0 && min(a, 7) == t);
          base += 8;
          break;
        }
        case F_LIBERTIES: {
          const int l = c ? lib[lab[p]] : -1;
          for (int t = 0; t < 8; ++t) op[t * P] = (l >= 1 && (l - 1 == t || (t == 7 && l >= 8)));
          base += 8;
          break;
        }
        case F_CAPTURE_SIZE: {
          const int idx = min(cap_size, 7);
          for (int t = 0; t < 8; ++t) op[t * P] = legal && idx == t;
          base += 8;
          break;
        }
        case F_SELF_ATARI_SIZE: {
          const int idx = min(size_after - 1, 7);
          for (int t = 0; t < 8; ++t) op[t * P] = legal && libs_after == 1 && idx == t;
          base += 8;
          break;
        }
        case F_LIBERTIES_AFTER: {
          int idx = min(7, libs_after - 1);
          if (idx < 0) idx += 8;  // python negative index semantics (features.cpp)
          for (int t = 0; t < 8; ++t) op[t * P] = legal && idx == t;
          base += 8;
          break;
        }
        case F_LADDER_CAPTURE:
          op[0] = legal && ladders && ladders[((size_t)pos * 2 + 0) * P + p];
          base += 1;
          break;
        case F_LADDER_ESCAPE:
          op[0] = legal && ladders && ladders[((size_t)pos * 2 + 1) * P + p];
          base += 1;
          break;
        case F_SENSIBLENESS:
          op[0] = (uint8_t)get_sensible();
          base += 1;
          break;
        case F_LEGAL:
          op[0] = legal;
          base += 1;
          break;
        default:
          break;
      }
    }
  }
}

}  // namespace

// colors [n][S*S] int8, ages [n][S*S] int16 (-1 = empty), meta [n][4] int32 (player to move,
// ko point, 0, 0), extra_illegal [n][S*S] uint8 or null (positional-superko points),
// ladders [n][2][S*S] uint8 or null (capture, escape), fids [nf] int32 on the device,
// out [n][F][S*S] uint8, sens [n][S*S] uint8 or null (the sensible-move mask of the player to
// move, written in the same pass). S <= 19.
RAG_API int rag_features(const void* colors, const void* ages, const int32_t* meta,
                         const uint8_t* extra_illegal, const uint8_t* ladders, int n_pos, int S,
                         const int* fids, int nf, int F, uint8_t* out, uint8_t* sens,
                         hipStream_t stream) {
  if (S < 2 || S * S > kPMAX || n_pos <= 0) return -1;
  const int threads = (S * S + 63) / 64 * 64;
  static const int wpe = [] {
    const char* e = getenv("RAG_FEATURES_WPE");
    return e && atoi(e) == 4 ? 4 : 2;
  }();
  if (wpe == 4)
    features_kernel<4><<<dim3(n_pos), threads, 0, stream>>>(
        (const int8_t*)colors, (const int16_t*)ages, meta, extra_illegal, ladders, n_pos, S, fids,
        nf, F, out, sens);
  else
    features_kernel<2><<<dim3(n_pos), threads, 0, stream>>>(
        (const int8_t*)colors, (const int16_t*)ages, meta, extra_illegal, ladders, n_pos, S, fids,
        nf, F, out, sens);
  return (int)hipGetLastError();
}

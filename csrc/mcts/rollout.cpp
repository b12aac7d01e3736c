// Fast rollout policy (see rollout.hpp).
#include "rollout.hpp"

#include <cmath>
#include <memory>
#include <mutex>

namespace rag {

const Ring8* Ring8::get(int S) {
  static std::mutex mu;
  static std::unique_ptr<Ring8> tabs[MAXS + 1];
  std::lock_guard<std::mutex> lock(mu);
  if (!tabs[S]) {
    auto r = std::make_unique<Ring8>();
    r->S = S;
    // clockwise from north; "north" = y+1 (GTP row up), x = column
    static const int dx[8] = {0, 1, 1, 1, 0, -1, -1, -1};
    static const int dy[8] = {1, 1, 0, -1, -1, -1, 0, 1};
    for (int x = 0; x < S; ++x)
      for (int y = 0; y < S; ++y)
        for (int k = 0; k < 8; ++k) {
          const int nx = x + dx[k], ny = y + dy[k];
          r->nb[x * S + y][k] = (nx < 0 || ny < 0 || nx >= S || ny >= S) ? -1 : nx * S + ny;
        }
    tabs[S] = std::move(r);
  }
  return tabs[S].get();
}

RolloutPolicy::RolloutPolicy() : pattern(RP_PATTERNS, 0.f) {
  w[RF_RESPONSE] = 1.0f;
  w[RF_SAVE_ATARI] = 2.0f;
  w[RF_CAPTURE] = 3.0f;
  w[RF_SELF_ATARI] = -3.0f;
  w[RF_NEAR2] = 0.5f;
  w[RF_OWN_NEAR] = 0.3f;
  w[RF_EDGE] = -0.8f;
}

bool rollout_is_own_eye(const Board& b, int p, int c) {
  const Geometry& g = b.geom();
  for (int i = 0; i < g.nnbr[p]; ++i)
    if (b.color(g.nbr[p][i]) != c) return false;
  int bad = 0;
  for (int i = 0; i < g.ndiag[p]; ++i)
    if (b.color(g.diag[p][i]) == -c) ++bad;
  const bool edge = g.nnbr[p] < 4;
  return edge ? bad == 0 : bad <= 1;
}

int RolloutPolicy::candidates(const Board& b, int* moves, uint8_t* fbits, int32_t* pat) const {
  const int S = b.size(), P = b.npoints();
  const int c = b.current_player();
  const Geometry& g = b.geom();
  const Ring8& r8 = *Ring8::get(S);
  const int l1 = b.last1(), l2 = b.last2();
  const int l1x = l1 >= 0 ? l1 / S : -100, l1y = l1 >= 0 ? l1 % S : -100;
  const int l2x = l2 >= 0 ? l2 / S : -100, l2y = l2 >= 0 ? l2 % S : -100;
  int n = 0;
  for (int a = 0; a < P; ++a) {
    if (b.color(a) != EMPTY) continue;
    if (rollout_is_own_eye(b, a, c)) continue;
    const int x = a / S, y = a % S;
    uint8_t f = 0;
    const int d1x = std::abs(x - l1x), d1y = std::abs(y - l1y);
    if (d1x <= 1 && d1y <= 1) f |= 1 << RF_RESPONSE;
    else if (d1x + d1y <= 2) f |= 1 << RF_NEAR2;
    if (std::abs(x - l2x) <= 1 && std::abs(y - l2y) <= 1) f |= 1 << RF_OWN_NEAR;
    if (x == 0 || y == 0 || x == S - 1 || y == S - 1) f |= 1 << RF_EDGE;
    int empty_nb = 0, own_libs = 0;
    bool capture = false, own_atari = false;
    for (int i = 0; i < g.nnbr[a]; ++i) {
      const int q = g.nbr[a][i];
      const int cq = b.color(q);
      if (cq == EMPTY) {
        ++empty_nb;
      } else if (cq == c) {
        const int lc = b.liberty_count(q);
        if (lc == 1) own_atari = true;
        own_libs += lc - 1;  // a itself is one of them (upper bound: shared liberties)
      } else if (b.liberty_count(q) == 1) {
        capture = true;
      }
    }
    if (capture) f |= 1 << RF_CAPTURE;
    if (own_atari && (empty_nb >= 2 || capture)) f |= 1 << RF_SAVE_ATARI;
    if (!capture && empty_nb + own_libs <= 1) f |= 1 << RF_SELF_ATARI;
    int pidx = 0;
    for (int k = 0; k < 8; ++k) {
      const int q = r8.nb[a][k];
      int code = 3;
      if (q >= 0) {
        const int cq = b.color(q);
        code = cq == EMPTY ? 0 : (cq == c ? 1 : 2);
      }
      pidx |= code << (2 * k);
    }
    moves[n] = a;
    fbits[n] = f;
    pat[n] = pidx;
    ++n;
  }
  return n;
}

int RolloutPolicy::sample(const Board& b, Rng& rng, int* mv, float* p) const {
  uint8_t fb[MAXP];
  int32_t pt[MAXP];
  int n = candidates(b, mv, fb, pt);
  float tot = 0.f;
  for (int i = 0; i < n; ++i) {
    float s = pattern[pt[i]];
    for (int f = 0; f < RF_COUNT; ++f)
      if (fb[i] >> f & 1) s += w[f];
    p[i] = std::exp(std::fmin(s, 30.f));
    tot += p[i];
  }
  while (n > 0) {
    float u = rng.uniform() * tot;
    int k = 0;
    for (; k < n - 1; ++k) {
      u -= p[k];
      if (u <= 0.f) break;
    }
    if (b.is_legal(mv[k])) return mv[k];
    tot -= p[k];
    mv[k] = mv[n - 1];
    p[k] = p[n - 1];
    --n;
    if (tot <= 0.f) {  // numerical leftovers: recompute
      tot = 0.f;
      for (int i = 0; i < n; ++i) tot += p[i];
    }
  }
  return PASS;
}

int RolloutPolicy::rollout(Board& b, Rng& rng, int limit) const {
  b.set_light(true);
  int mv[MAXP];
  float p[MAXP];
  for (int i = 0; i < limit && !b.end_of_game(); ++i) b.play_unchecked(sample(b, rng, mv, p));
  return b.get_winner();
}

}  // namespace rag

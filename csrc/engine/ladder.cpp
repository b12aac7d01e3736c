// Ladder reading on one working board with in-place moves and an undo journal.
//
// Behavioural contract: GameState.is_ladder_capture / is_ladder_escape of the reference
// (AlphaGo/go.py:329-463, remaining_attempts = 80) and the feature planes built from them
// (AlphaGo/preprocessing/preprocessing.py:172-187). The recursive reader on Board
// (go_engine.cpp) copies the whole state at every ply; this one makes ONE copy per position and
// then plays / takes back moves on it: every write to the point arrays is journaled
// (address + old value) and undone in reverse, and the two scalars a ladder ply changes (ko
// point, player to move) are saved per frame. The control flow, candidate order and escape /
// capture point order are exactly those of the recursive reader, so the planes are bit-identical
// (tests/test_ladders.py checks both readers on the reference scenarios and on random games).
//
// Positional superko makes legality depend on the game history, which a ladder ply would have
// to extend: boards that enforce it keep using the copying reader.
#include <algorithm>

#include "go_engine.hpp"

namespace rag {

void LadderReader::reset(const Board& b) {
  b_ = b;
  b_.set_light(true);
  j8_.clear();
  j16_.clear();
  frames_.clear();
}

void LadderReader::play(int a) {
  Board& b = b_;
  const Geometry& g = *b.g_;
  frames_.push_back(Frame{(uint32_t)j8_.size(), (uint32_t)j16_.size(), b.ko_, b.current_player_});
  const int c = b.current_player_;
  b.ko_ = -1;
  // place_stone (go_engine.cpp) with journaled writes; hash / ages / history are not read by a
  // ladder search and are left alone
  set8(b.color_[a], (int8_t)c);
  int fh[4], eh[4];
  int nf = 0, ne = 0;
  for (int i = 0; i < g.nnbr[a]; ++i) {
    const int n = g.nbr[a][i];
    const int h = b.head_[n];
    if (h < 0) continue;
    int* lst = b.color_[n] == c ? fh : eh;
    int& cnt = b.color_[n] == c ? nf : ne;
    bool dup = false;
    for (int t = 0; t < cnt; ++t) dup |= (lst[t] == h);
    if (!dup) lst[cnt++] = h;
  }
  for (int t = 0; t < ne; ++t) set16(b.libcnt_[eh[t]], (int16_t)(b.libcnt_[eh[t]] - 1));
  if (nf == 0) {
    set16(b.head_[a], (int16_t)a);
    set16(b.nxt_[a], (int16_t)a);
    set16(b.gsize_[a], 1);
    int lc = 0;
    for (int i = 0; i < g.nnbr[a]; ++i) lc += (b.color_[g.nbr[a][i]] == EMPTY);
    set16(b.libcnt_[a], (int16_t)lc);
  } else {
    int tgt = fh[0];
    for (int t = 1; t < nf; ++t)
      if (b.gsize_[fh[t]] > b.gsize_[tgt]) tgt = fh[t];
    set16(b.head_[a], (int16_t)tgt);
    set16(b.nxt_[a], b.nxt_[tgt]);
    set16(b.nxt_[tgt], (int16_t)a);
    set16(b.gsize_[tgt], (int16_t)(b.gsize_[tgt] + 1));
    for (int t = 0; t < nf; ++t) {
      const int h = fh[t];
      if (h == tgt) continue;
      int s = h;
      do {
        set16(b.head_[s], (int16_t)tgt);
        s = b.nxt_[s];
      } while (s != h);
      const int16_t nt = b.nxt_[tgt], nh = b.nxt_[h];
      set16(b.nxt_[tgt], nh);
      set16(b.nxt_[h], nt);
      set16(b.gsize_[tgt], (int16_t)(b.gsize_[tgt] + b.gsize_[h]));
    }
    Bitset l;
    b.liberty_set(tgt, l);
    set16(b.libcnt_[tgt], (int16_t)l.count(b.W_));
  }
  // captures in neighbour order, ko for a lone capturing stone left with one liberty
  for (int i = 0; i < g.nnbr[a]; ++i) {
    const int n = g.nbr[a][i];
    if (b.color_[n] != -c) continue;
    const int h = b.head_[n];
    if (b.libcnt_[h] != 0) continue;
    const int num = b.gsize_[h];
    int stones[MAXP];
    int ns = 0;
    int s = h;
    do {
      stones[ns++] = s;
      s = b.nxt_[s];
    } while (s != h);
    for (int k = 0; k < ns; ++k) set8(b.color_[stones[k]], (int8_t)EMPTY);
    for (int k = 0; k < ns; ++k) {
      const int r = stones[k];
      set16(b.head_[r], -1);
      set16(b.nxt_[r], -1);
      int seen[4];
      int kk = 0;
      for (int j = 0; j < g.nnbr[r]; ++j) {
        const int hn = b.head_[g.nbr[r][j]];
        if (hn < 0) continue;
        bool dup = false;
        for (int t = 0; t < kk; ++t) dup |= (seen[t] == hn);
        if (dup) continue;
        seen[kk++] = hn;
        set16(b.libcnt_[hn], (int16_t)(b.libcnt_[hn] + 1));
      }
    }
    if (num == 1) {
      const int hp = b.head_[a];
      if (b.libcnt_[hp] == 1 && b.gsize_[hp] == 1) b.ko_ = n;
    }
  }
  b.current_player_ = -c;
}

void LadderReader::undo() {
  const Frame f = frames_.back();
  frames_.pop_back();
  for (size_t k = j16_.size(); k-- > f.n16;) *j16_[k].p = j16_[k].old;
  j16_.resize(f.n16);
  for (size_t k = j8_.size(); k-- > f.n8;) *j8_[k].p = j8_[k].old;
  j8_.resize(f.n8);
  b_.ko_ = f.ko;
  b_.current_player_ = f.player;
}

// is_legal of a light board without superko (go.py:219-240)
inline bool LadderReader::legal(int a) const { return b_.is_legal(a); }

bool LadderReader::capture(int a, int prey, int remaining) {
  const Board& b = b_;
  if (!legal(a)) return false;
  if (remaining <= 0) return true;
  const int hunter = b.current_player_;
  int cand[4];
  int nc = 0;
  if (prey < 0) {
    int heads[4];
    const int nh = b.groups_around(a, heads);
    for (int i = 0; i < nh; ++i)
      if (b.color_[heads[i]] == -hunter && b.libcnt_[heads[i]] == 2) cand[nc++] = heads[i];
  } else {
    cand[nc++] = prey;
  }
  const Geometry& g = *b.g_;
  for (int c = 0; c < nc; ++c) {
    const int pr = cand[c];
    play(a);
    Bitset esc;
    b.liberty_set(pr, esc);
    if (b.head_[pr] >= 0) {
      int s = pr;
      do {
        for (int i = 0; i < g.nnbr[s]; ++i) {
          const int n = g.nbr[s][i];
          if (b.color_[n] == hunter && b.libcnt_[b.head_[n]] == 1) {
            Bitset l;
            b.liberty_set(n, l);
            esc.or_with(l, b.W_);
          }
        }
        s = b.nxt_[s];
      } while (s != pr);
    }
    bool any_escape = false;
    for (int k = 0; k < b.W_ && !any_escape; ++k) {
      uint64_t x = esc.w[k];
      while (x && !any_escape) {
        const int e = k * 64 + __builtin_ctzll(x);
        x &= x - 1;
        if (escape(e, pr, remaining - 1)) any_escape = true;
      }
    }
    undo();
    if (!any_escape) return true;
  }
  return false;
}

bool LadderReader::escape(int a, int prey, int remaining) {
  const Board& b = b_;
  if (!legal(a)) return false;
  if (remaining <= 0) return false;
  const int prey_player = b.current_player_;
  int cand[4];
  int nc = 0;
  if (prey < 0) {
    int heads[4];
    const int nh = b.groups_around(a, heads);
    for (int i = 0; i < nh; ++i)
      if (b.color_[heads[i]] == prey_player && b.libcnt_[heads[i]] == 1) cand[nc++] = heads[i];
  } else {
    cand[nc++] = prey;
  }
  for (int c = 0; c < nc; ++c) {
    const int pr = cand[c];
    play(a);
    const int lc = b.liberty_count(pr);
    if (lc >= 3) {
      undo();
      return true;
    }
    if (lc == 1) {
      undo();
      continue;
    }
    Bitset libs;
    b.liberty_set(pr, libs);
    bool captured = false;
    for (int k = 0; k < b.W_ && !captured; ++k) {
      uint64_t x = libs.w[k];
      while (x && !captured) {
        const int q = k * 64 + __builtin_ctzll(x);
        x &= x - 1;
        if (capture(q, pr, remaining - 1)) captured = true;
      }
    }
    undo();
    if (captured) continue;
    return true;
  }
  return false;
}

// Both ladder planes of one position (1 where is_ladder_capture / is_ladder_escape holds).
// Only points that are a liberty of an opponent group with two liberties (capture) or of an own
// group in atari (escape) can read true; every other point is answered without touching the
// working board, which is copied at most once.
void ladder_planes(const Board& b, uint8_t* cap, uint8_t* esc, LadderReader* reader) {
  const int P = b.npoints();
  std::memset(cap, 0, P);
  std::memset(esc, 0, P);
  if (b.enforce_superko()) {
    for (int p = 0; p < P; ++p) {
      if (b.color(p) != EMPTY) continue;
      cap[p] = b.is_ladder_capture(p, -1, 80) ? 1 : 0;
      esc[p] = b.is_ladder_escape(p, -1, 80) ? 1 : 0;
    }
    return;
  }
  const int me = b.current_player();
  bool loaded = false;
  LadderReader local;
  LadderReader& R = reader ? *reader : local;
  for (int p = 0; p < P; ++p) {
    if (b.color(p) != EMPTY) continue;
    int heads[4];
    const int nh = b.groups_around(p, heads);
    bool want_cap = false, want_esc = false;
    for (int i = 0; i < nh; ++i) {
      const int lc = b.liberty_count(heads[i]);
      if (b.color(heads[i]) == -me && lc == 2) want_cap = true;
      if (b.color(heads[i]) == me && lc == 1) want_esc = true;
    }
    if (!want_cap && !want_esc) continue;
    if (!loaded) {
      R.reset(b);
      loaded = true;
    }
    if (want_cap) cap[p] = R.capture(p, -1, 80) ? 1 : 0;
    if (want_esc) esc[p] = R.escape(p, -1, 80) ? 1 : 0;
  }
}

}  // namespace rag

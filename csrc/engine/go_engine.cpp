// Native Go rules engine — see go_engine.hpp for the behavioural contract.
#include "go_engine.hpp"

#include <algorithm>
#include <mutex>
#include <string>

namespace rag {

// ------------------------------------------------------------------ geometry
const Geometry* Geometry::get(int S) {
  static Geometry* cache[MAXS + 1] = {nullptr};
  static std::mutex mu;
  if (S < 1 || S > MAXS) throw std::invalid_argument("board size out of range (1..25)");
  std::lock_guard<std::mutex> lk(mu);
  if (cache[S]) return cache[S];
  Geometry* g = new Geometry();
  g->S = S;
  g->P = S * S;
  g->W = (g->P + 63) / 64;
  auto on = [S](int x, int y) { return x >= 0 && y >= 0 && x < S && y < S; };
  for (int x = 0; x < S; ++x)
    for (int y = 0; y < S; ++y) {
      int p = x * S + y;
      const int nx[4] = {x - 1, x + 1, x, x};
      const int ny[4] = {y, y, y - 1, y + 1};
      int k = 0;
      for (int i = 0; i < 4; ++i)
        if (on(nx[i], ny[i])) g->nbr[p][k++] = (int16_t)(nx[i] * S + ny[i]);
      g->nnbr[p] = (int8_t)k;
      for (int i = k; i < 4; ++i) g->nbr[p][i] = -1;
      const int dx[4] = {x - 1, x + 1, x + 1, x - 1};
      const int dy[4] = {y - 1, y + 1, y - 1, y + 1};
      k = 0;
      for (int i = 0; i < 4; ++i)
        if (on(dx[i], dy[i])) g->diag[p][k++] = (int16_t)(dx[i] * S + dy[i]);
      g->ndiag[p] = (int8_t)k;
      for (int i = k; i < 4; ++i) g->diag[p][i] = -1;
    }
  cache[S] = g;
  return g;
}

// ------------------------------------------------------------------ construction / copy
Board::Board(int size, double komi, bool enforce_superko, std::shared_ptr<const Zobrist> zob)
    : g_(Geometry::get(size)), zob_(std::move(zob)), S_(size), P_(size * size),
      W_((size * size + 63) / 64), enforce_superko_(enforce_superko), komi_(komi) {
  if (!zob_ || (int)zob_->white.size() != P_ || (int)zob_->black.size() != P_)
    throw std::invalid_argument("zobrist tables must have size*size entries");
  history_ = std::make_shared<std::vector<int16_t>>();
  prev_hashes_ = std::make_shared<std::vector<uint64_t>>();
  std::memset(color_, 0, P_);
  for (int p = 0; p < P_; ++p) {
    head_[p] = -1;
    nxt_[p] = -1;
    gsize_[p] = 0;
    libcnt_[p] = 0;
    placed_[p] = 0;
  }
}

void Board::copy_from(const Board& o) {
  g_ = o.g_;
  // shared pointers are assigned only when they differ: search threads copy one root board into
  // recycled leaf boards that already share its tables, and an unconditional assignment would
  // bounce the control blocks' reference counts between all of them
  if (zob_ != o.zob_) zob_ = o.zob_;
  S_ = o.S_;
  P_ = o.P_;
  W_ = o.W_;
  current_player_ = o.current_player_;
  ko_ = o.ko_;
  black_prisoners_ = o.black_prisoners_;
  white_prisoners_ = o.white_prisoners_;
  passes_black_ = o.passes_black_;
  passes_white_ = o.passes_white_;
  end_of_game_ = o.end_of_game_;
  enforce_superko_ = o.enforce_superko_;
  light_ = o.light_;
  last1_ = o.last1_;
  last2_ = o.last2_;
  nmoves_ = o.nmoves_;
  komi_ = o.komi_;
  hash_ = o.hash_;
  clock_ = o.clock_;
  if (history_ != o.history_) history_ = o.history_;                // copy-on-write
  if (prev_hashes_ != o.prev_hashes_) prev_hashes_ = o.prev_hashes_;  // copy-on-write
  if (!(handicaps_.empty() && o.handicaps_.empty())) handicaps_ = o.handicaps_;
  std::memcpy(color_, o.color_, P_);
  std::memcpy(head_, o.head_, sizeof(int16_t) * P_);
  std::memcpy(nxt_, o.nxt_, sizeof(int16_t) * P_);
  std::memcpy(gsize_, o.gsize_, sizeof(int16_t) * P_);
  std::memcpy(libcnt_, o.libcnt_, sizeof(int16_t) * P_);
  std::memcpy(placed_, o.placed_, sizeof(uint32_t) * P_);
}

Board Board::from_arrays(int S, double komi, std::shared_ptr<const Zobrist> zob,
                         const int8_t* colors, const int16_t* ages, const int32_t* meta8) {
  Board b(S, komi, false, std::move(zob));
  b.light_ = true;
  const int P = b.P_;
  const Geometry& g = *b.g_;
  // stone ages: age = clock - placed; a clock above every age keeps placed >= 0
  b.clock_ = 1u << 20;
  for (int p = 0; p < P; ++p) {
    b.color_[p] = colors[p];
    if (colors[p] != EMPTY) {
      const int age = ages ? std::max<int>(ages[p], 0) : 0;
      b.placed_[p] = b.clock_ - (uint32_t)age;
      b.hash_ ^= colors[p] == WHITE ? b.zob_->white[p] : b.zob_->black[p];
    }
  }
  // groups: flood fill into circular lists headed by their first point
  int stack[MAXP];
  for (int p = 0; p < P; ++p) {
    if (b.color_[p] == EMPTY || b.head_[p] >= 0) continue;
    const int c = b.color_[p];
    int n = 0, prev = p;
    stack[n++] = p;
    b.head_[p] = (int16_t)p;
    int size = 0;
    while (n) {
      const int q = stack[--n];
      ++size;
      if (q != p) {
        b.nxt_[prev] = (int16_t)q;
        prev = q;
      }
      for (int i = 0; i < g.nnbr[q]; ++i) {
        const int r = g.nbr[q][i];
        if (b.color_[r] == c && b.head_[r] < 0) {
          b.head_[r] = (int16_t)p;
          stack[n++] = r;
        }
      }
    }
    b.nxt_[prev] = (int16_t)p;
    b.gsize_[p] = (int16_t)size;
    b.recount_libs(p);
  }
  if (meta8) {
    b.current_player_ = meta8[0];
    b.ko_ = meta8[1];
    b.last1_ = meta8[2];
    b.last2_ = meta8[3];
    b.passes_black_ = meta8[4];
    b.passes_white_ = meta8[5];
    b.nmoves_ = meta8[6];
    b.end_of_game_ = meta8[7] != 0;
  }
  return b;
}

void Board::push_history(int a) {
  nmoves_++;
  last2_ = last1_;
  last1_ = a;
  if (light_) return;
  if (history_.use_count() > 1) history_ = std::make_shared<std::vector<int16_t>>(*history_);
  history_->push_back((int16_t)a);
}

void Board::push_hash(uint64_t h) {
  if (light_) return;
  if (prev_hashes_.use_count() > 1)
    prev_hashes_ = std::make_shared<std::vector<uint64_t>>(*prev_hashes_);
  prev_hashes_->push_back(h);
}

// ------------------------------------------------------------------ group helpers
void Board::group_stones(int p, std::vector<int>& out) const {
  out.clear();
  if (head_[p] < 0) return;
  int s = p;
  do {
    out.push_back(s);
    s = nxt_[s];
  } while (s != p);
}

void Board::liberty_set(int p, Bitset& out) const {
  out.clear(W_);
  if (head_[p] < 0) {
    // reference liberty_sets semantics for an empty point: its empty neighbours
    for (int i = 0; i < g_->nnbr[p]; ++i) {
      int n = g_->nbr[p][i];
      if (color_[n] == EMPTY) out.set(n);
    }
    return;
  }
  int s = p;
  do {
    for (int i = 0; i < g_->nnbr[s]; ++i) {
      int n = g_->nbr[s][i];
      if (color_[n] == EMPTY) out.set(n);
    }
    s = nxt_[s];
  } while (s != p);
}

void Board::recount_libs(int h) {
  Bitset b;
  liberty_set(h, b);
  libcnt_[h] = (int16_t)b.count(W_);
}

int Board::groups_around(int p, int* heads) const {
  int n = 0;
  for (int i = 0; i < g_->nnbr[p]; ++i) {
    int q = g_->nbr[p][i];
    int h = head_[q];
    if (h < 0) continue;
    bool seen = false;
    for (int j = 0; j < n; ++j) seen |= (heads[j] == h);
    if (!seen) heads[n++] = h;
  }
  return n;
}

void Board::remove_group(int h, int col) {
  // first pass: clear stones + hash  (go.py:163-168)
  int stones[MAXP];
  int ns = 0;
  int s = h;
  do {
    stones[ns++] = s;
    s = nxt_[s];
  } while (s != h);
  const uint64_t* z = (col == WHITE) ? zob_->white.data() : zob_->black.data();
  for (int i = 0; i < ns; ++i) {
    hash_ ^= z[stones[i]];
    color_[stones[i]] = EMPTY;
  }
  // second pass: each removed point becomes a liberty of every distinct adjacent group
  for (int i = 0; i < ns; ++i) {
    int r = stones[i];
    head_[r] = -1;
    nxt_[r] = -1;
    int seen[4];
    int k = 0;
    for (int j = 0; j < g_->nnbr[r]; ++j) {
      int n = g_->nbr[r][j];
      int hn = head_[n];
      if (hn < 0) continue;
      bool dup = false;
      for (int t = 0; t < k; ++t) dup |= (seen[t] == hn);
      if (dup) continue;
      seen[k++] = hn;
      libcnt_[hn]++;
    }
  }
}

void Board::place_stone(int p, int c) {
  color_[p] = (int8_t)c;
  hash_ ^= (c == WHITE ? zob_->white[p] : zob_->black[p]);
  placed_[p] = clock_;
  int fh[4], eh[4];
  int nf = 0, ne = 0;
  for (int i = 0; i < g_->nnbr[p]; ++i) {
    int n = g_->nbr[p][i];
    int h = head_[n];
    if (h < 0) continue;
    if (color_[n] == c) {
      bool dup = false;
      for (int t = 0; t < nf; ++t) dup |= (fh[t] == h);
      if (!dup) fh[nf++] = h;
    } else {
      bool dup = false;
      for (int t = 0; t < ne; ++t) dup |= (eh[t] == h);
      if (!dup) eh[ne++] = h;
    }
  }
  for (int t = 0; t < ne; ++t) libcnt_[eh[t]]--;
  if (nf == 0) {
    head_[p] = (int16_t)p;
    nxt_[p] = (int16_t)p;
    gsize_[p] = 1;
    int lc = 0;
    for (int i = 0; i < g_->nnbr[p]; ++i) lc += (color_[g_->nbr[p][i]] == EMPTY);
    libcnt_[p] = (int16_t)lc;
  } else {
    int tgt = fh[0];
    for (int t = 1; t < nf; ++t)
      if (gsize_[fh[t]] > gsize_[tgt]) tgt = fh[t];
    head_[p] = (int16_t)tgt;
    nxt_[p] = nxt_[tgt];
    nxt_[tgt] = (int16_t)p;
    gsize_[tgt]++;
    for (int t = 0; t < nf; ++t) {
      int h = fh[t];
      if (h == tgt) continue;
      int s = h;
      do {
        head_[s] = (int16_t)tgt;
        s = nxt_[s];
      } while (s != h);
      std::swap(nxt_[tgt], nxt_[h]);
      gsize_[tgt] += gsize_[h];
    }
    recount_libs(tgt);
  }
  // captures, in neighbour order (go.py:543-561)
  for (int i = 0; i < g_->nnbr[p]; ++i) {
    int n = g_->nbr[p][i];
    if (color_[n] != -c) continue;
    int h = head_[n];
    if (libcnt_[h] != 0) continue;
    int num = gsize_[h];
    remove_group(h, -c);
    if (c == BLACK)
      white_prisoners_ += num;
    else
      black_prisoners_ += num;
    if (num == 1) {
      int hp = head_[p];
      if (libcnt_[hp] == 1 && gsize_[hp] == 1) ko_ = n;
    }
  }
}

// ------------------------------------------------------------------ legality (go.py:219-285)
bool Board::is_suicide(int a) const {
  int empty_nbrs = 0;
  for (int i = 0; i < g_->nnbr[a]; ++i) empty_nbrs += (color_[g_->nbr[a][i]] == EMPTY);
  if (empty_nbrs > 0) return false;
  for (int i = 0; i < g_->nnbr[a]; ++i) {
    int n = g_->nbr[a][i];
    int h = head_[n];
    if (h < 0) continue;
    bool other_libs = libcnt_[h] > 1;  // a is one of its liberties
    if (color_[n] == current_player_ && other_libs) return false;
    if (color_[n] == -current_player_ && !other_libs) return false;
  }
  return true;
}

bool Board::is_positional_superko(int a) const {
  const std::vector<int16_t>& hist = *history_;
  int start;
  bool has_h = !handicaps_.empty();
  if (!has_h && current_player_ == BLACK)
    start = 0;
  else if (has_h && current_player_ == WHITE)
    start = 0;
  else
    start = 1;
  bool seen = std::find(handicaps_.begin(), handicaps_.end(), (int16_t)a) != handicaps_.end();
  for (size_t i = start; !seen && i < hist.size(); i += 2) seen = (hist[i] == a);
  if (!seen) return false;
  Board tmp(*this);
  tmp.enforce_superko_ = false;
  tmp.light_ = true;
  tmp.do_move(a, 0);
  const std::vector<uint64_t>& ph = *prev_hashes_;
  return std::find(ph.begin(), ph.end(), tmp.hash_) != ph.end();
}

bool Board::is_legal(int a) const {
  if (a == PASS) return true;
  if (a < 0 || a >= P_) return false;
  if (color_[a] != EMPTY) return false;
  if (is_suicide(a)) return false;
  if (a == ko_) return false;
  if (enforce_superko_ && is_positional_superko(a)) return false;
  return true;
}

// ------------------------------------------------------------------ eyes (go.py:287-327)
bool Board::is_eyeish(int p, int owner) const {
  if (color_[p] != EMPTY) return false;
  for (int i = 0; i < g_->nnbr[p]; ++i)
    if (color_[g_->nbr[p][i]] != owner) return false;
  return true;
}

// The rule's result does not depend on the order of the diagonals (the recursion restores its
// stack), so the opponent stones are counted first, and a point stops recursing as soon as its
// bad count exceeds the allowance or its remaining empty diagonals could not push it over.
bool Board::is_eye_stack(int p, int owner, std::vector<int>& stack) const {
  if (!is_eyeish(p, owner)) return false;
  const int allow = (g_->nnbr[p] == 4) ? 1 : 0;
  int num_bad = 0, rem = 0;
  int cand[4];
  for (int i = 0; i < g_->ndiag[p]; ++i) {
    const int d = g_->diag[p][i];
    if (color_[d] == -owner) {
      num_bad++;
    } else if (color_[d] == EMPTY && std::find(stack.begin(), stack.end(), d) == stack.end()) {
      cand[rem++] = d;
    }
  }
  if (num_bad > allow) return false;
  for (int i = 0; i < rem; ++i) {
    if (num_bad + (rem - i) <= allow) return true;
    stack.push_back(p);
    if (!is_eye_stack(cand[i], owner, stack)) num_bad++;
    stack.pop_back();
    if (num_bad > allow) return false;
  }
  return true;
}

bool Board::is_eye(int p, int owner) const {
  std::vector<int> stack;
  stack.reserve(16);
  return is_eye_stack(p, owner, stack);
}

// ------------------------------------------------------------------ ladders (go.py:329-463)
bool Board::is_ladder_capture(int a, int prey, int remaining) const {
  if (!is_legal(a)) return false;
  if (remaining <= 0) return true;
  const int hunter = current_player_;
  const int prey_player = -hunter;
  int cand[4];
  int nc = 0;
  if (prey < 0) {
    int heads[4];
    int nh = groups_around(a, heads);
    for (int i = 0; i < nh; ++i)
      if (color_[heads[i]] == prey_player && libcnt_[heads[i]] == 2) cand[nc++] = heads[i];
  } else {
    cand[nc++] = prey;
  }
  for (int c = 0; c < nc; ++c) {
    const int pr = cand[c];
    Board tmp(*this);
    if (!enforce_superko_) tmp.light_ = true;
    tmp.do_move(a, 0);
    Bitset esc;
    tmp.liberty_set(pr, esc);
    if (tmp.head_[pr] >= 0) {
      int s = pr;
      do {
        for (int i = 0; i < g_->nnbr[s]; ++i) {
          int n = g_->nbr[s][i];
          if (tmp.color_[n] == hunter && tmp.libcnt_[tmp.head_[n]] == 1) {
            Bitset l;
            tmp.liberty_set(n, l);
            esc.or_with(l, W_);
          }
        }
        s = tmp.nxt_[s];
      } while (s != pr);
    }
    bool any_escape = false;
    for (int k = 0; k < W_ && !any_escape; ++k) {
      uint64_t x = esc.w[k];
      while (x && !any_escape) {
        int e = k * 64 + __builtin_ctzll(x);
        x &= x - 1;
        if (tmp.is_ladder_escape(e, pr, remaining - 1)) any_escape = true;
      }
    }
    if (!any_escape) return true;
  }
  return false;
}

bool Board::is_ladder_escape(int a, int prey, int remaining) const {
  if (!is_legal(a)) return false;
  if (remaining <= 0) return false;
  const int prey_player = current_player_;
  int cand[4];
  int nc = 0;
  if (prey < 0) {
    int heads[4];
    int nh = groups_around(a, heads);
    for (int i = 0; i < nh; ++i)
      if (color_[heads[i]] == prey_player && libcnt_[heads[i]] == 1) cand[nc++] = heads[i];
  } else {
    cand[nc++] = prey;
  }
  for (int c = 0; c < nc; ++c) {
    const int pr = cand[c];
    Board tmp(*this);
    if (!enforce_superko_) tmp.light_ = true;
    tmp.do_move(a, 0);
    int lc = tmp.liberty_count(pr);
    if (lc >= 3) return true;
    if (lc == 1) continue;
    Bitset libs;
    tmp.liberty_set(pr, libs);
    bool captured = false;
    for (int k = 0; k < W_ && !captured; ++k) {
      uint64_t x = libs.w[k];
      while (x && !captured) {
        int q = k * 64 + __builtin_ctzll(x);
        x &= x - 1;
        if (tmp.is_ladder_capture(q, pr, remaining - 1)) captured = true;
      }
    }
    if (captured) continue;
    return true;
  }
  return false;
}

// ------------------------------------------------------------------ moves / scoring
void Board::legal_moves(std::vector<int>& non_eye, std::vector<int>& eyes) const {
  non_eye.clear();
  eyes.clear();
  for (int p = 0; p < P_; ++p) {
    if (!is_legal(p)) continue;
    if (!is_eye(p, current_player_))
      non_eye.push_back(p);
    else
      eyes.push_back(p);
  }
}

void Board::score(double& black, double& white) const {
  int sb = 0, sw = 0;
  for (int p = 0; p < P_; ++p) {
    if (color_[p] == BLACK)
      sb++;
    else if (color_[p] == WHITE)
      sw++;
    else if (is_eyeish(p, BLACK))
      sb++;
    else if (is_eyeish(p, WHITE))
      sw++;
  }
  white = sw + komi_ - passes_white_;
  black = sb - passes_black_;
}

int Board::get_winner() const {
  double b, w;
  score(b, w);
  if (b > w) return BLACK;
  if (w > b) return WHITE;
  return 0;
}

void Board::place_handicaps(const std::vector<int>& actions) {
  if (nmoves_ > 0) throw IllegalMoveError("Cannot place handicap on a started game");
  for (int a : actions) handicaps_.push_back((int16_t)a);
  for (int a : actions) do_move(a, BLACK);
  clear_history();
  nmoves_ = 0;
  last1_ = last2_ = -2;
}

bool Board::do_move(int a, int color) {
  const int c = color ? color : current_player_;
  const int reset = current_player_;
  current_player_ = c;
  if (!is_legal(a)) {
    current_player_ = reset;
    if (a == PASS) throw IllegalMoveError("None");
    throw IllegalMoveError("(" + std::to_string(a / S_) + ", " + std::to_string(a % S_) + ")");
  }
  ko_ = -1;
  clock_++;
  if (a != PASS) {
    place_stone(a, c);
    push_hash(hash_);
  } else {
    if (c == BLACK) passes_black_++;
    if (c == WHITE) passes_white_++;
  }
  current_player_ = -c;
  push_history(a);
  if (nmoves_ > 1 && last1_ == PASS && last2_ == PASS && current_player_ == WHITE)
    end_of_game_ = true;
  return end_of_game_;
}

void Board::play_unchecked(int a) {
  const int c = current_player_;
  ko_ = -1;
  clock_++;
  if (a != PASS) {
    place_stone(a, c);
    push_hash(hash_);
  } else {
    if (c == BLACK) passes_black_++;
    if (c == WHITE) passes_white_++;
  }
  current_player_ = -c;
  push_history(a);
  if (nmoves_ > 1 && last1_ == PASS && last2_ == PASS && current_player_ == WHITE)
    end_of_game_ = true;
}

}  // namespace rag

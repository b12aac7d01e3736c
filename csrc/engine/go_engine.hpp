// Native Go rules engine (C++17, CPU).
//
// Behavioural contract: AlphaGo/go.py of the reference (GameState, go.py:9-581). Every rule
// detail that the reference's tests or feature planes observe is reproduced exactly:
//   * neighbour order (x-1,y),(x+1,y),(x,y-1),(x,y+1)            go.py:103-116
//   * capture loop order + the "ko only for 1-stone capture whose
//     capturing stone is a lone stone left with 1 liberty" rule   go.py:543-561  (quirk Q15)
//   * end of game = two passes AND current_player == WHITE after   go.py:576-581  (quirk Q3)
//   * positional superko evaluated only for moves already in the
//     mover's own history or the handicap list                    go.py:242-265  (quirk Q11)
//   * area scoring counting only single-point eyeish empties       go.py:482-506  (quirk Q12)
//   * recursive true-eye rule with an ancestor stack               go.py:298-327
//   * ladder reading (mutual recursion, remaining_attempts=80)     go.py:329-463
//
// Representation (designed for cheap copies in ladder reading / MCTS, not a translation of the
// reference's shared python sets): flat per-point arrays over idx = x*S + y, groups as circular
// linked lists with a head index, liberty *counts* per head maintained incrementally and exact
// liberty *sets* recomputed on demand by walking a group into a bitset. A full state copy is
// ~4 KB of memcpy plus two copy-on-write vectors (history / previous hashes).
#pragma once
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

namespace rag {

constexpr int EMPTY = 0;
constexpr int BLACK = 1;
constexpr int WHITE = -1;
constexpr int PASS = -1;       // flat index of the pass move
constexpr int MAXS = 25;       // largest supported board edge
constexpr int MAXP = MAXS * MAXS;
constexpr int MAXW = (MAXP + 63) / 64;

struct IllegalMoveError : public std::runtime_error {
  explicit IllegalMoveError(const std::string& s) : std::runtime_error(s) {}
};

// Immutable per-size neighbour tables (reference: the class-level neighbour cache, go.py:15,103-116).
struct Geometry {
  int S = 0, P = 0, W = 0;
  int16_t nbr[MAXP][4];
  int8_t nnbr[MAXP];
  int16_t diag[MAXP][4];  // reference order: (x-1,y-1),(x+1,y+1),(x+1,y-1),(x-1,y+1)  go.py:118-123
  int8_t ndiag[MAXP];
  static const Geometry* get(int S);
};

struct Zobrist {
  std::vector<uint64_t> white, black;  // P entries each, idx = x*S+y
};

struct Bitset {
  uint64_t w[MAXW];
  void clear(int W) { std::memset(w, 0, sizeof(uint64_t) * W); }
  void set(int i) { w[i >> 6] |= (1ull << (i & 63)); }
  void reset(int i) { w[i >> 6] &= ~(1ull << (i & 63)); }
  bool test(int i) const { return (w[i >> 6] >> (i & 63)) & 1ull; }
  int count(int W) const {
    int c = 0;
    for (int k = 0; k < W; ++k) c += __builtin_popcountll(w[k]);
    return c;
  }
  void or_with(const Bitset& o, int W) {
    for (int k = 0; k < W; ++k) w[k] |= o.w[k];
  }
  template <class F>
  void for_each(int W, F&& f) const {
    for (int k = 0; k < W; ++k) {
      uint64_t x = w[k];
      while (x) {
        int b = __builtin_ctzll(x);
        f(k * 64 + b);
        x &= x - 1;
      }
    }
  }
};

class Board {
 public:
  // ----- construction -----
  Board() = default;
  Board(int size, double komi, bool enforce_superko, std::shared_ptr<const Zobrist> zob);
  Board(const Board& o) { copy_from(o); }
  Board& operator=(const Board& o) {
    if (this != &o) copy_from(o);
    return *this;
  }
  void copy_from(const Board& o);
  // A light board (no history, superko off) rebuilt from the per-point arrays a search leaf is
  // shipped as (search/distributed.py): colours, stone ages (-1 = empty, may be null) and meta
  // = (player, ko, last move, second-to-last, black passes, white passes, moves, end of game).
  static Board from_arrays(int S, double komi, std::shared_ptr<const Zobrist> zob,
                           const int8_t* colors, const int16_t* ages, const int32_t* meta8);

  // ----- reference API (go.py) -----
  bool is_suicide(int a) const;
  bool is_positional_superko(int a) const;
  bool is_legal(int a) const;
  bool is_eyeish(int p, int owner) const;
  bool is_eye(int p, int owner) const;
  bool is_eye_stack(int p, int owner, std::vector<int>& stack) const;
  bool is_ladder_capture(int a, int prey, int remaining) const;
  bool is_ladder_escape(int a, int prey, int remaining) const;
  // legal moves in reference order (x-major); non-eye moves first, eye moves second
  void legal_moves(std::vector<int>& non_eye, std::vector<int>& eyes) const;
  int get_winner() const;
  void score(double& black, double& white) const;
  void place_handicaps(const std::vector<int>& actions);
  // returns is_end_of_game; throws IllegalMoveError
  bool do_move(int a, int color /*0 = current player*/);
  // no-throw fast path used by rollouts / search (assumes legality already established)
  void play_unchecked(int a);

  // ----- queries -----
  int size() const { return S_; }
  int npoints() const { return P_; }
  int color(int p) const { return color_[p]; }
  int group_head(int p) const { return head_[p]; }
  int group_size(int p) const { return head_[p] < 0 ? 0 : gsize_[head_[p]]; }
  int liberty_count(int p) const { return head_[p] < 0 ? -1 : libcnt_[head_[p]]; }
  int stone_age(int p) const { return head_[p] < 0 ? -1 : (int)(clock_ - placed_[p]); }
  // group stones of p (empty vector if empty)
  void group_stones(int p, std::vector<int>& out) const;
  // exact liberty set; for an EMPTY point: its empty neighbours (reference liberty_sets semantics)
  void liberty_set(int p, Bitset& out) const;
  // distinct neighbouring group heads in neighbour order  (go.py:82-99 get_groups_around)
  int groups_around(int p, int* heads) const;

  int current_player() const { return current_player_; }
  void set_current_player(int c) { current_player_ = c; }
  int ko() const { return ko_; }
  void set_ko(int k) { ko_ = k; }
  double komi() const { return komi_; }
  void set_komi(double k) { komi_ = k; }
  bool enforce_superko() const { return enforce_superko_; }
  void set_enforce_superko(bool e) { enforce_superko_ = e; }
  bool end_of_game() const { return end_of_game_; }
  void set_end_of_game(bool e) { end_of_game_ = e; }
  int black_prisoners() const { return black_prisoners_; }
  int white_prisoners() const { return white_prisoners_; }
  void set_prisoners(int b, int w) { black_prisoners_ = b; white_prisoners_ = w; }
  int passes_black() const { return passes_black_; }
  int passes_white() const { return passes_white_; }
  void set_passes(int b, int w) { passes_black_ = b; passes_white_ = w; }
  uint64_t hash() const { return hash_; }
  const std::vector<int16_t>& history() const { return *history_; }
  void clear_history() { history_ = std::make_shared<std::vector<int16_t>>(); }
  const std::vector<int16_t>& handicaps() const { return handicaps_; }
  const std::vector<uint64_t>& previous_hashes() const { return *prev_hashes_; }
  int move_count() const { return (int)history_->size(); }
  int last_move() const { return history_->empty() ? -2 : history_->back(); }
  // last two moves, also valid in light mode (-2 = none)
  int last1() const { return last1_; }
  int last2() const { return last2_; }
  int nmoves() const { return nmoves_; }
  const Zobrist& zobrist() const { return *zob_; }
  std::shared_ptr<const Zobrist> zobrist_ptr() const { return zob_; }
  const Geometry& geom() const { return *g_; }
  // Search copies skip history / previous-hash bookkeeping when superko is off (pure speed).
  void set_light(bool light) { light_ = light; }

 private:
  friend class LadderReader;
  void place_stone(int p, int c);
  void remove_group(int h, int c);
  void recount_libs(int h);
  void push_history(int a);
  void push_hash(uint64_t h);

  const Geometry* g_ = nullptr;
  std::shared_ptr<const Zobrist> zob_;
  int S_ = 0, P_ = 0, W_ = 0;
  int current_player_ = BLACK;
  int ko_ = -1;
  int black_prisoners_ = 0, white_prisoners_ = 0;
  int passes_black_ = 0, passes_white_ = 0;
  bool end_of_game_ = false;
  bool enforce_superko_ = false;
  bool light_ = false;
  int last1_ = -2, last2_ = -2;  // last two moves (works in light mode)
  int nmoves_ = 0;
  double komi_ = 7.5;
  uint64_t hash_ = 0;
  uint32_t clock_ = 0;
  std::shared_ptr<std::vector<int16_t>> history_;
  std::shared_ptr<std::vector<uint64_t>> prev_hashes_;
  std::vector<int16_t> handicaps_;
  int8_t color_[MAXP];
  int16_t head_[MAXP];
  int16_t nxt_[MAXP];
  int16_t gsize_[MAXP];
  int16_t libcnt_[MAXP];
  uint32_t placed_[MAXP];
};

// ------------------------------------------------------------------ ladders without copies
// The reference's ladder reading (go.py:329-463) on one working copy of a board: moves are
// played in place and taken back from a write journal (ladder.cpp). Results are identical to
// Board::is_ladder_capture / is_ladder_escape for boards that do not enforce superko.
class LadderReader {
 public:
  void reset(const Board& b);
  bool capture(int a, int prey, int remaining);
  bool escape(int a, int prey, int remaining);

 private:
  struct E8 {
    int8_t* p;
    int8_t old;
  };
  struct E16 {
    int16_t* p;
    int16_t old;
  };
  struct Frame {
    uint32_t n8, n16;
    int ko, player;
  };
  void set8(int8_t& r, int8_t v) {
    j8_.push_back(E8{&r, r});
    r = v;
  }
  void set16(int16_t& r, int16_t v) {
    j16_.push_back(E16{&r, r});
    r = v;
  }
  void play(int a);
  void undo();
  bool legal(int a) const;
  Board b_;
  std::vector<E8> j8_;
  std::vector<E16> j16_;
  std::vector<Frame> frames_;
};

// Both ladder planes (capture, escape; P bytes each) of one position; `reader` (optional) is a
// reusable working board.
void ladder_planes(const Board& b, uint8_t* cap, uint8_t* esc, LadderReader* reader = nullptr);

// ------------------------------------------------------------------ features (preprocessing.py)
// Feature ids; order matches the registry of the reference (preprocessing.py:209-258) plus
// "color" (value-net 49th plane).
enum FeatureId : int {
  F_BOARD = 0, F_ONES, F_TURNS_SINCE, F_LIBERTIES, F_CAPTURE_SIZE, F_SELF_ATARI_SIZE,
  F_LIBERTIES_AFTER, F_LADDER_CAPTURE, F_LADDER_ESCAPE, F_SENSIBLENESS, F_ZEROS, F_LEGAL, F_COLOR,
  F_COUNT
};
int feature_planes(int fid);
// Writes sum(planes) x S x S uint8 planes, layout [plane][x][y].
void extract_features(const Board& b, const int* fids, int nf, uint8_t* out);

}  // namespace rag

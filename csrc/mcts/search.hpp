// Native APV-MCTS core (the reference's ParallelMCTS is an empty stub,
// AlphaGo/mcts.py:219-220, and its sequential MCTS is AlphaGo/mcts.py:79-216).
//
// Asynchronous policy-and-value MCTS in the AlphaGo style, restructured for a GPU evaluator:
// the search advances in *waves*. select(B) descends the tree B times with virtual loss, so the
// descents spread over different leaves, and returns a wave id. For every wave
//   * the policy / value networks evaluate all its leaves in one batched GPU pass, and
//     backup_value() expands the leaves with the network priors and backs up the value-net
//     statistics (N_v, W_v) at once;
//   * the fast-rollout playouts of the same leaves run asynchronously — on the GPU rollout kernel
//     (several waves in flight) or on a native thread pool — and backup_rollout() later adds the
//     rollout statistics (N_r, W_r) and removes the wave's virtual losses.
// As in AlphaGo, the two estimates are kept apart and mixed at selection time:
//   Q(s,a) = (1 - lambda) W_v/N_v + lambda W_r/N_r
//   a      = argmax  Q(s,a) + c_puct P(s,a) sqrt(N(s)) / (1 + N(s,a))
// with n_vl virtual losses per in-flight descent (counted as rollout losses when rollouts are
// used, value losses otherwise). Values are from the perspective of the player to move at the
// leaf; a node stores them for the player who played its move (negamax signs on backup).
//
// Children are created for the leaf's sensible moves (legal, not an own true eye — the set the
// players use) with priors renormalised over them; PASS is the only child when no sensible move
// exists. Terminal leaves (end of game) are scored exactly and backed up at once.
#pragma once

#include <algorithm>
#include <cstring>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <tuple>
#include <vector>

#include <sys/mman.h>

#include "../engine/go_engine.hpp"
#include "../engine/thread_pool.hpp"
#include "rollout.hpp"

namespace rag {

namespace mcts_detail {

enum : uint8_t { N_NEW = 0, N_PENDING = 1, N_EXPANDED = 2 };

struct Node {
  int32_t parent;
  int32_t first;   // first child (children are contiguous)
  int16_t nchild;
  int16_t move;    // flat index, PASS = -1
  float prior;
  int32_t n;       // value-net visits (every completed evaluation)
  int32_t nr;      // rollouts
  int32_t vl;      // in-flight descents through this node
  float w;         // value-net sum, for the player who played `move`
  float wr;        // rollout sum, same perspective
  uint8_t state;
};

// Node storage: one anonymous mapping reserved up front (virtual until written, transparent
// huge pages requested), so the tree never moves while it grows, and resize() leaves the new
// slots uninitialised (backup_value fills them in parallel). A std::vector would zero-fill new
// slots serially and copy the whole tree on every doubling.
class NodeArena {
 public:
  NodeArena() = default;
  ~NodeArena() { unmap(p_, cap_); }
  NodeArena(const NodeArena&) = delete;
  NodeArena& operator=(const NodeArena&) = delete;
  void reserve(size_t cap) {
    if (cap > cap_) grow(cap);
  }
  size_t size() const { return n_; }
  size_t capacity() const { return cap_; }
  Node& operator[](size_t i) { return p_[i]; }
  const Node& operator[](size_t i) const { return p_[i]; }
  void clear() { n_ = 0; }
  void push_back(const Node& x) {
    if (n_ == cap_) grow(cap_ ? 2 * cap_ : (size_t)1 << 16);
    p_[n_++] = x;
  }
  void resize(size_t n) {
    if (n > cap_) grow(std::max(n, 2 * cap_));
    n_ = n;
  }
  void swap(NodeArena& o) {
    std::swap(p_, o.p_);
    std::swap(n_, o.n_);
    std::swap(cap_, o.cap_);
  }

 private:
  static void unmap(Node* p, size_t cap) {
    if (p) munmap(p, cap * sizeof(Node));
  }
  void grow(size_t cap) {
    void* m = mmap(nullptr, cap * sizeof(Node), PROT_READ | PROT_WRITE,
                   MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) throw std::bad_alloc();
    madvise(m, cap * sizeof(Node), MADV_HUGEPAGE);
    if (n_) std::memcpy(m, p_, n_ * sizeof(Node));
    unmap(p_, cap_);
    p_ = static_cast<Node*>(m);
    cap_ = cap;
  }
  Node* p_ = nullptr;
  size_t n_ = 0, cap_ = 0;
};

struct Leaf {
  Board board;
  std::vector<int32_t> path;  // root .. leaf
  float z = 0.f;
};

struct Wave {
  std::vector<Leaf> leaves;
  bool value_done = false;
  std::thread worker;  // CPU rollouts
  bool rolling = false;
};

using rag::Pool;

}  // namespace mcts_detail

using mcts_detail::Leaf;
using mcts_detail::Node;
using mcts_detail::NodeArena;
using mcts_detail::Wave;
using mcts_detail::N_EXPANDED;
using mcts_detail::N_NEW;
using mcts_detail::N_PENDING;

// Node pool capacity reserved up front: growth by reallocation copies the whole tree (tens of
// MB per doubling) inside backup_value; the reservation is virtual until nodes are written.
constexpr size_t kNodeReserve = size_t(1) << 23;

class Search {
 public:
  float c_puct = 5.f, lambda = 0.5f;
  int n_vl = 3, rollout_limit = 500, max_depth = 722;
  // networks with a pass logit: priors rows carry S*S + 1 entries and every
  // expanded node also gets a PASS child with the network's pass prior
  bool pass_prior = false;
  uint64_t seed = 1;
  std::shared_ptr<RolloutPolicy> rollout_policy;

  explicit Search(const Board& root, int nthreads = 8)
      : rollout_policy(std::make_shared<RolloutPolicy>()), pool_(std::max(nthreads, 1)) {
    reset(root);
  }
  ~Search() { drop_waves(); }
  Search(const Search&) = delete;
  Search& operator=(const Search&) = delete;

  void reset(const Board& root) {
    drop_waves();
    root_board_ = root;
    nodes_.clear();
    nodes_.reserve(kNodeReserve);
    nodes_.push_back(Node{-1, -1, 0, (int16_t)PASS, 1.f, 0, 0, 0, 0.f, 0.f, N_NEW});
    root_ = 0;
  }

  const Board& root_board() const { return root_board_; }
  int nthreads() const { return pool_.size(); }

  // ------------------------------------------------------------------ selection
  // vl and state are changed by concurrent descents (descend_parallel): read them atomically
  static int32_t vl_of(const Node& c) { return __atomic_load_n(&c.vl, __ATOMIC_RELAXED); }
  static uint8_t state_of(const Node& c) { return __atomic_load_n(&c.state, __ATOMIC_RELAXED); }

  float child_score(const Node& c, float sq) const {
    const float vl = (float)(vl_of(c) * n_vl);
    const bool use_r = lambda > 0.f;
    const bool use_v = lambda < 1.f;
    float q = 0.f;
    if (use_r && use_v) {
      const float qv = c.n > 0 ? c.w / c.n : 0.f;
      const float den = c.nr + vl;
      const float qr = den > 0.f ? (c.wr - vl) / den : qv;
      q = (1.f - lambda) * qv + lambda * qr;
    } else if (use_r) {
      const float den = c.nr + vl;
      q = den > 0.f ? (c.wr - vl) / den : 0.f;
    } else {
      const float den = c.n + vl;
      q = den > 0.f ? (c.w - vl) / den : 0.f;
    }
    return q + c_puct * c.prior * sq / (1.f + (float)c.n + vl);
  }

  int select_child(int p) const {
    const Node& pn = nodes_[p];
    const float np = (float)(pn.n + vl_of(pn) * n_vl);
    const float sq = std::sqrt(std::max(np, 1.f));
    int best = pn.first;
    float bv = -1e30f;
    for (int k = 0; k < pn.nchild; ++k) {
      const float v = child_score(nodes_[pn.first + k], sq);
      if (v > bv) {
        bv = v;
        best = pn.first + k;
      }
    }
    return best;
  }

  // Returns (wave id, number of leaves); id -1 when nothing was selected.
  //
  // Three phases: (1) tree walks with virtual loss (descend(); on the pool for B >=
  // parallel_select_min, see descend_parallel); (2) the leaf boards (root copy + the path's moves) are built
  // in parallel on the pool; (3) descents that ended on a terminal position are scored on their
  // board and backed up at once (their virtual loss, taken in phase 1 so that later walks of the
  // same wave avoid them, is dropped again).
  std::pair<int, int> select(int B) {
    collisions_ = 0;
    std::vector<std::vector<int32_t>> paths;
    std::vector<uint8_t> term;
    paths.reserve(B);
    term.reserve(B);
    if (B >= parallel_select_min && pool_.size() > 1) {
      descend_parallel(B, paths, term);
    } else {
      int attempts = 0, claimed = 0;
      while (claimed < B && attempts < 4 * B) {
        ++attempts;
        std::vector<int32_t> path;
        bool terminal = false;
        if (!descend(path, terminal, false)) {
          ++collisions_;
          continue;
        }
        if (!terminal) ++claimed;
        paths.push_back(std::move(path));
        term.push_back(terminal ? 1 : 0);
      }
    }
    const Board& rb = root_board_;
    const int nd = (int)paths.size();
    int nleaf = 0;
    for (int i = 0; i < nd; ++i) nleaf += term[i] ? 0 : 1;
    // leaf boards go straight into a recycled wave (its Leaf storage is reused: no fresh pages);
    // terminal descents get a scratch board
    std::unique_ptr<Wave> wave = take_wave();
    wave->leaves.resize(nleaf);
    std::vector<int> slot(nd);
    int nt = 0, nl = 0;
    for (int i = 0; i < nd; ++i) slot[i] = term[i] ? nt++ : nl++;
    std::vector<Board> tboards(nt);
    const bool light = !rb.enforce_superko();
    pool_.run(nd, [&](int i) {
      Board& b = term[i] ? tboards[slot[i]] : wave->leaves[slot[i]].board;
      b = rb;
      b.set_light(light);
      const std::vector<int32_t>& path = paths[i];
      for (size_t d = 1; d < path.size(); ++d) b.play_unchecked(nodes_[path[d]].move);
      if (!term[i]) {
        Leaf& L = wave->leaves[slot[i]];
        L.path.swap(paths[i]);
        L.z = 0.f;
      }
    });
    for (int i = 0; i < nd; ++i) {
      if (!term[i]) continue;
      const Board& b = tboards[slot[i]];
      const int win = b.get_winner();
      const float v = win == 0 ? 0.f : (win == b.current_player() ? 1.f : -1.f);
      backup_value_path(paths[i], v, true);
      if (lambda > 0.f) backup_rollout_path(paths[i], v, false);
      ++terminal_;
    }
    const int n = (int)wave->leaves.size();
    if (n == 0) {
      recycle(std::move(wave));
      return {-1, 0};
    }
    const int id = next_wave_++;
    waves_[id] = std::move(wave);
    return {id, n};
  }

  // Descents of one wave in parallel on the pool (AlphaGo's asynchronous search threads):
  // virtual loss is taken on every node of a path as the walk passes it (atomic adds), so
  // concurrent walks spread over the tree; a leaf is claimed by one N_NEW -> N_PENDING
  // compare-and-swap, a walk that loses it (or arrives after B leaves are claimed) gives its
  // virtual loss back and is counted as a collision. Which leaves a wave gets then depends on
  // thread timing; select(B) with B < parallel_select_min (or one thread) is the serial,
  // deterministic walk.
  int parallel_select_min = 64;

  void descend_parallel(int B, std::vector<std::vector<int32_t>>& paths,
                        std::vector<uint8_t>& term) {
    std::atomic<int> nleaf{0}, attempts{0}, coll{0};
    std::mutex mu;
    const int nw = pool_.size();
    pool_.run(nw, [&](int) {
      std::vector<std::vector<int32_t>> mine;
      std::vector<uint8_t> mterm;
      while (nleaf.load(std::memory_order_relaxed) < B &&
             attempts.fetch_add(1, std::memory_order_relaxed) < 4 * B) {
        std::vector<int32_t> path;
        bool terminal = false;
        if (!descend(path, terminal, true)) {
          coll.fetch_add(1, std::memory_order_relaxed);
          continue;
        }
        if (!terminal && nleaf.fetch_add(1) >= B) {  // over-claimed: hand the leaf back
          __atomic_store_n(&nodes_[path.back()].state, (uint8_t)N_NEW, __ATOMIC_RELAXED);
          for (int id : path) __atomic_fetch_sub(&nodes_[id].vl, 1, __ATOMIC_RELAXED);
          break;
        }
        mine.push_back(std::move(path));
        mterm.push_back(terminal ? 1 : 0);
      }
      std::lock_guard<std::mutex> g(mu);
      for (size_t k = 0; k < mine.size(); ++k) {
        paths.push_back(std::move(mine[k]));
        term.push_back(mterm[k]);
      }
    });
    collisions_ = coll.load();
  }

  // One walk from the root with virtual loss. Tracks only what the walk needs (player to move,
  // the last two moves and the move count decide the end of the game, exactly as
  // Board::play_unchecked does). Returns false (virtual loss already given back) when the walk
  // ends on a leaf that another descent is waiting for; terminal = end of game / depth limit /
  // a node without children (its virtual loss stays until its immediate backup).
  bool descend(std::vector<int32_t>& path, bool& terminal, bool concurrent) {
    const Board& rb = root_board_;
    path.clear();
    path.reserve(32);
    int node = root_;
    path.push_back(node);
    if (concurrent) __atomic_fetch_add(&nodes_[node].vl, 1, __ATOMIC_RELAXED);
    int depth = 0;
    int ptm = rb.current_player(), l1 = rb.last1(), l2 = rb.last2(), nm = rb.nmoves();
    bool end = rb.end_of_game();
    while (state_of(nodes_[node]) == N_EXPANDED && nodes_[node].nchild > 0 && !end &&
           depth < max_depth) {
      node = select_child(node);
      path.push_back(node);
      if (concurrent) __atomic_fetch_add(&nodes_[node].vl, 1, __ATOMIC_RELAXED);
      ++depth;
      ++nm;
      l2 = l1;
      l1 = nodes_[node].move;
      ptm = -ptm;
      if (nm > 1 && l1 == PASS && l2 == PASS && ptm == WHITE) end = true;
    }
    Node& leaf = nodes_[node];
    terminal = end || depth >= max_depth || (state_of(leaf) == N_EXPANDED && leaf.nchild == 0);
    if (!terminal) {
      bool claimed;
      if (concurrent) {
        uint8_t expect = N_NEW;
        claimed = __atomic_compare_exchange_n(&leaf.state, &expect, (uint8_t)N_PENDING, false,
                                              __ATOMIC_RELAXED, __ATOMIC_RELAXED);
      } else {
        claimed = leaf.state != N_PENDING;
        if (claimed) leaf.state = N_PENDING;
      }
      if (!claimed) {  // already waiting for its evaluation
        if (concurrent)
          for (int id : path) __atomic_fetch_sub(&nodes_[id].vl, 1, __ATOMIC_RELAXED);
        return false;
      }
    }
    if (!concurrent)
      for (int id : path) nodes_[id].vl += 1;
    return true;
  }

  Wave& wave(int id) {
    auto it = waves_.find(id);
    if (it == waves_.end()) throw std::invalid_argument("unknown or finished wave");
    return *it->second;
  }
  int num_leaves(int id) { return (int)wave(id).leaves.size(); }
  std::vector<const Board*> leaf_boards(int id) {
    std::vector<const Board*> v;
    for (auto& L : wave(id).leaves) v.push_back(&L.board);
    return v;
  }

  // ------------------------------------------------------------------ value backup
  // priors: [n][stride] network move probabilities (nullptr => uniform); values: [n] (nullptr
  // => value statistics untouched: rollouts only).
  // sensible: optional [n][P] mask of the leaves' sensible moves (legal, not an own true eye),
  // e.g. the sensibleness plane the GPU feature kernel already produced; otherwise the moves
  // are generated natively on the pool.
  void backup_value(int id, const float* priors, int stride, const float* values,
                    const uint8_t* sensible = nullptr) {
    Wave& wv = wave(id);
    if (wv.value_done) throw std::runtime_error("value backup twice");
    const int n = (int)wv.leaves.size();
    const int P = root_board_.npoints();
    // pass 1 (parallel): children per leaf still to expand — the sensible-move mask's count, or
    // natively generated moves; then one contiguous block for all of them (the leaves of one
    // wave are distinct nodes: select() skips pending ones, so the blocks never overlap)
    std::vector<int32_t> cnt(n, -1);
    std::vector<std::vector<int>> moves(sensible ? 0 : n);
    pool_.run(n, [&](int i) {
      const Leaf& L = wv.leaves[i];
      if (nodes_[L.path.back()].state == N_EXPANDED) return;
      int c = 0;
      if (sensible) {
        const uint8_t* m = sensible + (size_t)i * P;
        for (int p = 0; p < P; ++p) c += m[p] != 0;
      } else {
        std::vector<int> eyes;
        L.board.legal_moves(moves[i], eyes);
        c = (int)moves[i].size();
      }
      cnt[i] = c;
    });
    const bool with_pass = pass_prior && priors != nullptr && stride > P;
    std::vector<int32_t> first(n, -1);
    size_t total = nodes_.size();
    for (int i = 0; i < n; ++i) {
      if (cnt[i] < 0) continue;
      first[i] = (int32_t)total;
      total += nchildren(cnt[i], with_pass);
    }
    nodes_.resize(total);
    // pass 2 (parallel): write the children into their block
    pool_.run(n, [&](int i) {
      if (first[i] < 0) return;
      const int node = wv.leaves[i].path.back();
      const float* pri = priors ? priors + (size_t)i * stride : nullptr;
      if (sensible) {
        const uint8_t* m = sensible + (size_t)i * P;
        int k = 0;
        fill_children(node, first[i], cnt[i], with_pass, pri, P, [&]() {
          while (!m[k]) ++k;
          return k++;
        });
      } else {
        size_t k = 0;
        fill_children(node, first[i], cnt[i], with_pass, pri, P,
                      [&]() { return moves[i][k++]; });
      }
    });
    for (int i = 0; i < n; ++i) {
      Leaf& L = wv.leaves[i];
      if (first[i] >= 0) {
        Node& nd = nodes_[L.path.back()];
        nd.first = first[i];
        nd.nchild = (int16_t)nchildren(cnt[i], with_pass);
        nd.state = N_EXPANDED;
      }
      backup_value_path(L.path, values ? values[i] : 0.f, lambda <= 0.f);
    }
    wv.value_done = true;
    sims_ += n;
    if (lambda <= 0.f) finish(id);
  }

  // ------------------------------------------------------------------ rollout backup
  // Inputs of the GPU rollout kernel: colours [n][P] int8 and per-leaf meta
  // (player to move, ko, last move, second-to-last move, black passes, white passes,
  // moves played, end-of-game flag).
  void rollout_inputs(int id, int8_t* colors, int32_t* meta) {
    Wave& wv = wave(id);
    const int P = root_board_.npoints();
    for (size_t i = 0; i < wv.leaves.size(); ++i) {
      const Board& b = wv.leaves[i].board;
      for (int p = 0; p < P; ++p) colors[i * P + p] = (int8_t)b.color(p);
      int32_t* m = meta + i * 8;
      m[0] = b.current_player();
      m[1] = b.ko();
      m[2] = b.last1();
      m[3] = b.last2();
      m[4] = b.passes_black();
      m[5] = b.passes_white();
      m[6] = b.nmoves();
      m[7] = b.end_of_game() ? 1 : 0;
    }
  }

  // black_z: mean rollout result per leaf from BLACK's point of view
  void backup_rollout(int id, const float* black_z) {
    Wave& wv = wave(id);
    if (!wv.value_done) throw std::runtime_error("rollout backup before the value backup");
    if (wv.rolling) {
      wv.worker.join();
      wv.rolling = false;
    }
    for (size_t i = 0; i < wv.leaves.size(); ++i) {
      Leaf& L = wv.leaves[i];
      float z = L.z;
      if (black_z) z = L.board.current_player() == BLACK ? black_z[i] : -black_z[i];
      backup_rollout_path(L.path, z, true);
    }
    rollouts_ += (long)wv.leaves.size();
    release(id);
  }

  // CPU rollouts of a wave on a background thread (the pool runs them)
  void start_rollouts(int id) {
    Wave& wv = wave(id);
    if (wv.rolling) return;
    wv.rolling = true;
    const uint64_t base = seed * 0x100000001B3ull + (uint64_t)id * 0x9E3779B9ull;
    Wave* w = &wv;
    if (!rpool_) rpool_ = std::make_unique<Pool>(pool_.size());
    wv.worker = std::thread([this, w, base]() {
      rpool_->run((int)w->leaves.size(), [&](int i) {
        Leaf& L = w->leaves[i];
        Board b = L.board;
        b.set_enforce_superko(false);
        b.set_light(true);
        Rng rng(base + (uint64_t)i * 7919ull);
        const int ptm = L.board.current_player();
        const int win = rollout_policy->rollout(b, rng, rollout_limit);
        L.z = win == 0 ? 0.f : (win == ptm ? 1.f : -1.f);
      });
    });
  }

  void finish_rollouts(int id) { backup_rollout(id, nullptr); }

  int pending_waves() const { return (int)waves_.size(); }

  // ------------------------------------------------------------------ results / tree reuse
  float node_q(const Node& c) const {
    const bool use_r = lambda > 0.f && c.nr > 0, use_v = lambda < 1.f && c.n > 0;
    if (use_r && use_v) return (1.f - lambda) * c.w / c.n + lambda * c.wr / c.nr;
    if (use_r) return c.wr / c.nr;
    if (use_v) return c.w / c.n;
    return 0.f;
  }

  int best_move() const {
    const Node& r = nodes_[root_];
    if (r.state != N_EXPANDED || r.nchild == 0) return PASS;
    int best = r.first;
    for (int k = 1; k < r.nchild; ++k)
      if (nodes_[r.first + k].n > nodes_[best].n) best = r.first + k;
    return nodes_[best].move;
  }

  // (moves, visits, Q, prior) of the root's children
  void root_stats(std::vector<int32_t>& mv, std::vector<int32_t>& vis, std::vector<float>& q,
                  std::vector<float>& pr) const {
    const Node& r = nodes_[root_];
    const int nc = r.state == N_EXPANDED ? r.nchild : 0;
    mv.resize(nc);
    vis.resize(nc);
    q.resize(nc);
    pr.resize(nc);
    for (int k = 0; k < nc; ++k) {
      const Node& c = nodes_[r.first + k];
      mv[k] = c.move;
      vis[k] = c.n;
      q[k] = node_q(c);
      pr[k] = c.prior;
    }
  }

  // Re-root at the child reached by `move` (played on the root board). All waves must have
  // been finished. Returns true when the subtree was kept.
  bool advance(int move) {
    if (!waves_.empty()) throw std::runtime_error("advance() with waves in flight");
    root_board_.do_move(move, 0);
    const Node& r = nodes_[root_];
    int child = -1;
    if (r.state == N_EXPANDED)
      for (int k = 0; k < r.nchild; ++k)
        if (nodes_[r.first + k].move == move) child = r.first + k;
    if (child < 0) {
      Board b = root_board_;
      reset(b);
      return false;
    }
    compact(child);
    return true;
  }

  long sims() const { return sims_; }
  long rollouts() const { return rollouts_; }
  long terminal() const { return terminal_; }
  int collisions() const { return collisions_; }
  size_t num_nodes() const { return nodes_.size(); }
  int root_visits() const { return nodes_[root_].n; }

 private:
  void finish(int id) {
    Wave& wv = wave(id);
    if (wv.rolling) {
      wv.worker.join();
      wv.rolling = false;
    }
    release(id);
  }

  // finished waves are kept (up to a few) and handed out again by select(): their leaf boards
  // and paths keep their storage, so a new wave touches no fresh memory
  std::unique_ptr<Wave> take_wave() {
    if (free_waves_.empty()) return std::make_unique<Wave>();
    std::unique_ptr<Wave> w = std::move(free_waves_.back());
    free_waves_.pop_back();
    return w;
  }
  void recycle(std::unique_ptr<Wave> w) {
    w->value_done = false;
    w->rolling = false;
    if (free_waves_.size() < 16) free_waves_.push_back(std::move(w));
  }
  void release(int id) {
    auto it = waves_.find(id);
    if (it == waves_.end()) return;
    std::unique_ptr<Wave> w = std::move(it->second);
    waves_.erase(it);
    recycle(std::move(w));
  }

  void drop_waves() {
    for (auto& kv : waves_)
      if (kv.second->rolling) kv.second->worker.join();
    waves_.clear();
  }

  static int nchildren(int count, bool with_pass) {
    return with_pass ? count + 1 : (count == 0 ? 1 : count);
  }

  // children of `node` for its `count` sensible moves (PASS alone when there are none; PASS
  // always, last, with the network's pass prior pri[P] when `with_pass`), moves in increasing
  // point order from `next_move()`, priors renormalised over them, written into the
  // preallocated slots [first, first + nchildren(count, with_pass))
  template <class F>
  void fill_children(int node, int first, int count, bool with_pass, const float* pri, int P,
                     F&& next_move) {
    const int nc = nchildren(count, with_pass);
    float tot = 0.f;
    for (int k = 0; k < nc; ++k) {
      const int mv = k < count ? next_move() : PASS;
      float p = 1.f;
      if (pri && mv != PASS) p = std::max(pri[mv], 0.f);
      if (pri && mv == PASS && with_pass) p = std::max(pri[P], 0.f);
      tot += p;
      nodes_[first + k] = Node{node, -1, 0, (int16_t)mv, p, 0, 0, 0, 0.f, 0.f, N_NEW};
    }
    for (int k = 0; k < nc; ++k) {
      Node& c = nodes_[first + k];
      c.prior = tot > 0.f ? c.prior / tot : 1.f / nc;
    }
  }

  // v: value for the player to move at the leaf; a node at depth d stores it for its mover,
  // who is the leaf's player to move iff D-d is odd.
  void backup_value_path(const std::vector<int32_t>& path, float v, bool drop_vl) {
    const int D = (int)path.size() - 1;
    for (int d = D; d >= 0; --d) {
      Node& nd = nodes_[path[d]];
      nd.n += 1;
      if (drop_vl) nd.vl -= 1;
      nd.w += ((D - d) & 1) ? v : -v;
    }
  }
  void backup_rollout_path(const std::vector<int32_t>& path, float z, bool drop_vl) {
    const int D = (int)path.size() - 1;
    for (int d = D; d >= 0; --d) {
      Node& nd = nodes_[path[d]];
      nd.nr += 1;
      if (drop_vl) nd.vl -= 1;
      nd.wr += ((D - d) & 1) ? z : -z;
    }
  }

  // copy the subtree under `keep` into a fresh pool (BFS keeps children contiguous)
  void compact(int keep) {
    NodeArena out;
    out.reserve(std::max<size_t>(nodes_.capacity(), kNodeReserve));
    std::vector<int32_t> q{keep};
    Node r = nodes_[keep];
    r.parent = -1;
    r.vl = 0;
    if (r.state == N_PENDING) r.state = N_NEW;
    out.push_back(r);
    std::vector<int32_t> newid{0};
    for (size_t h = 0; h < q.size(); ++h) {
      const Node& old = nodes_[q[h]];
      const int nid = newid[h];
      if (old.state != N_EXPANDED || old.nchild == 0) continue;
      const int first = (int)out.size();
      for (int k = 0; k < old.nchild; ++k) {
        Node c = nodes_[old.first + k];
        c.parent = nid;
        c.vl = 0;
        if (c.state == N_PENDING) c.state = N_NEW;
        out.push_back(c);
        q.push_back(old.first + k);
        newid.push_back(first + k);
      }
      out[nid].first = first;
    }
    nodes_.swap(out);
    root_ = 0;
  }

  Board root_board_;
  NodeArena nodes_;
  int root_ = 0;
  std::map<int, std::unique_ptr<Wave>> waves_;
  std::vector<std::unique_ptr<Wave>> free_waves_;
  int next_wave_ = 0;
  Pool pool_;                    // expansions
  std::unique_ptr<Pool> rpool_;  // CPU rollouts (run from a wave's worker thread)
  long sims_ = 0, rollouts_ = 0, terminal_ = 0;
  int collisions_ = 0;
};


}  // namespace rag

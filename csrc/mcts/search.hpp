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
// Tree layout (host memory is the bound of a GPU-fed search, profiles/mcts_null_r3.txt):
//   * an expansion writes one 12-byte *edge* (move, prior, child index) per sensible move; the
//     32-byte child *node* (statistics) is allocated only when a descent first selects the edge.
//     Most children of a 19x19 node are never visited, so a simulation writes ~4 KB instead of
//     ~14 KB of nodes;
//   * the first kSorted edges of a node are its highest priors in descending order (partial sort
//     at expansion). Every unvisited child scores c_puct P sqrt(N), monotone in P, so a descent
//     only scores the edges up to the first never-selected one (the node's high-water mark)
//     instead of all ~360; nodes whose mark passed the sorted prefix are scanned in full;
//   * node and edge storage are address-stable arenas (reserved virtual ranges, bump allocation,
//     never moved, so concurrent descents may allocate), recycled process-wide with their pages
//     already faulted in, and a helper thread faults the next megabytes in ahead of the
//     allocation frontier: fresh-page faults cost 8 us per simulation before (19x19, 8 threads).
//
// Children are created for the leaf's sensible moves (legal, not an own true eye — the set the
// players use) with priors renormalised over them; PASS is the only child when no sensible move
// exists. Terminal leaves (end of game) are scored exactly and backed up at once.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
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
#include "../engine/pack.hpp"
#include "../engine/thread_pool.hpp"
#include "rollout.hpp"

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

namespace rag {

namespace mcts_detail {

enum : uint8_t { N_NEW = 0, N_PENDING = 1, N_EXPANDED = 2 };

struct Node {
  int32_t edges;   // first edge in the edge arena (valid once state == N_EXPANDED)
  int16_t nedge;   // number of children
  int16_t move;    // flat index of the move that leads here, PASS = -1
  int32_t n;       // value-net visits (every completed evaluation)
  int32_t nr;      // rollouts
  int32_t vl;      // in-flight descents through this node
  float w;         // value-net sum, for the player who played `move`
  float wr;        // rollout sum, same perspective
  int16_t hwm;     // 1 + the highest edge index whose child node exists
  uint8_t state;
  uint8_t pad;
};
static_assert(sizeof(Node) == 32, "Node must stay 32 bytes (two per cache line)");

struct Edge {
  int32_t child;   // node index, -1 until a descent first selects this edge
  float prior;
  int16_t move;
  int16_t pad;
};
static_assert(sizeof(Edge) == 12, "Edge must stay 12 bytes");

// ------------------------------------------------------------------ memory
// Process-wide cache of reserved anonymous mappings: an arena returns its range here with the
// number of bytes whose pages are already resident ("warm"), and the next arena of the same size
// (a compaction, a new Search) takes it back instead of faulting fresh pages in.
class MapCache {
 public:
  static MapCache& get() {
    static MapCache* c = new MapCache();  // leaked: arenas may outlive static destruction
    return *c;
  }
  void* take(size_t bytes, size_t& warm) {
    {
      std::lock_guard<std::mutex> g(mu_);
      for (size_t i = 0; i < free_.size(); ++i)
        if (free_[i].bytes == bytes) {
          Entry e = free_[i];
          free_.erase(free_.begin() + i);
          warm_total_ -= e.warm;
          warm = e.warm;
          return e.p;
        }
    }
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE,
                   MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (m == MAP_FAILED) throw std::bad_alloc();
    madvise(m, bytes, MADV_HUGEPAGE);
    warm = 0;
    return m;
  }
  void give(void* p, size_t bytes, size_t warm) {
    std::lock_guard<std::mutex> g(mu_);
    // keep a bounded amount of resident (warm) memory for the next Search's arenas: one node +
    // one edge arena by default (RAG_TREE_CACHE_MB, 0 = keep nothing); beyond it the range is
    // unmapped and its pages go back to the OS
    if (free_.size() < 4 && warm_total_ + warm <= budget()) {
      free_.push_back(Entry{p, bytes, warm});
      warm_total_ += warm;
    } else {
      munmap(p, bytes);
    }
  }
  // Unmap every cached range (callers that have finished searching).
  size_t trim() {
    std::lock_guard<std::mutex> g(mu_);
    size_t freed = 0;
    for (const Entry& e : free_) {
      munmap(e.p, e.bytes);
      freed += e.warm;
    }
    free_.clear();
    warm_total_ = 0;
    return freed;
  }
  size_t cached_bytes() {
    std::lock_guard<std::mutex> g(mu_);
    return warm_total_;
  }
  static size_t budget() {
    static const size_t b = [] {
      const char* e = getenv("RAG_TREE_CACHE_MB");
      return (e && *e ? size_t(atoll(e)) : size_t(2560)) << 20;
    }();
    return b;
  }

 private:
  struct Entry {
    void* p;
    size_t bytes, warm;
  };
  std::mutex mu_;
  std::vector<Entry> free_;
  size_t warm_total_ = 0;
};

// Address-stable bump arena of T over a reserved virtual range (never moves: descents on other
// threads hold references while it grows).
template <class T>
class Arena {
 public:
  explicit Arena(size_t cap) : cap_(cap) {
    size_t warm = 0;
    p_ = static_cast<T*>(MapCache::get().take(cap_ * sizeof(T), warm));
    warm_.store(warm);
  }
  ~Arena() {
    if (p_) MapCache::get().give(p_, cap_ * sizeof(T), std::max(warm_.load(), bytes_used()));
  }
  Arena(const Arena&) = delete;
  Arena& operator=(const Arena&) = delete;

  T& operator[](size_t i) { return p_[i]; }
  const T& operator[](size_t i) const { return p_[i]; }
  size_t size() const { return n_.load(std::memory_order_relaxed); }
  size_t capacity() const { return cap_; }
  bool room(size_t k) const { return size() + k <= cap_; }
  // callers check room() for the whole batch before the (possibly concurrent) allocations
  size_t alloc(size_t k) { return n_.fetch_add(k, std::memory_order_relaxed); }
  void clear() { n_.store(0); }
  size_t bytes_used() const { return size() * sizeof(T); }
  size_t warm_bytes() const { return warm_.load(std::memory_order_relaxed); }
  // Fault pages in up to `upto` bytes (helper thread; contents are never modified).
  void populate(size_t upto) {
    upto = std::min(upto, cap_ * sizeof(T));
    const size_t chunk = size_t(2) << 20;
    size_t w = warm_.load();
    while (w < upto) {
      const size_t len = std::min(chunk, cap_ * sizeof(T) - w);
      char* base = reinterpret_cast<char*>(p_) + w;
      if (madvise(base, len, MADV_POPULATE_WRITE) != 0) {
        // kernels without MADV_POPULATE_WRITE: a no-op read-modify-write per page
        for (size_t off = 0; off < len; off += 4096)
          __atomic_fetch_or(reinterpret_cast<uint32_t*>(base + off), 0u, __ATOMIC_RELAXED);
      }
      w += len;
      warm_.store(w);
    }
  }

 private:
  T* p_ = nullptr;
  size_t cap_ = 0;
  std::atomic<size_t> n_{0};
  std::atomic<size_t> warm_{0};
};

struct Leaf {
  Board board;                // built unless the wave was selected for shipping (paths only)
  std::vector<int32_t> path;  // root .. leaf
  float z = 0.f;
  int8_t ptm = 0;             // player to move at the leaf
};

struct Wave {
  std::vector<Leaf> leaves;
  bool value_done = false;
  bool built = true;   // leaf boards exist (false: select(B, false), the multi-GPU master)
  std::thread worker;  // CPU rollouts
  bool rolling = false;
};

using rag::Pool;

inline void atomic_addf(float* p, float v) {
  uint32_t* u = reinterpret_cast<uint32_t*>(p);
  uint32_t old = __atomic_load_n(u, __ATOMIC_RELAXED), nw;
  do {
    float f;
    std::memcpy(&f, &old, 4);
    f += v;
    std::memcpy(&nw, &f, 4);
  } while (!__atomic_compare_exchange_n(u, &old, nw, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED));
}

inline void atomic_max16(int16_t* p, int16_t v) {
  int16_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (cur < v &&
         !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
}

}  // namespace mcts_detail

using mcts_detail::Edge;
using mcts_detail::Leaf;
using mcts_detail::Node;
using mcts_detail::Wave;
using mcts_detail::N_EXPANDED;
using mcts_detail::N_NEW;
using mcts_detail::N_PENDING;

// Reserved (virtual) capacities: 32 M nodes (1 GiB) and 128 M edges (1.5 GiB) — about 350 k
// 19x19 simulations per move; pages become resident only as they are written.
constexpr size_t kNodeCap = size_t(1) << 25;
constexpr size_t kEdgeCap = size_t(1) << 27;

class Search {
 public:
  float c_puct = 5.f, lambda = 0.5f;
  int n_vl = 3, rollout_limit = 500, max_depth = 722;
  // networks with a pass logit: priors rows carry S*S + 1 entries and every
  // expanded node also gets a PASS child with the network's pass prior
  bool pass_prior = false;
  uint64_t seed = 1;
  bool keyed_rollouts = false;  // CPU rollouts seeded by the leaf position (position_key_seed)
  std::shared_ptr<RolloutPolicy> rollout_policy;
  // waves of at least this many leaves descend (and back up) on the pool; smaller ones run
  // serially and deterministically
  int parallel_select_min = 64;
  // such waves deal their descents top-down (descend_batched) instead of walking them one by one
  bool batched_select = true;
  static constexpr int kSorted = 32;

  explicit Search(const Board& root, int nthreads = 8)
      : rollout_policy(std::make_shared<RolloutPolicy>()),
        nodes_(std::make_unique<mcts_detail::Arena<Node>>(kNodeCap)),
        edges_(std::make_unique<mcts_detail::Arena<Edge>>(kEdgeCap)),
        pool_(std::max(nthreads, 1)) {
    reset(root);
  }
  ~Search() {
    drop_waves();
    stop_prefault();
  }
  Search(const Search&) = delete;
  Search& operator=(const Search&) = delete;

  void reset(const Board& root) {
    drop_waves();
    root_board_ = root;
    nodes_->clear();
    edges_->clear();
    root_ = new_node((int16_t)PASS);
    clear_root_external();
    prefault();
  }

  const Board& root_board() const { return root_board_; }
  int nthreads() const { return pool_.size(); }

  // ------------------------------------------------------------------ selection
  // Shared statistics are changed by concurrent descents and backups: read them atomically.
  template <class T>
  static T ld(const T& x) {
    return __atomic_load_n(&x, __ATOMIC_RELAXED);
  }
  static float ld(const float& x) {
    float f;
    __atomic_load(&x, &f, __ATOMIC_RELAXED);
    return f;
  }
  static uint8_t state_of(const Node& c) { return __atomic_load_n(&c.state, __ATOMIC_ACQUIRE); }

  // PUCT score from explicit statistics (value visits / sum, rollouts / sum, in-flight descents)
  float score(float n, float w, float nr, float wr, int vlc, float prior, float sq) const {
    const float vl = (float)(vlc * n_vl);
    const bool use_r = lambda > 0.f;
    const bool use_v = lambda < 1.f;
    float q = 0.f;
    if (use_r && use_v) {
      const float qv = n > 0.f ? w / n : 0.f;
      const float den = nr + vl;
      const float qr = den > 0.f ? (wr - vl) / den : qv;
      q = (1.f - lambda) * qv + lambda * qr;
    } else if (use_r) {
      const float den = nr + vl;
      q = den > 0.f ? (wr - vl) / den : 0.f;
    } else {
      const float den = n + vl;
      q = den > 0.f ? (w - vl) / den : 0.f;
    }
    return q + c_puct * prior * sq / (1.f + n + vl);
  }
  float child_score(const Node& c, float prior, float sq) const {
    return score((float)ld(c.n), ld(c.w), (float)ld(c.nr), ld(c.wr), ld(c.vl), prior, sq);
  }

  // Edge index of the PUCT argmax at expanded node p (first maximum in edge order).
  int select_edge(int p) const {
    const Node& pn = (*nodes_)[p];
    const int ne = pn.nedge;
    const Edge* E = &(*edges_)[pn.edges];
    if (p == root_ && has_ext_) return select_root_ext(pn, E, ne);
    const float np = (float)(ld(pn.n) + ld(pn.vl) * n_vl);
    const float sq = std::sqrt(std::max(np, 1.f));
    // edges past the high-water mark have no node yet (unvisited): within the sorted prefix the
    // first of them is the best of them all
    const int h = ld(pn.hwm);
    const int lim = h < std::min(ne, (int)kSorted) ? h + 1 : ne;
    int best = 0;
    float bv = -1e30f;
    for (int k = 0; k < lim; ++k) {
      const int32_t c = __atomic_load_n(&E[k].child, __ATOMIC_ACQUIRE);
      const float v = c < 0 ? c_puct * E[k].prior * sq : child_score((*nodes_)[c], E[k].prior, sq);
      if (v > bv) {
        bv = v;
        best = k;
      }
    }
    return best;
  }

  // ------------------------------------------------------------------ shared root statistics
  // Distributed search (search/distributed.py SharedRootMCTS): every rank grows its own tree
  // from the same root, and the ranks exchange the statistics of the root's children each
  // round. The other ranks' totals enter this rank's root selection as *external* statistics
  // (indexed by move; PASS at P), so all ranks steer their descents by the job-wide root values
  // and visit counts. root_deltas() reports what this rank added since its previous call.
  void set_root_external(const float* n, const float* w, const float* nr, const float* wr) {
    // written between waves (the search's own thread); sized once, updated in place
    const int M = root_board_.npoints() + 1;
    if (ext_.size() != 4 * (size_t)M) ext_.assign(4 * (size_t)M, 0.f);
    ext_total_n_ = 0.f;
    for (int m = 0; m < M; ++m) {
      ext_[m] = n[m];
      ext_[M + m] = w[m];
      ext_[2 * M + m] = nr[m];
      ext_[3 * M + m] = wr[m];
      ext_total_n_ += n[m];
    }
    has_ext_ = true;
  }
  void clear_root_external() {
    ext_.clear();
    snap_.clear();
    has_ext_ = false;
    ext_total_n_ = 0.f;
  }
  // out: [4][P+1] (n, w, nr, wr) added by this rank at the root's children since the last call
  void root_deltas(float* out) {
    const int M = root_board_.npoints() + 1;
    if (snap_.size() != 4 * (size_t)M) snap_.assign(4 * (size_t)M, 0.f);
    std::fill(out, out + 4 * (size_t)M, 0.f);
    const Node& r = (*nodes_)[root_];
    if (ld(r.state) != N_EXPANDED) return;
    const Edge* E = &(*edges_)[r.edges];
    for (int k = 0; k < r.nedge; ++k) {
      const int32_t c = __atomic_load_n(&E[k].child, __ATOMIC_ACQUIRE);
      if (c < 0) continue;
      const Node& nd = (*nodes_)[c];
      const int m = E[k].move < 0 ? M - 1 : E[k].move;
      const float cur[4] = {(float)ld(nd.n), ld(nd.w), (float)ld(nd.nr), ld(nd.wr)};
      for (int j = 0; j < 4; ++j) {
        out[j * M + m] = cur[j] - snap_[j * M + m];
        snap_[j * M + m] = cur[j];
      }
    }
  }

 private:
  int select_root_ext(const Node& pn, const Edge* E, int ne) const {
    const int M = root_board_.npoints() + 1;
    const float np = (float)(ld(pn.n) + ld(pn.vl) * n_vl) + ext_total_n_;
    const float sq = std::sqrt(std::max(np, 1.f));
    int best = 0;
    float bv = -1e30f;
    for (int k = 0; k < ne; ++k) {
      const int m = E[k].move < 0 ? M - 1 : E[k].move;
      float n = ext_[m], w = ext_[M + m], nr = ext_[2 * M + m], wr = ext_[3 * M + m];
      int vl = 0;
      const int32_t c = __atomic_load_n(&E[k].child, __ATOMIC_ACQUIRE);
      if (c >= 0) {
        const Node& nd = (*nodes_)[c];
        n += (float)ld(nd.n);
        w += ld(nd.w);
        nr += (float)ld(nd.nr);
        wr += ld(nd.wr);
        vl = ld(nd.vl);
      }
      const float v = score(n, w, nr, wr, vl, E[k].prior, sq);
      if (v > bv) {
        bv = v;
        best = k;
      }
    }
    return best;
  }

 public:
  // Returns (wave id, number of leaves); id -1 when nothing was selected.
  //
  // Three phases: (1) tree walks with virtual loss (descend(); on the pool for B >=
  // parallel_select_min, see descend_parallel); (2) the leaf boards (root copy + the path's
  // moves) are built in parallel on the pool; (3) descents that ended on a terminal position are
  // scored on their board and backed up at once (their virtual loss, taken in phase 1 so that
  // later walks of the same wave avoid them, is dropped again).
  //
  // build = false (the multi-GPU master, csrc/mcts/master.hpp): the leaf boards are not built —
  // the evaluating rank rebuilds them from the root and the shipped move paths (write_paths /
  // load_paths) — only terminal descents get a board, to be scored.
  std::pair<int, int> select(int B, bool build = true) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    collisions_ = 0;
    if (!nodes_->room((size_t)4 * B + 16))
      throw std::runtime_error("search tree full (node arena); advance() or reset()");
    std::vector<std::vector<int32_t>> paths;
    std::vector<uint8_t> term;
    paths.reserve(B);
    term.reserve(B);
    if (B >= parallel_select_min && batched_select && !has_ext_) {
      descend_batched(B, paths, term);
    } else if (B >= parallel_select_min && pool_.size() > 1) {
      descend_parallel(B, paths, term);
    } else {
      int attempts = 0, claimed = 0;
      while (claimed < B && attempts < 4 * B) {
        ++attempts;
        std::vector<int32_t> path;
        bool terminal = false;
        if (!descend(path, terminal)) {
          ++collisions_;
          continue;
        }
        if (!terminal) ++claimed;
        paths.push_back(std::move(path));
        term.push_back(terminal ? 1 : 0);
      }
    }
    const auto t1 = clk::now();
    const Board& rb = root_board_;
    const int nd = (int)paths.size();
    int nleaf = 0;
    for (int i = 0; i < nd; ++i) nleaf += term[i] ? 0 : 1;
    // leaf boards go straight into a recycled wave (its Leaf storage is reused: no fresh pages);
    // terminal descents get a scratch board
    std::unique_ptr<Wave> wave = take_wave();
    wave->leaves.resize(nleaf);
    wave->built = build;
    std::vector<int> slot(nd);
    int nt = 0, nl = 0;
    for (int i = 0; i < nd; ++i) slot[i] = term[i] ? nt++ : nl++;
    std::vector<Board> tboards(nt);
    const bool light = !rb.enforce_superko();
    const int rptm = rb.current_player();
    auto leaf_job = [&](int i) {
      const std::vector<int32_t>& path = paths[i];
      if (build || term[i]) {
        Board& b = term[i] ? tboards[slot[i]] : wave->leaves[slot[i]].board;
        b = rb;
        b.set_light(light);
        for (size_t d = 1; d < path.size(); ++d) b.play_unchecked((*nodes_)[path[d]].move);
      }
      if (!term[i]) {
        Leaf& L = wave->leaves[slot[i]];
        // every move, a pass included, hands the turn over
        L.ptm = (int8_t)((path.size() - 1) & 1 ? -rptm : rptm);
        L.path.swap(paths[i]);
        L.z = 0.f;
      }
    };
    if (build || nt > 0) {
      pool_.run(nd, leaf_job);
    } else {
      for (int i = 0; i < nd; ++i) leaf_job(i);  // path swaps only: no pool wake-up
    }
    for (int i = 0; i < nd; ++i) {
      if (!term[i]) continue;
      const Board& b = tboards[slot[i]];
      const int win = b.get_winner();
      const float v = win == 0 ? 0.f : (win == b.current_player() ? 1.f : -1.f);
      backup_value_path(paths[i], v, true);
      if (lambda > 0.f) backup_rollout_path(paths[i], v, false);
      ++terminal_;
    }
    const auto t2 = clk::now();
    t_descend_ += std::chrono::duration<double>(t1 - t0).count();
    t_build_ += std::chrono::duration<double>(t2 - t1).count();
    prefault();
    const int n = (int)wave->leaves.size();
    if (n == 0) {
      recycle(std::move(wave));
      return {-1, 0};
    }
    std::lock_guard<std::mutex> g(wmu_);
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
        if (!descend(path, terminal)) {
          coll.fetch_add(1, std::memory_order_relaxed);
          continue;
        }
        if (!terminal && nleaf.fetch_add(1) >= B) {  // over-claimed: hand the leaf back
          __atomic_store_n(&(*nodes_)[path.back()].state, (uint8_t)N_NEW, __ATOMIC_RELEASE);
          for (int id : path) __atomic_fetch_sub(&(*nodes_)[id].vl, 1, __ATOMIC_RELAXED);
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

  // Batched wave descent: the B descents of a wave dealt top-down instead of walked one by one
  // (the wave-level form of virtual-loss selection). A node that k descents reach scores its
  // children ONCE and deals the k descents one at a time to the PUCT argmax, adding each dealt
  // descent's virtual loss to that child's score before the next deal (a max-heap: one child
  // changes per deal); the node's sqrt(N) counts all k of the wave's visits. A fresh leaf takes
  // one descent (its claim), a leaf awaiting its evaluation none, a terminal node any number
  // (each is scored). Every reached node is scored once per wave and takes its virtual loss in
  // one atomic add — instead of once per descent through it: B x depth scans of the root's ~360
  // edges, and every thread's atomics on the root's cache line, were the host ceiling of a
  // multi-GPU search (profiles/mcts_master_null_r6.txt) — and no descent collides with a leaf
  // another one claimed. The children of a node that >= kSplit descents reached form the next
  // level of tasks (dealt in parallel), those of smaller ones are walked depth-first by the
  // thread that dealt them.
  static constexpr int kSplit = 16;
  struct DTask {
    int node, k, depth, ptm, l1, l2, nm;
    bool end;
    std::vector<int32_t> path;  // root .. node
  };

  void descend_batched(int B, std::vector<std::vector<int32_t>>& paths,
                       std::vector<uint8_t>& term) {
    std::atomic<int> coll{0};
    const Board& rb = root_board_;
    // level-synchronous: the tasks of one level are handed out by an atomic counter (no queue
    // lock per task: that lock's waits were 2/3 of a 16-thread wave's descent time); a task
    // walks its subtree depth-first unless its node took >= kSplit descents, whose children
    // form the next level
    struct Scratch {
      std::vector<std::vector<int32_t>> out;
      std::vector<uint8_t> oterm;
      std::vector<DTask> local, next;
      std::vector<float> sc;
      std::vector<int> dealt;
      std::vector<int8_t> cap;
      std::vector<std::pair<float, int>> heap;
    };
    const int nw = std::max(1, pool_.size());
    std::vector<Scratch> scr(nw);
    std::vector<DTask> frontier;
    frontier.push_back(DTask{root_, B, 0, rb.current_player(), rb.last1(), rb.last2(),
                             rb.nmoves(), rb.end_of_game(), {root_}});
    while (!frontier.empty()) {
      std::atomic<int> next{0};
      const int nf = (int)frontier.size();
      auto slot = [&](int w) {
        Scratch& S = scr[w];
        for (int i = next.fetch_add(1); i < nf; i = next.fetch_add(1)) {
          S.local.push_back(std::move(frontier[i]));
          while (!S.local.empty()) {
            DTask u = std::move(S.local.back());
            S.local.pop_back();
            deal(u, S.local, S.next, S.out, S.oterm, coll, S.sc, S.dealt, S.cap, S.heap);
          }
        }
      };
      if (nf < 4 || nw == 1)
        slot(0);  // the root level: no pool wake-up
      else
        pool_.run(nw, slot);
      frontier.clear();
      for (Scratch& S : scr) {
        for (DTask& t : S.next) frontier.push_back(std::move(t));
        S.next.clear();
      }
    }
    for (Scratch& S : scr)
      for (size_t k = 0; k < S.out.size(); ++k) {
        paths.push_back(std::move(S.out[k]));
        term.push_back(S.oterm[k]);
      }
    collisions_ = coll.load();
  }

  void deal(DTask& u, std::vector<DTask>& local, std::vector<DTask>& shared,
            std::vector<std::vector<int32_t>>& out, std::vector<uint8_t>& oterm,
            std::atomic<int>& coll, std::vector<float>& sc, std::vector<int>& dealt,
            std::vector<int8_t>& cap, std::vector<std::pair<float, int>>& heap) {
    NodeArena& N = *nodes_;
    Node& nd = N[u.node];
    __atomic_fetch_add(&nd.vl, u.k, __ATOMIC_RELAXED);
    const uint8_t st = state_of(nd);
    const bool terminal = u.end || u.depth >= max_depth || (st == N_EXPANDED && nd.nedge == 0);
    auto give_back = [&](int extra) {
      for (int id : u.path) __atomic_fetch_sub(&N[id].vl, extra, __ATOMIC_RELAXED);
      coll.fetch_add(extra, std::memory_order_relaxed);
    };
    if (terminal) {  // every descent is scored (and backed up) on its own
      for (int i = 0; i < u.k; ++i) {
        out.push_back(u.path);
        oterm.push_back(1);
      }
      return;
    }
    if (st != N_EXPANDED) {  // a leaf: one descent claims it, the others collide
      uint8_t expect = N_NEW;
      const bool claimed = __atomic_compare_exchange_n(&nd.state, &expect, (uint8_t)N_PENDING,
                                                       false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
      const int extra = claimed ? u.k - 1 : u.k;
      if (extra > 0) give_back(extra);
      if (claimed) {
        out.push_back(std::move(u.path));
        oterm.push_back(0);
      }
      return;
    }
    const int ne = nd.nedge;
    const Edge* E = &(*edges_)[nd.edges];
    // candidates: within the sorted-prior prefix the unvisited edges score in prior order and
    // take one descent each, so k descents reach at most edges [0, hwm + k); else all edges
    const int h = ld(nd.hwm);
    const int lim = h + u.k <= std::min(ne, (int)kSorted) ? h + u.k : ne;
    const float np = (float)(ld(nd.n) + ld(nd.vl) * n_vl);  // the wave's k visits included
    const float sq = std::sqrt(std::max(np, 1.f));
    const int cptm = -u.ptm, cnm = u.nm + 1;
    sc.resize(lim);
    dealt.assign(lim, 0);
    cap.resize(lim);
    heap.clear();
    auto edge_score = [&](int e) {
      const int32_t c = __atomic_load_n(&E[e].child, __ATOMIC_ACQUIRE);
      if (c < 0) return c_puct * E[e].prior * sq;
      const Node& cn = N[c];
      return score((float)ld(cn.n), ld(cn.w), (float)ld(cn.nr), ld(cn.wr), ld(cn.vl) + dealt[e],
                   E[e].prior, sq);
    };
    for (int e = 0; e < lim; ++e) {
      const int m = E[e].move;
      const bool cend = cnm > 1 && m == PASS && u.l1 == PASS && cptm == WHITE;
      const int32_t c = __atomic_load_n(&E[e].child, __ATOMIC_ACQUIRE);
      int8_t cp = 1;  // a fresh leaf: one descent
      if (cend || u.depth + 1 >= max_depth) {
        cp = -1;  // terminal: any number
      } else if (c >= 0) {
        const uint8_t cs = state_of(N[c]);
        cp = cs == N_PENDING ? 0 : (cs == N_EXPANDED ? -1 : 1);
      }
      cap[e] = cp;
      if (cp != 0) heap.emplace_back(edge_score(e), -e);
    }
    // max-heap on (score, -edge): ties go to the lower edge, as select_edge's first maximum
    auto less = [](const std::pair<float, int>& a, const std::pair<float, int>& b) {
      return a.first < b.first || (a.first == b.first && a.second < b.second);
    };
    std::make_heap(heap.begin(), heap.end(), less);
    int left = u.k;
    while (left > 0 && !heap.empty()) {
      std::pop_heap(heap.begin(), heap.end(), less);
      const int e = -heap.back().second;
      heap.pop_back();
      ++dealt[e];
      --left;
      if (cap[e] < 0) {
        heap.emplace_back(edge_score(e), -e);
        std::push_heap(heap.begin(), heap.end(), less);
      }
    }
    if (left > 0) give_back(left);  // every child is awaiting its evaluation
    for (int e = 0; e < lim; ++e) {
      if (!dealt[e]) continue;
      const int child = child_of(u.node, e);
      const int m = E[e].move;
      const bool cend = cnm > 1 && m == PASS && u.l1 == PASS && cptm == WHITE;
      DTask t{child, dealt[e], u.depth + 1, cptm, m, u.l1, cnm, cend, u.path};
      t.path.push_back(child);
      // the children of a node many descents reached go to the next level (the root's ~200
      // small subtrees would otherwise all be walked by the thread that dealt them)
      if (u.k >= kSplit)
        shared.push_back(std::move(t));
      else
        local.push_back(std::move(t));
    }
  }

  // One walk from the root with virtual loss (atomic adds as the walk passes each node, so
  // concurrent walks spread). Tracks only what the walk needs (player to move, the last two
  // moves and the move count decide the end of the game, exactly as Board::play_unchecked
  // does). Returns false (virtual loss already given back) when the walk ends on a leaf that
  // another descent is waiting for; terminal = end of game / depth limit / a node without
  // children (its virtual loss stays until its immediate backup).
  bool descend(std::vector<int32_t>& path, bool& terminal) {
    NodeArena& N = *nodes_;
    const Board& rb = root_board_;
    path.clear();
    path.reserve(32);
    int node = root_;
    path.push_back(node);
    __atomic_fetch_add(&N[node].vl, 1, __ATOMIC_RELAXED);
    int depth = 0;
    int ptm = rb.current_player(), l1 = rb.last1(), l2 = rb.last2(), nm = rb.nmoves();
    bool end = rb.end_of_game();
    while (state_of(N[node]) == N_EXPANDED && N[node].nedge > 0 && !end && depth < max_depth) {
      node = child_of(node, select_edge(node));
      path.push_back(node);
      __atomic_fetch_add(&N[node].vl, 1, __ATOMIC_RELAXED);
      ++depth;
      ++nm;
      l2 = l1;
      l1 = N[node].move;
      ptm = -ptm;
      if (nm > 1 && l1 == PASS && l2 == PASS && ptm == WHITE) end = true;
    }
    Node& leaf = N[node];
    const uint8_t st = state_of(leaf);
    terminal = end || depth >= max_depth || (st == N_EXPANDED && leaf.nedge == 0);
    if (!terminal) {
      uint8_t expect = N_NEW;
      const bool claimed = __atomic_compare_exchange_n(&leaf.state, &expect, (uint8_t)N_PENDING,
                                                       false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
      if (!claimed) {  // already waiting for its evaluation
        for (int id : path) __atomic_fetch_sub(&N[id].vl, 1, __ATOMIC_RELAXED);
        return false;
      }
    }
    return true;
  }

  Wave& wave(int id) {
    std::lock_guard<std::mutex> g(wmu_);
    auto it = waves_.find(id);
    if (it == waves_.end()) throw std::invalid_argument("unknown or finished wave");
    return *it->second;
  }
  int num_leaves(int id) { return (int)wave(id).leaves.size(); }
  std::vector<const Board*> leaf_boards(int id) {
    Wave& wv = wave(id);
    if (!wv.built) throw std::invalid_argument("leaf_boards of a shipped wave (no leaf boards)");
    std::vector<const Board*> v;
    for (auto& L : wv.leaves) v.push_back(&L.board);
    return v;
  }

  // ------------------------------------------------------------------ leaf packing
  // Everything the GPU side needs about a wave's leaves, written in parallel straight into the
  // caller's (pinned) buffers: feature-kernel inputs, rollout-kernel meta and, optionally, the
  // host-read ladder planes / superko-illegal masks.
  void pack_inputs(int id, const PackOut& o) {
    Wave& wv = wave(id);
    if (!wv.built) throw std::invalid_argument("pack_inputs of a shipped wave (no leaf boards)");
    pool_.run((int)wv.leaves.size(), [&](int i) { pack_board(wv.leaves[i].board, i, o); });
  }

  // ------------------------------------------------------------------ shipped waves
  // The multi-GPU search (csrc/mcts/master.hpp) ships a leaf as its move path from the root:
  // record [depth, move_1 .. move_depth] (int16, PASS = -1) of `stride` entries. The evaluating
  // rank holds the same root board and replays the path (load_paths), so the master builds no
  // leaf boards and a record is a few dozen bytes instead of a board.
  // Writes leaves [lo, hi) of wave `id`; returns the deepest path written.
  int write_paths(int id, int lo, int hi, int16_t* out, int stride) {
    Wave& wv = wave(id);
    int deepest = 0;
    for (int i = lo; i < hi; ++i) {
      const std::vector<int32_t>& path = wv.leaves[i].path;
      const int d = (int)path.size() - 1;
      if (d + 1 > stride) throw std::runtime_error("leaf path longer than the record stride");
      int16_t* r = out + (size_t)(i - lo) * stride;
      r[0] = (int16_t)d;
      for (int k = 1; k <= d; ++k) r[k] = (int16_t)(*nodes_)[path[k]].move;
      deepest = std::max(deepest, d);
    }
    return deepest;
  }

  // A wave of n leaves rebuilt from shipped path records (an evaluating rank's search object:
  // its tree is never used). Boards are the root board + the path's moves, with the root's
  // history (superko) when the root enforces it — exactly the boards select() builds.
  int load_paths(const int16_t* recs, int n, int stride) {
    std::unique_ptr<Wave> wave = take_wave();
    wave->leaves.resize(n);
    wave->built = true;
    const Board& rb = root_board_;
    const bool light = !rb.enforce_superko();
    pool_.run(n, [&](int i) {
      const int16_t* r = recs + (size_t)i * stride;
      const int d = r[0];
      Leaf& L = wave->leaves[i];
      L.board = rb;
      L.board.set_light(light);
      for (int k = 1; k <= d && k < stride; ++k) L.board.play_unchecked(r[k]);
      L.path.clear();
      L.z = 0.f;
      L.ptm = (int8_t)L.board.current_player();
    });
    std::lock_guard<std::mutex> g(wmu_);
    const int id = next_wave_++;
    waves_[id] = std::move(wave);
    return id;
  }

  // Mean CPU rollout result per leaf from BLACK's point of view (joins start_rollouts()).
  void rollout_black_z(int id, float* out) {
    Wave& wv = wave(id);
    if (wv.rolling) {
      wv.worker.join();
      wv.rolling = false;
    }
    for (size_t i = 0; i < wv.leaves.size(); ++i)
      out[i] = wv.leaves[i].ptm == BLACK ? wv.leaves[i].z : -wv.leaves[i].z;
  }

  // Forget a wave without backing anything up (load_paths() waves once evaluated).
  void drop_wave(int id) { finish(id); }

  // ------------------------------------------------------------------ value backup
  // priors: [n][stride] network move probabilities (nullptr => uniform); values: [n] (nullptr
  // => value statistics untouched: rollouts only).
  // sensible: optional [n][P] mask of the leaves' sensible moves (legal, not an own true eye),
  // e.g. the sensibleness plane the GPU feature kernel already produced; otherwise the moves
  // are generated natively on the pool.
  void backup_value(int id, const float* priors, int stride, const float* values,
                    const uint8_t* sensible = nullptr) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    Wave& wv = wave(id);
    if (wv.value_done) throw std::runtime_error("value backup twice");
    if (!wv.built && !sensible)
      throw std::invalid_argument("a shipped wave (no leaf boards) needs the sensible masks");
    const int n = (int)wv.leaves.size();
    const int P = root_board_.npoints();
    const bool par = n >= parallel_select_min && pool_.size() > 1;
    const bool with_pass = pass_prior && priors != nullptr && stride > P;
    // one pass per leaf (parallel): its children — the sensible-move mask's moves, or natively
    // generated ones — get an edge block of their own from the arena's atomic bump pointer (the
    // leaves of one wave are distinct nodes: select() skips pending ones); then the expansion is
    // published. The path backups follow on this thread.
    if (!edges_->room((size_t)n * (P + 1)))
      throw std::runtime_error("search tree full (edge arena); advance() or reset()");
    auto body = [&](int i) {
      Leaf& L = wv.leaves[i];
      Node& nd = (*nodes_)[L.path.back()];
      if (state_of(nd) == N_EXPANDED) return;
      const float* pri = priors ? priors + (size_t)i * stride : nullptr;
      int nc;
      size_t e0;
      if (sensible) {
        const uint8_t* m = sensible + (size_t)i * P;
        int c = 0;
        for (int p = 0; p < P; ++p) c += m[p] != 0;
        nc = nchildren(c, with_pass);
        e0 = edges_->alloc(nc);
        int k = 0;
        fill_edges(e0, c, with_pass, pri, P, [&]() {
          while (!m[k]) ++k;
          return k++;
        });
      } else {
        std::vector<int> mv, eyes;
        L.board.legal_moves(mv, eyes);
        nc = nchildren((int)mv.size(), with_pass);
        e0 = edges_->alloc(nc);
        size_t k = 0;
        fill_edges(e0, (int)mv.size(), with_pass, pri, P, [&]() { return mv[k++]; });
      }
      nd.edges = (int32_t)e0;
      nd.nedge = (int16_t)nc;
      nd.hwm = 0;
      __atomic_store_n(&nd.state, (uint8_t)N_EXPANDED, __ATOMIC_RELEASE);
    };
    if (par) {
      pool_.run(n, body);
    } else {
      for (int i = 0; i < n; ++i) body(i);
    }
    // the path backups on this thread: every leaf's path ends at the root, so on the pool they
    // were all threads' compare-and-swap loops on the same few cache lines; here no other thread
    // touches the statistics (descents run only inside select()), so plain loads and stores
    for (int i = 0; i < n; ++i)
      backup_path_serial(wv.leaves[i].path, values ? values[i] : 0.f, lambda <= 0.f, false);
    wv.value_done = true;
    sims_ += n;
    t_backup_ += std::chrono::duration<double>(clk::now() - t0).count();
    prefault();
    if (lambda <= 0.f) finish(id);
  }

  // ------------------------------------------------------------------ rollout backup
  // Inputs of the GPU rollout kernel: colours [n][P] int8 and per-leaf meta
  // (player to move, ko, last move, second-to-last move, black passes, white passes,
  // moves played, end-of-game flag).
  void rollout_inputs(int id, int8_t* colors, int32_t* meta) {
    PackOut o;
    const int P = root_board_.npoints();
    o.colors = colors;
    o.s_colors = P;
    o.meta8 = meta;
    o.s_meta8 = 8 * sizeof(int32_t);
    pack_inputs(id, o);
  }
  // black_z: mean rollout result per leaf from BLACK's point of view
  void backup_rollout(int id, const float* black_z) {
    Wave& wv = wave(id);
    if (!wv.value_done) throw std::runtime_error("rollout backup before the value backup");
    if (wv.rolling) {
      wv.worker.join();
      wv.rolling = false;
    }
    const int n = (int)wv.leaves.size();
    // on this thread (see backup_value)
    for (int i = 0; i < n; ++i) {
      Leaf& L = wv.leaves[i];
      float z = L.z;
      if (black_z) z = L.ptm == BLACK ? black_z[i] : -black_z[i];
      backup_path_serial(L.path, z, true, true);
    }
    rollouts_ += (long)n;
    release(id);
  }

  // CPU rollouts of a wave on a background thread (the pool runs them)
  void start_rollouts(int id) {
    Wave& wv = wave(id);
    if (wv.rolling) return;
    if (!wv.built) throw std::invalid_argument("rollouts of a shipped wave (no leaf boards)");
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
        Rng rng(keyed_rollouts ? position_key_seed(L.board.hash(), L.board.current_player())
                               : base + (uint64_t)i * 7919ull);
        const int ptm = L.board.current_player();
        const int win = rollout_policy->rollout(b, rng, rollout_limit);
        L.z = win == 0 ? 0.f : (win == ptm ? 1.f : -1.f);
      });
    });
  }

  void finish_rollouts(int id) { backup_rollout(id, nullptr); }

  int pending_waves() const {
    std::lock_guard<std::mutex> g(wmu_);
    return (int)waves_.size();
  }

  // ------------------------------------------------------------------ results / tree reuse
  float node_q(const Node& c) const {
    const bool use_r = lambda > 0.f && c.nr > 0, use_v = lambda < 1.f && c.n > 0;
    if (use_r && use_v) return (1.f - lambda) * c.w / c.n + lambda * c.wr / c.nr;
    if (use_r) return c.wr / c.nr;
    if (use_v) return c.w / c.n;
    return 0.f;
  }

  int best_move() const {
    const Node& r = (*nodes_)[root_];
    if (r.state != N_EXPANDED || r.nedge == 0) return PASS;
    const Edge* E = &(*edges_)[r.edges];
    int best = 0, bn = -1;
    for (int k = 0; k < r.nedge; ++k) {
      const int v = E[k].child >= 0 ? (*nodes_)[E[k].child].n : 0;
      // most visits; ties to the lower point (pass last) whatever the edge order
      if (v > bn || (v == bn && move_key(E[k].move) < move_key(E[best].move))) {
        bn = v;
        best = k;
      }
    }
    return E[best].move;
  }

  // One 64-bit key per expanded node: a hash of its move path from the root (the same node of
  // two trees of the same root gets the same key). Used to measure how much of the work of
  // several ranks' trees is the same tree expanded twice (search/efficiency.py).
  std::vector<uint64_t> expanded_keys() const {
    std::vector<uint64_t> out;
    std::vector<std::pair<int32_t, uint64_t>> st{{root_, 0x243F6A8885A308D3ull}};
    while (!st.empty()) {
      const auto [i, h] = st.back();
      st.pop_back();
      const Node& nd = (*nodes_)[i];
      if (nd.state != N_EXPANDED) continue;
      out.push_back(h);
      const Edge* E = &(*edges_)[nd.edges];
      for (int k = 0; k < nd.nedge; ++k) {
        if (E[k].child < 0) continue;
        uint64_t x = h ^ (uint64_t(uint16_t(E[k].move)) + 0x9E3779B97F4A7C15ull);
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        st.push_back({E[k].child, x ^ (x >> 31)});
      }
    }
    return out;
  }

  // (moves, visits, Q, prior) of the root's children, in increasing point order (pass last)
  void root_stats(std::vector<int32_t>& mv, std::vector<int32_t>& vis, std::vector<float>& q,
                  std::vector<float>& pr) const {
    const Node& r = (*nodes_)[root_];
    const int nc = r.state == N_EXPANDED ? r.nedge : 0;
    std::vector<int> order(nc);
    for (int k = 0; k < nc; ++k) order[k] = k;
    const Edge* E = nc ? &(*edges_)[r.edges] : nullptr;
    std::sort(order.begin(), order.end(),
              [&](int a, int b) { return move_key(E[a].move) < move_key(E[b].move); });
    mv.resize(nc);
    vis.resize(nc);
    q.resize(nc);
    pr.resize(nc);
    for (int j = 0; j < nc; ++j) {
      const Edge& e = E[order[j]];
      mv[j] = e.move;
      pr[j] = e.prior;
      if (e.child >= 0) {
        const Node& c = (*nodes_)[e.child];
        vis[j] = c.n;
        q[j] = node_q(c);
      } else {
        vis[j] = 0;
        q[j] = 0.f;
      }
    }
  }

  // Re-root at the child reached by `move` (played on the root board). All waves must have
  // been finished. Returns true when the subtree was kept.
  bool advance(int move) {
    if (pending_waves()) throw std::runtime_error("advance() with waves in flight");
    root_board_.do_move(move, 0);
    const Node& r = (*nodes_)[root_];
    int child = -1;
    if (r.state == N_EXPANDED)
      for (int k = 0; k < r.nedge; ++k) {
        const Edge& e = (*edges_)[r.edges + k];
        if (e.move == move) child = e.child;
      }
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
  size_t num_nodes() const { return nodes_->size(); }
  size_t num_edges() const { return edges_->size(); }
  int root_visits() const { return (*nodes_)[root_].n; }
  // accumulated host seconds: descents, leaf-board construction, value backups
  std::tuple<double, double, double> timers() const { return {t_descend_, t_build_, t_backup_}; }

 private:
  using NodeArena = mcts_detail::Arena<Node>;

  static int move_key(int m) { return m < 0 ? (1 << 20) : m; }

  int new_node(int16_t move) {
    const int idx = (int)nodes_->alloc(1);
    (*nodes_)[idx] = Node{-1, 0, move, 0, 0, 0, 0.f, 0.f, 0, N_NEW, 0};
    return idx;
  }

  // Child node of edge k of p, allocated on first selection. Concurrent first selections race on
  // the edge's child slot; the loser's node stays unused.
  int child_of(int p, int k) {
    Node& pn = (*nodes_)[p];
    Edge& e = (*edges_)[pn.edges + k];
    int32_t c = __atomic_load_n(&e.child, __ATOMIC_ACQUIRE);
    if (c >= 0) return c;
    const int idx = new_node(e.move);
    // the mark first: a descent that sees the child also sees the edge inside the mark
    mcts_detail::atomic_max16(&pn.hwm, (int16_t)(k + 1));
    int32_t expect = -1;
    if (__atomic_compare_exchange_n(&e.child, &expect, idx, false, __ATOMIC_ACQ_REL,
                                    __ATOMIC_ACQUIRE))
      return idx;
    return expect;
  }

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
    std::lock_guard<std::mutex> g(wmu_);
    if (free_waves_.empty()) return std::make_unique<Wave>();
    std::unique_ptr<Wave> w = std::move(free_waves_.back());
    free_waves_.pop_back();
    return w;
  }
  void recycle(std::unique_ptr<Wave> w) {
    w->value_done = false;
    w->rolling = false;
    std::lock_guard<std::mutex> g(wmu_);
    if (free_waves_.size() < 16) free_waves_.push_back(std::move(w));
  }
  void release(int id) {
    std::unique_ptr<Wave> w;
    {
      std::lock_guard<std::mutex> g(wmu_);
      auto it = waves_.find(id);
      if (it == waves_.end()) return;
      w = std::move(it->second);
      waves_.erase(it);
    }
    recycle(std::move(w));
  }

  void drop_waves() {
    std::lock_guard<std::mutex> g(wmu_);
    for (auto& kv : waves_)
      if (kv.second->rolling) kv.second->worker.join();
    waves_.clear();
  }

  static int nchildren(int count, bool with_pass) {
    return with_pass ? count + 1 : (count == 0 ? 1 : count);
  }

  // edges of a leaf for its `count` sensible moves (PASS alone when there are none; PASS always,
  // with the network's pass prior pri[P], when `with_pass`), moves from `next_move()`, priors
  // renormalised over them; the kSorted highest priors first, in descending order (ties: lower
  // point first, pass last)
  template <class F>
  void fill_edges(size_t e0, int count, bool with_pass, const float* pri, int P, F&& next_move) {
    const int nc = nchildren(count, with_pass);
    Edge* E = &(*edges_)[e0];
    float tot = 0.f;
    for (int k = 0; k < nc; ++k) {
      const int mv = k < count ? next_move() : PASS;
      float p = 1.f;
      if (pri && mv != PASS) p = std::max(pri[mv], 0.f);
      if (pri && mv == PASS && with_pass) p = std::max(pri[P], 0.f);
      tot += p;
      E[k] = Edge{-1, p, (int16_t)mv, 0};
    }
    for (int k = 0; k < nc; ++k) E[k].prior = tot > 0.f ? E[k].prior / tot : 1.f / nc;
    auto before = [](const Edge& a, const Edge& b) {
      return a.prior > b.prior || (a.prior == b.prior && move_key(a.move) < move_key(b.move));
    };
    if (nc > kSorted) std::nth_element(E, E + kSorted, E + nc, before);
    std::sort(E, E + std::min(nc, (int)kSorted), before);
  }

  // v: value for the player to move at the leaf; a node at depth d stores it for its mover,
  // who is the leaf's player to move iff D-d is odd.
  void backup_value_path(const std::vector<int32_t>& path, float v, bool drop_vl) {
    const int D = (int)path.size() - 1;
    for (int d = D; d >= 0; --d) {
      Node& nd = (*nodes_)[path[d]];
      __atomic_fetch_add(&nd.n, 1, __ATOMIC_RELAXED);
      if (drop_vl) __atomic_fetch_sub(&nd.vl, 1, __ATOMIC_RELAXED);
      mcts_detail::atomic_addf(&nd.w, ((D - d) & 1) ? v : -v);
    }
  }
  // The same on the search's orchestrating thread while no descent runs: relaxed loads and
  // stores instead of read-modify-writes (rollout = the rollout statistics).
  void backup_path_serial(const std::vector<int32_t>& path, float v, bool drop_vl,
                          bool rollout) {
    const int D = (int)path.size() - 1;
    for (int d = D; d >= 0; --d) {
      Node& nd = (*nodes_)[path[d]];
      int32_t* cnt = rollout ? &nd.nr : &nd.n;
      float* sum = rollout ? &nd.wr : &nd.w;
      __atomic_store_n(cnt, __atomic_load_n(cnt, __ATOMIC_RELAXED) + 1, __ATOMIC_RELAXED);
      if (drop_vl)
        __atomic_store_n(&nd.vl, __atomic_load_n(&nd.vl, __ATOMIC_RELAXED) - 1, __ATOMIC_RELAXED);
      float f;
      __atomic_load(sum, &f, __ATOMIC_RELAXED);
      f += ((D - d) & 1) ? v : -v;
      __atomic_store(sum, &f, __ATOMIC_RELAXED);
    }
  }
  void backup_rollout_path(const std::vector<int32_t>& path, float z, bool drop_vl) {
    const int D = (int)path.size() - 1;
    for (int d = D; d >= 0; --d) {
      Node& nd = (*nodes_)[path[d]];
      __atomic_fetch_add(&nd.nr, 1, __ATOMIC_RELAXED);
      if (drop_vl) __atomic_fetch_sub(&nd.vl, 1, __ATOMIC_RELAXED);
      mcts_detail::atomic_addf(&nd.wr, ((D - d) & 1) ? z : -z);
    }
  }

  // copy the subtree under `keep` into fresh (recycled) arenas; children of a node keep their
  // edge order, nodes are renumbered breadth-first
  void compact(int keep) {
    auto nn = std::make_unique<mcts_detail::Arena<Node>>(kNodeCap);
    auto ne = std::make_unique<mcts_detail::Arena<Edge>>(kEdgeCap);
    std::vector<std::pair<int32_t, int32_t>> q;  // (old, new)
    auto copy_node = [&](int old) {
      const int nid = (int)nn->alloc(1);
      Node c = (*nodes_)[old];
      c.vl = 0;
      if (c.state == N_PENDING) c.state = N_NEW;
      (*nn)[nid] = c;
      q.emplace_back(old, nid);
      return nid;
    };
    copy_node(keep);
    for (size_t h = 0; h < q.size(); ++h) {
      const int old = q[h].first, nid = q[h].second;
      const Node o = (*nodes_)[old];
      if (o.state != N_EXPANDED || o.nedge == 0) continue;
      const size_t e0 = ne->alloc(o.nedge);
      (*nn)[nid].edges = (int32_t)e0;
      for (int k = 0; k < o.nedge; ++k) {
        Edge e = (*edges_)[o.edges + k];
        if (e.child >= 0) e.child = copy_node(e.child);
        (*ne)[e0 + k] = e;
      }
    }
    quiesce_prefault();  // the helper must not be inside the arenas that leave
    nodes_.swap(nn);
    edges_.swap(ne);
    root_ = 0;
    clear_root_external();  // the exchanged statistics were about the old root's children
    prefault();
  }

  // ------------------------------------------------------------------ page prefaulting
  // The helper thread keeps the pages just past each arena's allocation frontier resident.
  void prefault() {
    const size_t want_n = nodes_->bytes_used() + (size_t(8) << 20);
    const size_t want_e = edges_->bytes_used() + (size_t(48) << 20);
    if (nodes_->warm_bytes() >= want_n && edges_->warm_bytes() >= want_e) return;
    {
      std::lock_guard<std::mutex> g(pf_mu_);
      pf_nodes_ = nodes_.get();
      pf_edges_ = edges_.get();
      pf_want_n_ = want_n;
      pf_want_e_ = want_e;
      ++pf_gen_;
      if (!pf_thread_.joinable()) pf_thread_ = std::thread([this] { prefault_loop(); });
    }
    pf_cv_.notify_one();
  }
  void prefault_loop() {
    uint64_t seen = 0;
    while (true) {
      mcts_detail::Arena<Node>* an;
      mcts_detail::Arena<Edge>* ae;
      size_t wn, we;
      {
        std::unique_lock<std::mutex> lk(pf_mu_);
        pf_cv_.wait(lk, [&] { return pf_gen_ != seen || pf_stop_; });
        if (pf_stop_) return;
        seen = pf_gen_;
        an = pf_nodes_;
        ae = pf_edges_;
        wn = pf_want_n_;
        we = pf_want_e_;
        pf_busy_ = true;
      }
      if (an) an->populate(wn);
      if (ae) ae->populate(we);
      {
        std::lock_guard<std::mutex> g(pf_mu_);
        pf_busy_ = false;
      }
      pf_done_cv_.notify_all();
    }
  }
  // Arenas leave the search (compaction swaps, destruction) only when the helper is idle.
  void quiesce_prefault() {
    std::unique_lock<std::mutex> lk(pf_mu_);
    pf_done_cv_.wait(lk, [&] { return !pf_busy_; });
    pf_nodes_ = nullptr;
    pf_edges_ = nullptr;
  }
  void stop_prefault() {
    {
      std::lock_guard<std::mutex> g(pf_mu_);
      pf_stop_ = true;
    }
    pf_cv_.notify_all();
    if (pf_thread_.joinable()) pf_thread_.join();
  }

  Board root_board_;
  std::unique_ptr<mcts_detail::Arena<Node>> nodes_;
  std::unique_ptr<mcts_detail::Arena<Edge>> edges_;
  int root_ = 0;
  // waves_ / free_waves_ / next_wave_: select() may run on one host thread while another backs
  // an earlier wave up (the pipelined search); the tree itself is updated atomically
  mutable std::mutex wmu_;
  std::map<int, std::unique_ptr<Wave>> waves_;
  std::vector<std::unique_ptr<Wave>> free_waves_;
  int next_wave_ = 0;
  Pool pool_;                    // descents, leaf boards, expansions, backups
  std::unique_ptr<Pool> rpool_;  // CPU rollouts (run from a wave's worker thread)
  long sims_ = 0, rollouts_ = 0, terminal_ = 0;
  int collisions_ = 0;
  double t_descend_ = 0, t_build_ = 0, t_backup_ = 0;

  // external root statistics [4][P+1] (other ranks), this rank's last reported root totals
  std::vector<float> ext_, snap_;
  float ext_total_n_ = 0.f;
  bool has_ext_ = false;

  std::thread pf_thread_;
  std::mutex pf_mu_;
  std::condition_variable pf_cv_, pf_done_cv_;
  mcts_detail::Arena<Node>* pf_nodes_ = nullptr;
  mcts_detail::Arena<Edge>* pf_edges_ = nullptr;
  size_t pf_want_n_ = 0, pf_want_e_ = 0;
  uint64_t pf_gen_ = 0;
  bool pf_busy_ = false, pf_stop_ = false;
};

}  // namespace rag

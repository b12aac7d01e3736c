// Native APV-MCTS core (the reference's ParallelMCTS is an empty stub,
// AlphaGo/mcts.py:219-220, and its sequential MCTS is AlphaGo/mcts.py:79-216).
//
// Asynchronous policy-and-value MCTS in the AlphaGo style, restructured for a GPU evaluator:
// the search advances in *waves*. select(B) descends the tree B times with virtual loss, so the
// descents spread over different leaves, and returns the leaf positions. Their features are
// extracted natively (batch_features, threads), evaluated by the policy + value networks on the
// GPU in ONE batched launch sequence, and while the GPU works the fast-rollout playouts of the
// same leaves run on a native thread pool (start_rollouts / wait_rollouts). backup() expands the
// leaves with the network priors and backs up V = (1-lambda)*v + lambda*z with negamax signs,
// removing the virtual losses.
//
//   select:  a = argmax_a  Q(s,a) + c_puct * P(s,a) * sqrt(N(s)) / (1 + N(s,a))
//            with n_vl virtual losses per in-flight descent: N += n_vl, W -= n_vl
//   values:  from the perspective of the player to move at the leaf; W(s,a) is stored for the
//            player who played a.
//
// Children are created for the leaf's sensible moves (legal, not an own true eye — the same
// set the players use) with priors renormalised over them; PASS is the only child when no
// sensible move exists. Terminal leaves (end of game) are scored exactly and backed up at once.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <cmath>
#include <memory>
#include <thread>
#include <vector>

#include "../engine/go_engine.hpp"
#include "rollout.hpp"

namespace py = pybind11;

namespace rag {

namespace {

enum : uint8_t { N_NEW = 0, N_PENDING = 1, N_EXPANDED = 2 };

struct Node {
  int32_t parent;
  int32_t first;   // first child (children are contiguous)
  int16_t nchild;
  int16_t move;    // flat index, PASS = -1
  float prior;
  int32_t n;       // completed visits
  int32_t vl;      // in-flight descents through this node
  float w;         // value sum for the player who played `move`
  uint8_t state;
};

struct Leaf {
  Board board;
  std::vector<int32_t> path;  // root .. leaf
  float z = 0.f;
};

void parallel_for(int n, int nthreads, const std::function<void(int)>& fn) {
  if (nthreads <= 1 || n <= 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  nthreads = std::min(nthreads, n);
  std::atomic<int> next{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t)
    ts.emplace_back([&]() {
      for (int i = next++; i < n; i = next++) fn(i);
    });
  for (auto& t : ts) t.join();
}

}  // namespace

class Search {
 public:
  float c_puct = 5.f, lambda = 0.5f;
  int n_vl = 3, rollout_limit = 500, max_depth = 722, nthreads = 8;
  uint64_t seed = 1;
  std::shared_ptr<RolloutPolicy> rollout_policy;

  Search(const Board& root) : rollout_policy(std::make_shared<RolloutPolicy>()) { reset(root); }
  ~Search() { wait_rollouts(); }
  Search(const Search&) = delete;
  Search& operator=(const Search&) = delete;

  void reset(const Board& root) {
    root_board_ = root;
    nodes_.clear();
    nodes_.reserve(1 << 16);
    nodes_.push_back(Node{-1, -1, 0, (int16_t)PASS, 1.f, 0, 0, 0.f, N_NEW});
    root_ = 0;
    leaves_.clear();
  }

  const Board& root_board() const { return root_board_; }

  // ------------------------------------------------------------------ wave: select
  int select(int B) {
    if (rolling_) throw std::runtime_error("select() while rollouts are running");
    leaves_.clear();
    collisions_ = 0;
    int attempts = 0;
    const int P = root_board_.npoints();
    (void)P;
    while ((int)leaves_.size() < B && attempts < 4 * B) {
      ++attempts;
      Leaf L;
      L.board = root_board_;
      L.board.set_light(!root_board_.enforce_superko());
      int node = root_;
      L.path.push_back(node);
      int depth = 0;
      while (nodes_[node].state == N_EXPANDED && nodes_[node].nchild > 0 &&
             !L.board.end_of_game() && depth < max_depth) {
        node = select_child(node);
        L.board.play_unchecked(nodes_[node].move);
        L.path.push_back(node);
        ++depth;
      }
      if (L.board.end_of_game() || depth >= max_depth ||
          (nodes_[node].state == N_EXPANDED && nodes_[node].nchild == 0)) {
        const int win = L.board.get_winner();
        const int ptm = L.board.current_player();
        backup_path(L.path, win == 0 ? 0.f : (win == ptm ? 1.f : -1.f), ptm, false);
        ++terminal_;
        continue;
      }
      if (nodes_[node].state == N_PENDING) {  // already in this wave
        ++collisions_;
        continue;
      }
      nodes_[node].state = N_PENDING;
      for (int id : L.path) nodes_[id].vl += 1;
      leaves_.push_back(std::move(L));
    }
    return (int)leaves_.size();
  }

  int select_child(int p) const {
    const Node& pn = nodes_[p];
    const float np = (float)(pn.n + pn.vl * n_vl);
    const float sq = std::sqrt(std::max(np, 1.f));
    int best = pn.first;
    float bv = -1e30f;
    for (int k = 0; k < pn.nchild; ++k) {
      const Node& c = nodes_[pn.first + k];
      const float nv = (float)(c.n + c.vl * n_vl);
      const float q = nv > 0.f ? (c.w - (float)(c.vl * n_vl)) / nv : 0.f;
      const float v = q + c_puct * c.prior * sq / (1.f + nv);
      if (v > bv) {
        bv = v;
        best = pn.first + k;
      }
    }
    return best;
  }

  // ------------------------------------------------------------------ wave: leaf data
  int num_leaves() const { return (int)leaves_.size(); }
  const Board& leaf_board(int i) const { return leaves_.at(i).board; }

  // ------------------------------------------------------------------ wave: rollouts
  void start_rollouts() {
    if (rolling_) return;
    rolling_ = true;
    const uint64_t base = seed * 0x100000001B3ull + (wave_++) * 0x9E3779B9ull;
    worker_ = std::thread([this, base]() {
      parallel_for((int)leaves_.size(), nthreads, [&](int i) {
        Leaf& L = leaves_[i];
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

  void wait_rollouts() {
    if (!rolling_) return;
    worker_.join();
    rolling_ = false;
  }

  // ------------------------------------------------------------------ wave: backup
  // priors: [n][P] network move probabilities (nullptr => uniform); values: [n] (nullptr =>
  // rollouts only). Rollouts are used when lambda > 0.
  // Rollout outcomes computed elsewhere (the HIP rollout kernel): mean result per leaf from
  // BLACK's point of view (+1 black wins, -1 white wins, 0 draw).
  void set_rollout_results(const float* black_z) {
    wait_rollouts();
    for (size_t i = 0; i < leaves_.size(); ++i)
      leaves_[i].z = leaves_[i].board.current_player() == BLACK ? black_z[i] : -black_z[i];
    z_ready_ = true;
  }

  // Inputs of the GPU rollout kernel: colours [n][P] int8 and per-leaf meta
  // (player to move, ko, last move, second-to-last move, black passes, white passes,
  // moves played, end-of-game flag).
  void rollout_inputs(int8_t* colors, int32_t* meta) const {
    const int P = root_board_.npoints();
    for (size_t i = 0; i < leaves_.size(); ++i) {
      const Board& b = leaves_[i].board;
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

  void backup(const float* priors, int prior_stride, const float* values) {
    if (lambda > 0.f && !z_ready_) {
      if (!rolling_) start_rollouts();
      wait_rollouts();
    }
    std::vector<int> non_eye, eyes;
    for (size_t i = 0; i < leaves_.size(); ++i) {
      Leaf& L = leaves_[i];
      const int node = L.path.back();
      expand(node, L.board, priors ? priors + i * (size_t)prior_stride : nullptr, non_eye,
             eyes);
      float v;
      if (values == nullptr) v = L.z;
      else if (lambda <= 0.f) v = values[i];
      else v = (1.f - lambda) * values[i] + lambda * L.z;
      backup_path(L.path, v, L.board.current_player(), true);
    }
    sims_ += (long)leaves_.size();
    leaves_.clear();
    z_ready_ = false;
  }

  void expand(int node, const Board& b, const float* pri, std::vector<int>& non_eye,
              std::vector<int>& eyes) {
    Node& nd = nodes_[node];
    if (nd.state == N_EXPANDED) return;
    b.legal_moves(non_eye, eyes);
    const int first = (int)nodes_.size();
    const int nc = non_eye.empty() ? 1 : (int)non_eye.size();
    float tot = 0.f;
    for (int k = 0; k < nc; ++k) {
      const int mv = non_eye.empty() ? PASS : non_eye[k];
      float p = 1.f;
      if (pri && mv != PASS) p = std::max(pri[mv], 0.f);
      tot += p;
      nodes_.push_back(Node{node, -1, 0, (int16_t)mv, p, 0, 0, 0.f, N_NEW});
    }
    const float inv = tot > 0.f ? 1.f / tot : 1.f / nc;
    for (int k = 0; k < nc; ++k) {
      Node& c = nodes_[first + k];
      c.prior = tot > 0.f ? c.prior * inv : inv;
    }
    Node& nd2 = nodes_[node];  // nodes_ may have reallocated
    nd2.first = first;
    nd2.nchild = (int16_t)nc;
    nd2.state = N_EXPANDED;
  }

  // v: value for player `ptm` (to move at the leaf). Node values are for the mover into it.
  void backup_path(const std::vector<int32_t>& path, float v, int ptm, bool had_vl) {
    const int D = (int)path.size() - 1;
    for (int d = D; d >= 0; --d) {
      Node& nd = nodes_[path[d]];
      nd.n += 1;
      if (had_vl) nd.vl -= 1;
      // mover of the node at depth d is the player to move at the leaf iff D-d is odd
      nd.w += ((D - d) & 1) ? v : -v;
    }
    (void)ptm;
  }

  // ------------------------------------------------------------------ results / tree reuse
  int best_move() const {
    const Node& r = nodes_[root_];
    if (r.state != N_EXPANDED || r.nchild == 0) return PASS;
    int best = r.first;
    for (int k = 1; k < r.nchild; ++k)
      if (nodes_[r.first + k].n > nodes_[best].n) best = r.first + k;
    return nodes_[best].move;
  }

  py::tuple root_stats() const {
    const Node& r = nodes_[root_];
    const int nc = r.state == N_EXPANDED ? r.nchild : 0;
    py::array_t<int32_t> mv(nc), vis(nc);
    py::array_t<float> q(nc), pr(nc);
    for (int k = 0; k < nc; ++k) {
      const Node& c = nodes_[r.first + k];
      mv.mutable_data()[k] = c.move;
      vis.mutable_data()[k] = c.n;
      q.mutable_data()[k] = c.n ? c.w / c.n : 0.f;
      pr.mutable_data()[k] = c.prior;
    }
    return py::make_tuple(mv, vis, q, pr);
  }

  // Re-root at the child reached by `move` (played on the root board). Returns true when the
  // subtree was kept.
  bool advance(int move) {
    if (rolling_) throw std::runtime_error("advance() while rollouts are running");
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
  long terminal() const { return terminal_; }
  int collisions() const { return collisions_; }
  size_t num_nodes() const { return nodes_.size(); }
  int root_visits() const { return nodes_[root_].n; }

 private:
  // copy the subtree under `keep` into a fresh pool (BFS keeps children contiguous)
  void compact(int keep) {
    std::vector<Node> out;
    out.reserve(std::max<size_t>(nodes_.size() / 4, 1 << 16));
    std::vector<int32_t> q{keep};
    Node r = nodes_[keep];
    r.parent = -1;
    r.state = nodes_[keep].state == N_PENDING ? N_NEW : nodes_[keep].state;
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
  std::vector<Node> nodes_;
  int root_ = 0;
  std::vector<Leaf> leaves_;
  std::thread worker_;
  bool rolling_ = false;
  bool z_ready_ = false;
  uint64_t wave_ = 0;
  long sims_ = 0, terminal_ = 0;
  int collisions_ = 0;
};

void register_search(py::module_& m) {
  py::class_<Search>(m, "Search")
      .def(py::init<const Board&>(), py::arg("root"))
      .def("reset", &Search::reset)
      .def_readwrite("c_puct", &Search::c_puct)
      .def_readwrite("lmbda", &Search::lambda)
      .def_readwrite("n_vl", &Search::n_vl)
      .def_readwrite("rollout_limit", &Search::rollout_limit)
      .def_readwrite("max_depth", &Search::max_depth)
      .def_readwrite("nthreads", &Search::nthreads)
      .def_readwrite("seed", &Search::seed)
      .def("set_rollout_policy",
           [](Search& s, std::shared_ptr<RolloutPolicy> p) { s.rollout_policy = p; })
      .def("select", &Search::select, py::arg("batch"))
      .def("num_leaves", &Search::num_leaves)
      .def("leaf_boards",
           [](const Search& s) {
             std::vector<const Board*> v;
             for (int i = 0; i < s.num_leaves(); ++i) v.push_back(&s.leaf_board(i));
             return v;
           },
           py::return_value_policy::reference_internal)
      .def("start_rollouts", &Search::start_rollouts)
      .def("wait_rollouts", &Search::wait_rollouts, py::call_guard<py::gil_scoped_release>())
      .def("backup",
           [](Search& s, py::object priors, py::object values) {
             const float* pp = nullptr;
             const float* vp = nullptr;
             int stride = 0;
             py::array_t<float, py::array::c_style | py::array::forcecast> pa, va;
             const int n = s.num_leaves();
             if (!priors.is_none()) {
               pa = py::array_t<float, py::array::c_style | py::array::forcecast>(priors);
               if (pa.ndim() != 2 || pa.shape(0) < n ||
                   pa.shape(1) < s.root_board().npoints())
                 throw std::invalid_argument("priors must be [num_leaves, S*S]");
               pp = pa.data();
               stride = (int)pa.shape(1);
             }
             if (!values.is_none()) {
               va = py::array_t<float, py::array::c_style | py::array::forcecast>(values);
               if (va.size() < n) throw std::invalid_argument("values must be [num_leaves]");
               vp = va.data();
             }
             py::gil_scoped_release nogil;
             s.backup(pp, stride, vp);
           },
           py::arg("priors") = py::none(), py::arg("values") = py::none())
      .def("set_rollout_results",
           [](Search& s, py::array_t<float, py::array::c_style | py::array::forcecast> z) {
             if (z.size() < s.num_leaves()) throw std::invalid_argument("need one z per leaf");
             s.set_rollout_results(z.data());
           })
      .def("rollout_inputs",
           [](const Search& s) {
             const int n = s.num_leaves(), P = s.root_board().npoints();
             py::array_t<int8_t> c({n, P});
             py::array_t<int32_t> m({n, 8});
             s.rollout_inputs(c.mutable_data(), m.mutable_data());
             return py::make_tuple(c, m);
           })
      .def("best_move", &Search::best_move)
      .def("root_stats", &Search::root_stats)
      .def("advance", &Search::advance)
      .def_property_readonly("sims", &Search::sims)
      .def_property_readonly("terminal", &Search::terminal)
      .def_property_readonly("collisions", &Search::collisions)
      .def_property_readonly("num_nodes", &Search::num_nodes)
      .def_property_readonly("root_visits", &Search::root_visits)
      .def_property_readonly("root_board", &Search::root_board,
                             py::return_value_policy::reference_internal);
}

void register_rollout(py::module_& m) {
  py::class_<RolloutPolicy, std::shared_ptr<RolloutPolicy>>(m, "RolloutPolicy")
      .def(py::init<>())
      .def_property(
          "weights",
          [](const RolloutPolicy& p) {
            py::array_t<float> a(RF_COUNT);
            std::copy(p.w, p.w + RF_COUNT, a.mutable_data());
            return a;
          },
          [](RolloutPolicy& p, py::array_t<float, py::array::c_style | py::array::forcecast> a) {
            if (a.size() != RF_COUNT) throw std::invalid_argument("bad weight count");
            std::copy(a.data(), a.data() + RF_COUNT, p.w);
          })
      .def_property(
          "pattern",
          [](const RolloutPolicy& p) {
            py::array_t<float> a(RP_PATTERNS);
            std::copy(p.pattern.begin(), p.pattern.end(), a.mutable_data());
            return a;
          },
          [](RolloutPolicy& p, py::array_t<float, py::array::c_style | py::array::forcecast> a) {
            if (a.size() != RP_PATTERNS) throw std::invalid_argument("bad pattern count");
            std::copy(a.data(), a.data() + RP_PATTERNS, p.pattern.begin());
          })
      .def("candidates",
           [](const RolloutPolicy& p, const Board& b) {
             std::vector<int> mv(MAXP);
             std::vector<uint8_t> fb(MAXP);
             std::vector<int32_t> pt(MAXP);
             const int n = p.candidates(b, mv.data(), fb.data(), pt.data());
             py::array_t<int32_t> m(n), pp(n);
             py::array_t<uint8_t> f(n);
             std::copy(mv.begin(), mv.begin() + n, m.mutable_data());
             std::copy(fb.begin(), fb.begin() + n, f.mutable_data());
             std::copy(pt.begin(), pt.begin() + n, pp.mutable_data());
             return py::make_tuple(m, f, pp);
           })
      .def("sample",
           [](const RolloutPolicy& p, const Board& b, uint64_t seed) {
             Rng rng(seed);
             std::vector<int> mv(MAXP);
             std::vector<float> pr(MAXP);
             return p.sample(b, rng, mv.data(), pr.data());
           })
      .def("rollout",
           [](const RolloutPolicy& p, const Board& b, uint64_t seed, int limit) {
             Board c = b;
             c.set_enforce_superko(false);
             Rng rng(seed);
             const int w = p.rollout(c, rng, limit);
             return py::make_tuple(w, c.nmoves() - b.nmoves());
           },
           py::arg("board"), py::arg("seed") = 1, py::arg("limit") = 500)
      .def("rollouts",
           [](const RolloutPolicy& p, const std::vector<const Board*>& boards, uint64_t seed,
              int limit, int nthreads) {
             const int n = (int)boards.size();
             py::array_t<int8_t> out(n);
             int8_t* o = out.mutable_data();
             {
               py::gil_scoped_release nogil;
               parallel_for(n, nthreads, [&](int i) {
                 Board c = *boards[i];
                 c.set_enforce_superko(false);
                 Rng rng(seed + (uint64_t)i * 7919ull);
                 o[i] = (int8_t)p.rollout(c, rng, limit);
               });
             }
             return out;
           },
           py::arg("boards"), py::arg("seed") = 1, py::arg("limit") = 500,
           py::arg("nthreads") = 8);
  m.attr("ROLLOUT_FEATURES") = py::int_((int)RF_COUNT);
  m.attr("ROLLOUT_PATTERNS") = py::int_((int)RP_PATTERNS);
}

}  // namespace rag

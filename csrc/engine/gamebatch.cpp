// Native self-play game batch (RL policy training, value-dataset generation): N boards that
// advance in lock-step, one call per ply for all of them on the thread pool.
//
// The reference plays its games in a Python loop over GameState objects — per ply, every game's
// features are extracted in Python and `do_move` is called game by game
// (AlphaGo/training/reinforcement_policy_trainer.py:51-75, AlphaGo/ai.py:107-133). Here the
// boards stay native: pack() writes the feature-kernel inputs of the games to move straight into
// pinned buffers, play() applies a whole ply (the moves the GPU sampler chose) in parallel, and
// only the per-game move lists / winners come back to Python.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <memory>
#include <vector>

#include "go_engine.hpp"
#include "pack.hpp"
#include "pyviews.hpp"
#include "thread_pool.hpp"

namespace py = pybind11;

namespace rag {

std::shared_ptr<const Zobrist> make_zobrist(py::array_t<uint64_t, py::array::c_style> w,
                                            py::array_t<uint64_t, py::array::c_style> b);

class GameBatch {
 public:
  GameBatch(int n, int size, double komi, bool superko, std::shared_ptr<const Zobrist> zob,
            int nthreads)
      : pool_(std::max(1, nthreads)) {
    boards_.reserve(n);
    for (int i = 0; i < n; ++i) boards_.emplace_back(size, komi, superko, zob);
    done_.assign(n, 0);
  }
  int size() const { return (int)boards_.size(); }
  Board& board(int i) {
    if (i < 0 || i >= size()) throw std::out_of_range("game index");
    return boards_[i];
  }
  std::vector<int32_t> active() const {
    std::vector<int32_t> v;
    for (int i = 0; i < size(); ++i)
      if (!done_[i]) v.push_back(i);
    return v;
  }
  void check(const int32_t* idx, int n) const {
    for (int k = 0; k < n; ++k)
      if (idx[k] < 0 || idx[k] >= size()) throw std::out_of_range("game index");
  }
  void pack(const int32_t* idx, int n, const PackOut& o) {
    pool_.run(n, [&](int k) { pack_board(boards_[idx[k]], k, o); });
  }
  // One ply: game idx[k] plays moves[k] (flat point, -1 = pass). Over `move_limit` moves
  // (reference ai.py: len(history) > move_limit) a game passes; a move that is not legal
  // (cannot come from the sensible-move sampler) is played as a pass and counted. Returns the
  // number of games still unfinished among idx.
  int play(const int32_t* idx, const int32_t* moves, int n, int move_limit, int32_t* played) {
    std::atomic<int> live{0};
    pool_.run(n, [&](int k) {
      Board& b = boards_[idx[k]];
      int a = moves[k];
      if (move_limit >= 0 && b.move_count() > move_limit) a = PASS;
      if (a != PASS && (a < 0 || a >= b.npoints() || !b.is_legal(a))) {
        a = PASS;
        illegal_.fetch_add(1, std::memory_order_relaxed);
      }
      b.do_move(a, 0);
      if (played) played[k] = a;
      if (b.end_of_game())
        done_[idx[k]] = 1;
      else
        live.fetch_add(1, std::memory_order_relaxed);
    });
    return live.load();
  }
  long illegal() const { return illegal_.load(); }
  void winners(int8_t* out) {
    pool_.run(size(), [&](int i) { out[i] = (int8_t)boards_[i].get_winner(); });
  }

 private:
  std::vector<Board> boards_;
  std::vector<uint8_t> done_;
  Pool pool_;
  std::atomic<long> illegal_{0};
};

void register_gamebatch(py::module_& m) {
  using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
  py::class_<GameBatch>(m, "GameBatch")
      .def(py::init([](int n, int size, double komi, bool superko,
                       py::array_t<uint64_t, py::array::c_style> zw,
                       py::array_t<uint64_t, py::array::c_style> zb, int nthreads) {
             return std::make_unique<GameBatch>(n, size, komi, superko, make_zobrist(zw, zb),
                                                nthreads);
           }),
           py::arg("n"), py::arg("size"), py::arg("komi"), py::arg("superko"),
           py::arg("zobrist_white"), py::arg("zobrist_black"), py::arg("nthreads") = 8)
      .def("__len__", &GameBatch::size)
      .def("board", &GameBatch::board, py::return_value_policy::reference_internal)
      .def("active",
           [](const GameBatch& g) {
             auto v = g.active();
             return py::array_t<int32_t>((py::ssize_t)v.size(), v.data());
           })
      .def("pack",
           [](GameBatch& g, I32 idx, py::object colors, py::object ages, py::object meta4,
              py::object ladders, py::object illegal) {
             const int n = (int)idx.size();
             g.check(idx.data(), n);
             const size_t P = n ? (size_t)g.board(idx.data()[0]).npoints() : 0;
             PackOut o;
             o.colors = out_view<int8_t>(colors, n, P, o.s_colors, "colors");
             o.ages = out_view<int16_t>(ages, n, P, o.s_ages, "ages");
             o.meta4 = out_view<int32_t>(meta4, n, 4, o.s_meta4, "meta4");
             o.ladders = out_view<uint8_t>(ladders, n, 2 * P, o.s_ladders, "ladders");
             o.illegal = out_view<uint8_t>(illegal, n, P, o.s_illegal, "illegal");
             py::gil_scoped_release nogil;
             g.pack(idx.data(), n, o);
           },
           py::arg("idx"), py::arg("colors") = py::none(), py::arg("ages") = py::none(),
           py::arg("meta4") = py::none(), py::arg("ladders") = py::none(),
           py::arg("illegal") = py::none(),
           "Feature-kernel inputs of games idx into caller arrays [len(idx), ...]")
      .def("play",
           [](GameBatch& g, I32 idx, I32 moves, int move_limit) {
             const int n = (int)idx.size();
             if (moves.size() < n) throw std::invalid_argument("one move per game");
             g.check(idx.data(), n);
             py::array_t<int32_t> played(n);
             int live;
             {
               py::gil_scoped_release nogil;
               live = g.play(idx.data(), moves.data(), n, move_limit, played.mutable_data());
             }
             return py::make_tuple(live, played);
           },
           py::arg("idx"), py::arg("moves"), py::arg("move_limit") = -1,
           "Apply one ply (flat moves, -1 pass) to games idx; returns (unfinished, played)")
      .def_property_readonly("illegal", &GameBatch::illegal)
      .def("winners", [](GameBatch& g) {
        py::array_t<int8_t> out(g.size());
        {
          py::gil_scoped_release nogil;
          g.winners(out.mutable_data());
        }
        return out;
      });
}

}  // namespace rag

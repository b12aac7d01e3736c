// Python bindings of the native APV-MCTS (search.hpp) and the fast rollout policy.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "../engine/pyviews.hpp"
#include "search.hpp"

namespace py = pybind11;

namespace rag {

namespace {
using FArr = py::array_t<float, py::array::c_style | py::array::forcecast>;

}  // namespace

void register_search(py::module_& m) {
  m.def("trim_tree_cache", [] { return rag::mcts_detail::MapCache::get().trim(); },
        "unmap the cached (warm) tree arenas kept for the next Search; returns the bytes freed");
  m.def("tree_cache_bytes", [] { return rag::mcts_detail::MapCache::get().cached_bytes(); });
  py::class_<Search>(m, "Search")
      .def(py::init<const Board&, int>(), py::arg("root"), py::arg("nthreads") = 8)
      .def("reset", &Search::reset)
      .def_readwrite("c_puct", &Search::c_puct)
      .def_readwrite("lmbda", &Search::lambda)
      .def_readwrite("n_vl", &Search::n_vl)
      .def_readwrite("rollout_limit", &Search::rollout_limit)
      .def_readwrite("max_depth", &Search::max_depth)
      .def_readwrite("seed", &Search::seed)
      .def_readwrite("keyed_rollouts", &Search::keyed_rollouts)
      .def_property_readonly("nthreads", &Search::nthreads)
      .def("set_rollout_policy",
           [](Search& s, std::shared_ptr<RolloutPolicy> p) { s.rollout_policy = p; })
      .def("select", &Search::select, py::arg("batch"), py::arg("build") = true,
           py::call_guard<py::gil_scoped_release>(),
           "(wave id, leaves); build=False: no leaf boards (the leaves ship as move paths)")
      .def("write_paths",
           [](Search& s, int id, int stride) {
             const int n = s.num_leaves(id);
             py::array_t<int16_t> a({n, stride});
             s.write_paths(id, 0, n, a.mutable_data(), stride);
             return a;
           },
           py::arg("wave"), py::arg("stride") = 64,
           "[n, stride] int16 path records (depth, moves from the root) of a wave's leaves")
      .def("load_paths",
           [](Search& s, py::array_t<int16_t, py::array::c_style | py::array::forcecast> recs) {
             if (recs.ndim() != 2) throw std::invalid_argument("path records must be [n, stride]");
             const int n = (int)recs.shape(0), stride = (int)recs.shape(1);
             const int16_t* p = recs.data();
             py::gil_scoped_release nogil;
             return s.load_paths(p, n, stride);
           },
           "A wave of leaf boards rebuilt from path records (root board + moves); returns its id")
      .def("rollout_black_z",
           [](Search& s, int id) {
             py::array_t<float> a(s.num_leaves(id));
             float* o = a.mutable_data();
             {
               py::gil_scoped_release nogil;
               s.rollout_black_z(id, o);
             }
             return a;
           },
           "CPU rollout results of a wave (start_rollouts) from BLACK's point of view")
      .def("drop_wave", &Search::drop_wave, py::call_guard<py::gil_scoped_release>())
      .def_readwrite("parallel_select_min", &Search::parallel_select_min)
      .def_readwrite("batched_select", &Search::batched_select,
                     "waves of >= parallel_select_min leaves deal their descents top-down")
      .def_readwrite("pass_prior", &Search::pass_prior)
      .def("leaf_nodes",
           [](Search& s, int id) {
             std::vector<int32_t> v;
             for (const Leaf& L : s.wave(id).leaves) v.push_back(L.path.back());
             return v;
           })
      .def("num_leaves", &Search::num_leaves)
      .def("leaf_boards", &Search::leaf_boards, py::return_value_policy::reference_internal)
      .def("backup_value",
           [](Search& s, int id, py::object priors, py::object values, py::object sensible) {
             const int n = s.num_leaves(id);
             const uint8_t* sp = nullptr;
             py::array_t<uint8_t, py::array::c_style | py::array::forcecast> sa;
             if (!sensible.is_none()) {
               sa = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>(sensible);
               if (sa.size() < (py::ssize_t)n * s.root_board().npoints())
                 throw std::invalid_argument("sensible must be [num_leaves, S*S]");
               sp = sa.data();
             }
             const float* pp = nullptr;
             const float* vp = nullptr;
             int stride = 0;
             FArr pa, va;
             if (!priors.is_none()) {
               pa = FArr(priors);
               if (pa.ndim() != 2 || pa.shape(0) < n || pa.shape(1) < s.root_board().npoints())
                 throw std::invalid_argument("priors must be [num_leaves, S*S]");
               pp = pa.data();
               stride = (int)pa.shape(1);
             }
             if (!values.is_none()) {
               va = FArr(values);
               if (va.size() < n) throw std::invalid_argument("values must be [num_leaves]");
               vp = va.data();
             }
             py::gil_scoped_release nogil;
             s.backup_value(id, pp, stride, vp, sp);
           },
           py::arg("wave"), py::arg("priors") = py::none(), py::arg("values") = py::none(),
           py::arg("sensible") = py::none())
      .def("rollout_inputs",
           [](Search& s, int id) {
             const int n = s.num_leaves(id), P = s.root_board().npoints();
             py::array_t<int8_t> c({n, P});
             py::array_t<int32_t> m({n, 8});
             s.rollout_inputs(id, c.mutable_data(), m.mutable_data());
             return py::make_tuple(c, m);
           })
      .def("pack_inputs",
           [](Search& s, int id, py::object colors, py::object ages, py::object meta4,
              py::object meta8, py::object illegal, py::object ladders) {
             const int n = s.num_leaves(id);
             const size_t P = (size_t)s.root_board().npoints();
             PackOut o;
             o.colors = out_view<int8_t>(colors, n, P, o.s_colors, "colors");
             o.ages = out_view<int16_t>(ages, n, P, o.s_ages, "ages");
             o.meta4 = out_view<int32_t>(meta4, n, 4, o.s_meta4, "meta4");
             o.meta8 = out_view<int32_t>(meta8, n, 8, o.s_meta8, "meta8");
             o.illegal = out_view<uint8_t>(illegal, n, P, o.s_illegal, "illegal");
             o.ladders = out_view<uint8_t>(ladders, n, 2 * P, o.s_ladders, "ladders");
             py::gil_scoped_release nogil;
             s.pack_inputs(id, o);
           },
           py::arg("wave"), py::arg("colors") = py::none(), py::arg("ages") = py::none(),
           py::arg("meta4") = py::none(), py::arg("meta8") = py::none(),
           py::arg("illegal") = py::none(), py::arg("ladders") = py::none(),
           "Write the wave's leaf inputs (feature-kernel colours / stone ages / meta, rollout "
           "meta8, superko-illegal masks, host ladder planes) into caller arrays [n, ...]")
      .def("backup_rollout",
           [](Search& s, int id, FArr z) {
             if (z.size() < s.num_leaves(id)) throw std::invalid_argument("need one z per leaf");
             py::gil_scoped_release nogil;
             s.backup_rollout(id, z.data());
           })
      .def("start_rollouts", &Search::start_rollouts)
      .def("finish_rollouts", &Search::finish_rollouts, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("pending_waves", &Search::pending_waves)
      .def("best_move", &Search::best_move)
      .def("expanded_keys",
           [](const Search& s) {
             const auto k = s.expanded_keys();
             py::array_t<uint64_t> a(k.size());
             std::copy(k.begin(), k.end(), a.mutable_data());
             return a;
           })
      .def("root_stats",
           [](const Search& s) {
             std::vector<int32_t> mv, vis;
             std::vector<float> q, pr;
             s.root_stats(mv, vis, q, pr);
             return py::make_tuple(py::array_t<int32_t>(mv.size(), mv.data()),
                                   py::array_t<int32_t>(vis.size(), vis.data()),
                                   py::array_t<float>(q.size(), q.data()),
                                   py::array_t<float>(pr.size(), pr.data()));
           })
      .def("advance", &Search::advance)
      .def_property_readonly("sims", &Search::sims)
      .def_property_readonly("rollouts", &Search::rollouts)
      .def_property_readonly("terminal", &Search::terminal)
      .def_property_readonly("collisions", &Search::collisions)
      .def_property_readonly("num_nodes", &Search::num_nodes)
      .def_property_readonly("num_edges", &Search::num_edges)
      .def("root_deltas",
           [](Search& s) {
             const int M = s.root_board().npoints() + 1;
             py::array_t<float> out({4, M});
             s.root_deltas(out.mutable_data());
             return out;
           },
           "[4, P+1] (visits, value sum, rollouts, rollout sum) this rank added at the root's "
           "children since the previous call (index P = pass)")
      .def("set_root_external",
           [](Search& s, FArr ext) {
             const int M = s.root_board().npoints() + 1;
             if (ext.size() != 4 * M) throw std::invalid_argument("external stats must be [4, P+1]");
             const float* e = ext.data();
             s.set_root_external(e, e + M, e + 2 * M, e + 3 * M);
           },
           "Other ranks' cumulative root-child statistics [4, P+1], mixed into root selection")
      .def("clear_root_external", &Search::clear_root_external)
      .def_property_readonly("timers", &Search::timers)

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
          [](RolloutPolicy& p, FArr a) {
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
          [](RolloutPolicy& p, FArr a) {
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
              int limit, int nthreads, bool keyed) {
             const int n = (int)boards.size();
             py::array_t<int8_t> out(n);
             int8_t* o = out.mutable_data();
             {
               py::gil_scoped_release nogil;
               shared_pool(std::max(1, std::min(nthreads, 64))).run(n, [&](int i) {
                 Board c = *boards[i];
                 c.set_enforce_superko(false);
                 Rng rng(keyed ? position_key_seed(c.hash(), c.current_player())
                               : seed + (uint64_t)i * 7919ull);
                 o[i] = (int8_t)p.rollout(c, rng, limit);
               });
             }
             return out;
           },
           py::arg("boards"), py::arg("seed") = 1, py::arg("limit") = 500,
           py::arg("nthreads") = 8, py::arg("keyed") = false,
           "Winner of one rollout per board; keyed: seeded by the board's position "
           "(position_key_seed) instead of seed and index");
  m.attr("ROLLOUT_FEATURES") = py::int_((int)RF_COUNT);
  m.attr("ROLLOUT_PATTERNS") = py::int_((int)RP_PATTERNS);
}

}  // namespace rag

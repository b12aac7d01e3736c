// Python bindings of the multi-GPU search channel and master loop (master.hpp).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "master.hpp"

namespace py = pybind11;

namespace rag {

void register_master(py::module_& m) {
  py::class_<ShmChannel>(m, "SearchChannel")
      .def(py::init<const std::string&, bool, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                    uint32_t>(),
           py::arg("name"), py::arg("create"), py::arg("nranks") = 0, py::arg("nslots") = 0,
           py::arg("cap") = 0, py::arg("P") = 0, py::arg("PW") = 0, py::arg("stride") = 0,
           "POSIX shared-memory channel of the multi-GPU search (create on the master, attach "
           "on the evaluating ranks)")
      .def_property_readonly("name", &ShmChannel::name)
      .def_property_readonly("nranks", &ShmChannel::nranks)
      .def_property_readonly("nslots", &ShmChannel::nslots)
      .def_property_readonly("cap", &ShmChannel::cap)
      .def_property_readonly("P", &ShmChannel::P)
      .def_property_readonly("PW", &ShmChannel::PW)
      .def_property_readonly("stride", &ShmChannel::stride)
      .def("unlink", &ShmChannel::unlink)
      .def(
          "view",
          [](py::object self, uint32_t r, uint32_t k, const std::string& what) -> py::array {
            ShmChannel& c = self.cast<ShmChannel&>();
            const py::ssize_t cap = c.cap();
            if (what == "paths")
              return py::array(py::dtype::of<int16_t>(), {cap, (py::ssize_t)c.stride()},
                               c.paths(r, k), self);
            if (what == "priors")
              return py::array(py::dtype::of<float>(), {cap, (py::ssize_t)c.PW()},
                               c.priors(r, k), self);
            if (what == "values")
              return py::array(py::dtype::of<float>(), {cap}, c.values(r, k), self);
            if (what == "sens")
              return py::array(py::dtype::of<uint8_t>(), {cap, (py::ssize_t)c.P()}, c.sens(r, k),
                               self);
            if (what == "z") return py::array(py::dtype::of<float>(), {cap}, c.z(r, k), self);
            if (what == "root_meta")
              return py::array(py::dtype::of<int64_t>(), {8}, c.root_meta(), self);
            if (what == "root_moves")
              return py::array(py::dtype::of<int16_t>(), {4096}, c.root_moves(), self);
            throw std::invalid_argument(
                "view: paths | priors | values | sens | z | root_meta | root_moves");
          },
          "numpy view (no copy) of one slot's section, shape [cap, ...]")
      .def("slot_info",
           [](const ShmChannel& c, uint32_t r, uint32_t k) {
             const SlotHead* s = c.slot(r, k);
             return py::make_tuple(s->req_seq.load(std::memory_order_acquire), s->n, s->wave,
                                   s->seed, s->root_hash);
           },
           "(request sequence, leaves, wave number, rollout seed, root hash) of a slot")
      .def("wait_request", &ShmChannel::wait_request, py::arg("rank"), py::arg("slot"),
           py::arg("last_req"), py::arg("last_cmd"), py::arg("timeout_us") = 100,
           py::call_guard<py::gil_scoped_release>(),
           "1: a new request in the slot, 2: a new command, 0: timed out")
      .def("post_values", &ShmChannel::post_values)
      .def("post_z", &ShmChannel::post_z)
      .def("post_cmd", &ShmChannel::post_cmd)
      .def("cmd",
           [](const ShmChannel& c) {
             const ChanHead* h = c.head();
             const uint32_t s = h->cmd_seq.load(std::memory_order_acquire);
             return py::make_tuple(s, h->cmd, h->arg);
           })
      .def("abort", &ShmChannel::set_abort)
      .def_property_readonly("aborted", &ShmChannel::aborted)
      .def_property_readonly("why", &ShmChannel::why);
  m.attr("CHAN_CMD_MOVE") = (int)ShmChannel::CMD_MOVE;
  m.attr("CHAN_CMD_STOP") = (int)ShmChannel::CMD_STOP;

  m.def(
      "run_master",
      [](Search& s, ShmChannel& ch, std::vector<int> batch, int depth, int nslots, long budget,
         uint32_t seed, double stall_s) {
        MasterConfig cfg;
        cfg.batch = std::move(batch);
        cfg.depth = depth;
        cfg.nslots = nslots;
        cfg.budget = budget;
        cfg.seed = seed;
        cfg.stall_s = stall_s;
        MasterStats st;
        {
          py::gil_scoped_release nogil;
          st = run_master(s, ch, cfg);
        }
        py::dict d;
        d["waves"] = st.waves;
        d["sims"] = st.sims;
        d["rollout_waves"] = st.rollout_waves;
        d["empty_selects"] = st.empty_selects;
        d["t_select"] = st.t_select;
        d["t_ship"] = st.t_ship;
        d["t_value"] = st.t_value;
        d["t_rollout"] = st.t_rollout;
        d["t_idle"] = st.t_idle;
        d["wall"] = st.wall;
        d["leaves"] = st.leaves;
        d["max_inflight"] = st.max_inflight;
        return d;
      },
      py::arg("search"), py::arg("channel"), py::arg("batch"), py::arg("depth") = 2,
      py::arg("nslots") = 8, py::arg("budget") = 0, py::arg("seed") = 1,
      py::arg("stall_s") = 120.0,
      "The multi-GPU search's master loop (master.hpp): select / ship / back up waves of the "
      "tree over the channel until `budget` simulations were added. GIL released.");
}

}  // namespace rag

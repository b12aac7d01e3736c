// placeholder: APV-MCTS bindings are registered here (filled in by the search milestone)
#include <pybind11/pybind11.h>
namespace py = pybind11;
namespace rag {
void register_search(py::module_& m) {}
void register_rollout(py::module_& m) {}
}  // namespace rag

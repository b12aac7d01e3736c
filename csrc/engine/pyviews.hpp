// numpy output views for the packing entry points (search.cpp, gamebatch.cpp).
#pragma once
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

namespace rag {

// A writable [n, ...] output view: dtype itemsize sizeof(T), at least `row` items per row,
// contiguous within a row (rows may be strided, e.g. columns of a record array). None -> null.
template <class T>
T* out_view(pybind11::object o, int n, size_t row, size_t& stride, const char* what) {
  namespace py = pybind11;
  if (o.is_none()) return nullptr;
  py::array a = py::reinterpret_borrow<py::array>(o);
  if (!a.writeable()) throw std::invalid_argument(std::string(what) + ": not writeable");
  if (a.itemsize() != (py::ssize_t)sizeof(T))
    throw std::invalid_argument(std::string(what) + ": wrong dtype");
  if (a.ndim() < 2 || a.shape(0) < n)
    throw std::invalid_argument(std::string(what) + ": need [n, ...]");
  size_t inner = 1;
  for (py::ssize_t d = 1; d < a.ndim(); ++d) inner *= (size_t)a.shape(d);
  if (inner < row) throw std::invalid_argument(std::string(what) + ": rows too short");
  py::ssize_t expect = (py::ssize_t)sizeof(T);
  for (py::ssize_t d = a.ndim() - 1; d >= 1; --d) {
    if (a.shape(d) > 1 && a.strides(d) != expect)
      throw std::invalid_argument(std::string(what) + ": rows must be contiguous");
    expect *= a.shape(d);
  }
  stride = (size_t)a.strides(0);
  return static_cast<T*>(a.mutable_data());
}

}  // namespace rag

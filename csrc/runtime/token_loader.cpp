// Python binding of the native token loader (csrc/runtime/token_loader.h) -> finetune_controller_amd/_rt.so
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "token_loader.h"

namespace py = pybind11;
using ftc_rt::TokenLoader;

PYBIND11_MODULE(_rt, m) {
  m.doc() = "finetune_controller_amd native runtime: prefetching memory-mapped token loader";
  py::class_<TokenLoader>(m, "TokenLoader")
      .def(py::init<const std::string&, int, int64_t, int64_t, int, int, int, int64_t, int64_t>(), py::arg("path"),
           py::arg("itemsize"), py::arg("seq_len"), py::arg("batch"), py::arg("rank"), py::arg("world"),
           py::arg("threads") = 2, py::arg("offset") = 0, py::arg("vocab") = 0)
      .def_property_readonly("n_windows", &TokenLoader::n_windows)
      .def_property_readonly("n_tokens", &TokenLoader::n_tokens)
      .def("set_buffers", &TokenLoader::set_buffers)
      .def("start",
           [](TokenLoader& self, py::array_t<int64_t, py::array::c_style | py::array::forcecast> order, int64_t first,
              int64_t last) { self.start(order.data(), (size_t)order.size(), first, last); })
      .def("acquire", &TokenLoader::acquire, py::call_guard<py::gil_scoped_release>())
      .def("release", &TokenLoader::release)
      .def("stop", &TokenLoader::stop, py::call_guard<py::gil_scoped_release>());
}

// pybind11 module `_host`: the native host runtime of the framework.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "crc32c.h"

namespace py = pybind11;

void register_bundle(py::module_& m);
void register_events(py::module_& m);
void register_ps(py::module_& m);

PYBIND11_MODULE(_host, m) {
  m.doc() = "native host runtime: CRC32C, TF-V2 checkpoints, TFRecord events, TCP parameter server";
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return dtfx_host::crc32c(s.data(), s.size());
  });
  m.def("crc32c_extend", [](uint32_t crc, py::bytes b) {
    std::string s = b;
    return dtfx_host::crc32c_extend(crc, s.data(), s.size());
  });
  m.def("crc32c_sw", [](py::bytes b) {
    std::string s = b;
    return dtfx_host::crc32c_extend_sw(0, reinterpret_cast<const uint8_t*>(s.data()), s.size());
  });
  m.def("crc32c_mask", &dtfx_host::crc32c_mask);
  m.def("crc32c_unmask", &dtfx_host::crc32c_unmask);
  register_bundle(m);
  register_events(m);
  register_ps(m);
}

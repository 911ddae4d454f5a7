// module.cpp — pybind11 module `_ss_host` (host runtime).
#include <pybind11/pybind11.h>

#include "ss/hash.h"

namespace py = pybind11;

PYBIND11_MODULE(_ss_host, m) {
  m.doc() = "SwiftSnails-AMD host runtime";
  m.def("fmix64", &ss::fmix64);
}

#include <pybind11/pybind11.h>
namespace py = pybind11;
namespace mxar {
void bind_hip(py::module_& m) { (void)m; }
}  // namespace mxar

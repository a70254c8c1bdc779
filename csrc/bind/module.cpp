// imitation_amd._C — module definition.
#include "common.h"

void register_io(py::module& m);      // io.cpp
void register_events(py::module& m);  // events.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "imitation_amd native runtime + HIP/CDNA4 kernels (gfx950)";
  m.attr("arch") = "gfx950";
  register_envs(m);
  register_kernels(m);
  register_engine(m);
  register_disc(m);
  register_airl(m);
  register_wide(m);
  register_conv(m);
  register_comm(m);
  register_pref(m);
  register_io(m);
  register_events(m);
}

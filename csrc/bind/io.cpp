// Host I/O runtime bindings: TensorBoard event encoding (csrc/runtime/tb_events.cpp).
#include "common.h"

namespace ia {
uint32_t crc32c(const uint8_t* p, size_t n);
uint32_t masked_crc32c(const uint8_t* p, size_t n);
std::string tb_scalar_records(double wall_time, int64_t step, const std::vector<std::string>& tags,
                              const std::vector<float>& values);
}  // namespace ia

void register_io(py::module& m) {
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return ia::crc32c((const uint8_t*)s.data(), s.size());
  });
  m.def("masked_crc32c", [](py::bytes b) {
    std::string s = b;
    return ia::masked_crc32c((const uint8_t*)s.data(), s.size());
  });
  m.def(
      "tb_scalar_records",
      [](double wall_time, long long step, const std::vector<std::string>& tags, const std::vector<float>& values) {
        std::string out;
        {
          py::gil_scoped_release nogil;
          out = ia::tb_scalar_records(wall_time, (int64_t)step, tags, values);
        }
        return py::bytes(out);
      },
      "Framed TFRecords of Event{wall_time, step, Summary{Value{tag, simple_value}}}, one per scalar");
}

// Torch-facing wrappers of the one-shot all-reduce (comm.hip).  Regions are passed around
// as integer device addresses; the Python communicator (parallel/oneshot.py) owns them.
#include "common.h"
#include "launchers.h"

namespace {

#define IA_HIP_CHECK(expr)                                                            \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e)); \
  } while (0)

py::tuple oneshot_alloc(int64_t stage_bytes) {
  TORCH_CHECK(stage_bytes > 0 && stage_bytes % 16 == 0, "stage_bytes must be a positive multiple of 16");
  void* p = nullptr;
  std::string h(ia::oneshot_handle_bytes(), '\0');
  IA_HIP_CHECK(ia::oneshot_alloc((size_t)stage_bytes, &p, &h[0]));
  return py::make_tuple((int64_t)reinterpret_cast<uintptr_t>(p), py::bytes(h));
}

int64_t oneshot_open(py::bytes handle) {
  std::string h = handle;
  TORCH_CHECK(h.size() == ia::oneshot_handle_bytes(), "bad IPC handle size");
  void* p = nullptr;
  IA_HIP_CHECK(ia::oneshot_open(h.data(), &p));
  return (int64_t)reinterpret_cast<uintptr_t>(p);
}

void oneshot_allreduce(const std::vector<int64_t>& bases, int64_t rank, torch::Tensor in, torch::Tensor out, double scale,
                       int64_t stage_bytes, double timeout_s) {
  TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous(), "contiguous GPU tensors");
  TORCH_CHECK(in.scalar_type() == out.scalar_type() &&
                  (in.scalar_type() == torch::kFloat32 || in.scalar_type() == torch::kFloat64),
              "float32 or float64 in/out of one dtype");
  TORCH_CHECK(in.numel() == out.numel(), "in/out size mismatch");
  TORCH_CHECK(!bases.empty() && bases.size() <= (size_t)ia::kOneShotMaxRanks, "1..8 ranks");
  TORCH_CHECK(rank >= 0 && rank < (int64_t)bases.size(), "rank out of range");
  TORCH_CHECK((size_t)in.numel() * in.element_size() <= (size_t)stage_bytes, "bucket larger than the staging slot");
  TORCH_CHECK(((uintptr_t)in.data_ptr() | (uintptr_t)out.data_ptr()) % 16 == 0, "in/out must be 16-B aligned");
  ia::OneShotArgs a{};
  for (size_t r = 0; r < bases.size(); ++r) a.base[r] = reinterpret_cast<char*>((uintptr_t)bases[r]);
  a.in = in.data_ptr();
  a.out = out.data_ptr();
  a.n = (int)in.numel();
  a.rank = (int)rank;
  a.world = (int)bases.size();
  a.f64 = in.scalar_type() == torch::kFloat64;
  a.scale = scale;
  a.stage_bytes = (size_t)stage_bytes;
  a.timeout_ticks = (long long)(timeout_s * (double)ia::oneshot_ticks_per_second());
  IA_HIP_CHECK(ia::oneshot_allreduce(a, ia_stream()));
}

int64_t oneshot_error(int64_t local) {
  int e = 0;
  IA_HIP_CHECK(ia::oneshot_read_error(reinterpret_cast<void*>((uintptr_t)local), &e));
  return e;
}

}  // namespace

void register_comm(py::module& m) {
  m.def("oneshot_alloc", &oneshot_alloc, "zeroed uncached staging region -> (address, IPC handle bytes)");
  m.def("oneshot_open", &oneshot_open, "map a peer's region from its IPC handle -> address");
  m.def("oneshot_close", [](int64_t p) { IA_HIP_CHECK(ia::oneshot_close(reinterpret_cast<void*>((uintptr_t)p))); });
  m.def("oneshot_free", [](int64_t p) { IA_HIP_CHECK(ia::oneshot_free(reinterpret_cast<void*>((uintptr_t)p))); });
  m.def("oneshot_region_bytes", [](int64_t s) { return (int64_t)ia::oneshot_region_bytes((size_t)s); });
  m.def("oneshot_blocks", [](int64_t n, int64_t stage, int64_t elem_bytes) { return ia::oneshot_blocks((int)n, (size_t)stage, (int)elem_bytes); },
        py::arg("n"), py::arg("stage"), py::arg("elem_bytes") = 4);
  m.def("oneshot_allreduce", &oneshot_allreduce, "one-shot sum all-reduce of in*scale over the mapped ranks into out");
  m.def("oneshot_error", &oneshot_error, "error word of a local region (1: a block timed out)");
  m.def("oneshot_error_async",
        [](int64_t local, torch::Tensor pinned) {
          TORCH_CHECK(!pinned.is_cuda() && pinned.is_pinned() && pinned.scalar_type() == torch::kInt32 && pinned.numel() >= 1,
                      "oneshot_error_async: pinned int32 host tensor");
          IA_HIP_CHECK(ia::oneshot_read_error_async(reinterpret_cast<void*>((uintptr_t)local), pinned.data_ptr<int>(),
                                                    ia_stream()));
        },
        "stream-ordered copy of the error word into a pinned host int32 tensor");
  m.def("oneshot_clear_error",
        [](int64_t p) { IA_HIP_CHECK(ia::oneshot_clear_error(reinterpret_cast<void*>((uintptr_t)p))); });
}

// Torch-facing wrappers of the wide-layer MFMA kernels (csrc/kernels/wlin.hip).
#include "common.h"
#include "launchers.h"

#include <map>
#include <mutex>

namespace {

#define IA_HIP_CHECK_W(expr)                                                          \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e)); \
  } while (0)

// Y = act(X W^T + b)
torch::Tensor wlin_forward(torch::Tensor X, torch::Tensor W, c10::optional<torch::Tensor> b, int64_t act) {
  IA_CHECK_GPU_F32(X);
  IA_CHECK_GPU_F32(W);
  TORCH_CHECK(X.dim() == 2 && W.dim() == 2 && X.size(1) == W.size(1), "X [M, K], W [N, K]");
  ia::WideLinArgs a{};
  a.M = (int)X.size(0);
  a.K = (int)X.size(1);
  a.N = (int)W.size(0);
  a.X = X.data_ptr<float>();
  a.W = W.data_ptr<float>();
  if (b.has_value() && b->defined()) {
    IA_CHECK_GPU_F32(*b);
    TORCH_CHECK(b->numel() == a.N, "bias size");
    a.b = b->data_ptr<float>();
  }
  a.act = (int)act;
  auto Y = torch::empty({a.M, a.N}, X.options());
  a.Y = Y.data_ptr<float>();
  IA_HIP_CHECK_W(ia::wlin_forward(a, ia_stream()));
  return Y;
}

// G = (dZ W) * act'(H) [* scale]
torch::Tensor wlin_backward_x(torch::Tensor dZ, torch::Tensor W, c10::optional<torch::Tensor> H, int64_t act,
                              c10::optional<torch::Tensor> scale) {
  IA_CHECK_GPU_F32(dZ);
  IA_CHECK_GPU_F32(W);
  TORCH_CHECK(dZ.dim() == 2 && W.dim() == 2 && dZ.size(1) == W.size(0), "dZ [M, N], W [N, K]");
  ia::WideLinArgs a{};
  a.M = (int)dZ.size(0);
  a.N = (int)W.size(0);
  a.K = (int)W.size(1);
  a.dZ = dZ.data_ptr<float>();
  a.W = W.data_ptr<float>();
  if (H.has_value() && H->defined()) {
    IA_CHECK_GPU_F32(*H);
    TORCH_CHECK(H->size(0) == a.M && H->size(1) == a.K, "H [M, K]");
    a.H = H->data_ptr<float>();
  }
  a.act = (int)act;
  if (scale.has_value() && scale->defined()) {
    IA_CHECK_GPU_F32(*scale);
    TORCH_CHECK(scale->numel() == a.K, "scale [K]");
    a.scale = scale->data_ptr<float>();
  }
  auto G = torch::empty({a.M, a.K}, dZ.options());
  a.G = G.data_ptr<float>();
  IA_HIP_CHECK_W(ia::wlin_backward_x(a, ia_stream()));
  return G;
}

// Zero-initialised dW tile counters, one buffer per (device, stream): launches on one stream
// are ordered and every launch leaves the counters at zero again, so the buffer is reused
// across launches (and across replays of a captured graph).
int* dw_counters(const torch::Tensor& like, int tiles) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, torch::Tensor> bufs;
  std::lock_guard<std::mutex> g(mu);
  auto& t = bufs[{like.get_device(), ia_stream()}];
  if (!t.defined() || t.numel() < tiles)
    t = torch::zeros({std::max(tiles, 1024)}, like.options().dtype(torch::kInt32));
  return t.data_ptr<int>();
}

// (dW = dZ^T X, db = sum_m dZ)
py::tuple wlin_backward_w(torch::Tensor dZ, torch::Tensor X, bool need_db) {
  IA_CHECK_GPU_F32(dZ);
  IA_CHECK_GPU_F32(X);
  TORCH_CHECK(dZ.dim() == 2 && X.dim() == 2 && dZ.size(0) == X.size(0), "dZ [M, N], X [M, K]");
  ia::WideLinArgs a{};
  a.M = (int)dZ.size(0);
  a.N = (int)dZ.size(1);
  a.K = (int)X.size(1);
  a.dZ = dZ.data_ptr<float>();
  a.X = X.data_ptr<float>();
  auto dW = torch::empty({a.N, a.K}, dZ.options());
  a.dW = dW.data_ptr<float>();
  torch::Tensor db;
  if (need_db) {
    db = torch::empty({a.N}, dZ.options());
    a.db = db.data_ptr<float>();
  }
  torch::Tensor ws;
  const size_t nws = ia::wlin_dw_ws_floats(a.M, a.N, a.K);
  if (nws) {
    ws = torch::empty({(int64_t)nws}, dZ.options());
    a.ws = ws.data_ptr<float>();
    a.cnt = dw_counters(dZ, ia::wlin_dw_tiles(a.N, a.K));
  }
  IA_HIP_CHECK_W(ia::wlin_backward_w(a, ia_stream()));
  return py::make_tuple(dW, need_db ? py::cast(db) : py::none());
}

}  // namespace

void register_wide(py::module& m) {
  m.def("wlin_forward", &wlin_forward, py::arg("x"), py::arg("w"), py::arg("b"), py::arg("act"),
        "Y = act(x w^T + b) on MFMA (bf16 operands, fp32 accumulate)");
  m.def("wlin_backward_x", &wlin_backward_x, py::arg("dz"), py::arg("w"), py::arg("h"), py::arg("act"), py::arg("scale"),
        "G = (dz w) * act'(h) [* scale]");
  m.def("wlin_backward_w", &wlin_backward_w, py::arg("dz"), py::arg("x"), py::arg("need_db"), "(dW, db)");
}

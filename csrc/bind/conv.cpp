// Torch-facing wrappers of the NHWC conv kernels (csrc/kernels/conv.hip).
#include "common.h"
#include "launchers.h"

namespace {

#define IA_HIP_CHECK3(expr)                                                           \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e)); \
  } while (0)

int in_kind(const torch::Tensor& x) {
  switch (x.scalar_type()) {
    case torch::kFloat32: return 0;
    case torch::kBFloat16: return 1;
    case torch::kUInt8: return 2;
    default: TORCH_CHECK(false, "conv input must be float32, bfloat16 or uint8");
  }
  return -1;
}

ia::ConvGeo geo(const torch::Tensor& x, int64_t N, int64_t KH, int64_t KW, int64_t S) {
  TORCH_CHECK(x.dim() == 4, "x must be NHWC [B, H, W, C]");
  ia::ConvGeo g{};
  g.B = (int)x.size(0);
  g.H = (int)x.size(1);
  g.W = (int)x.size(2);
  g.C = (int)x.size(3);
  g.KH = (int)KH;
  g.KW = (int)KW;
  g.S = (int)S;
  g.OH = (g.H - g.KH) / g.S + 1;
  g.OW = (g.W - g.KW) / g.S + 1;
  g.N = (int)N;
  TORCH_CHECK(ia::conv_geo_ok(g), "conv geometry outside the kernel (K % 32, KW*C % 8, N in {16,32,48,64})");
  return g;
}

// x NHWC, wb bf16 [N][KH][KW][C] -> y bf16 [B, OH, OW, N]
torch::Tensor conv_fwd(torch::Tensor x, torch::Tensor wb, c10::optional<torch::Tensor> bias, int64_t stride,
                       double in_scale, bool relu) {
  IA_CHECK_CUDA(x);
  IA_CHECK_CONTIG(x);
  IA_CHECK_CUDA(wb);
  IA_CHECK_CONTIG(wb);
  TORCH_CHECK(wb.scalar_type() == torch::kBFloat16 && wb.dim() == 4, "wb must be bf16 [N, KH, KW, C]");
  auto g = geo(x, wb.size(0), wb.size(1), wb.size(2), stride);
  TORCH_CHECK(wb.size(3) == g.C, "channel mismatch");
  const float* b = nullptr;
  if (bias.has_value() && bias->defined()) {
    IA_CHECK_GPU_F32(*bias);
    TORCH_CHECK(bias->numel() == g.N, "bias size");
    b = bias->data_ptr<float>();
  }
  auto y = torch::empty({g.B, g.OH, g.OW, g.N}, x.options().dtype(torch::kBFloat16));
  IA_HIP_CHECK3(ia::conv_forward(in_kind(x), x.data_ptr(), wb.data_ptr(), b, y.data_ptr(), g, (float)in_scale, relu ? 1 : 0,
                                 ia_stream()));
  return y;
}

// (dW fp32 [N][KH][KW][C], db fp32 [N]); dZ = dy * [y > 0] if relu_out
py::tuple conv_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor y, int64_t KH, int64_t KW, int64_t stride,
                     double in_scale, bool relu_out) {
  IA_CHECK_CUDA(x);
  IA_CHECK_CONTIG(x);
  IA_CHECK_CUDA(dy);
  IA_CHECK_CONTIG(dy);
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16, "dy must be bf16 NHWC");
  auto g = geo(x, dy.size(3), KH, KW, stride);
  TORCH_CHECK(dy.size(0) == g.B && dy.size(1) == g.OH && dy.size(2) == g.OW, "dy shape");
  if (relu_out) {
    IA_CHECK_CUDA(y);
    IA_CHECK_CONTIG(y);
    TORCH_CHECK(y.sizes() == dy.sizes() && y.scalar_type() == torch::kBFloat16, "y must match dy");
  }
  auto f32 = x.options().dtype(torch::kFloat32);
  auto slab = torch::empty({(int64_t)ia::conv_wgrad_slab_floats(g)}, f32);
  auto dW = torch::empty({g.N, g.KH, g.KW, g.C}, f32);
  auto db = torch::empty({g.N}, f32);
  IA_HIP_CHECK3(ia::conv_wgrad(in_kind(x), x.data_ptr(), dy.data_ptr(), relu_out ? y.data_ptr() : nullptr,
                               slab.data_ptr<float>(), dW.data_ptr<float>(), db.data_ptr<float>(), g, (float)in_scale,
                               relu_out ? 1 : 0, ia_stream()));
  return py::make_tuple(dW, db);
}

// dZp bf16 [B, H, W, C] = [xp > 0] * conv^T(dy * [y > 0]); wt bf16 [C][KH][KW][N]
torch::Tensor conv_dgrad(torch::Tensor dy, torch::Tensor y, torch::Tensor wt, torch::Tensor xp, int64_t stride,
                         bool relu_out, bool relu_in) {
  IA_CHECK_CUDA(dy);
  IA_CHECK_CONTIG(dy);
  IA_CHECK_CUDA(wt);
  IA_CHECK_CONTIG(wt);
  IA_CHECK_CUDA(xp);
  IA_CHECK_CONTIG(xp);
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16 && wt.scalar_type() == torch::kBFloat16 &&
                  xp.scalar_type() == torch::kBFloat16, "dy, wt, xp must be bf16");
  TORCH_CHECK(wt.dim() == 4, "wt must be [C, KH, KW, N]");
  auto g = geo(xp, dy.size(3), wt.size(1), wt.size(2), stride);
  TORCH_CHECK(wt.size(0) == g.C && wt.size(3) == g.N, "wt shape");
  TORCH_CHECK(dy.size(0) == g.B && dy.size(1) == g.OH && dy.size(2) == g.OW, "dy shape");
  if (relu_out) {
    IA_CHECK_CUDA(y);
    IA_CHECK_CONTIG(y);
    TORCH_CHECK(y.sizes() == dy.sizes() && y.scalar_type() == torch::kBFloat16, "y must match dy");
  }
  auto dz = torch::empty({g.B, g.H, g.W, g.C}, xp.options());
  IA_HIP_CHECK3(ia::conv_dgrad(dy.data_ptr(), relu_out ? y.data_ptr() : nullptr, wt.data_ptr(), xp.data_ptr(),
                               dz.data_ptr(), g, relu_out ? 1 : 0, relu_in ? 1 : 0, ia_stream()));
  return dz;
}

}  // namespace

void register_conv(py::module& m) {
  m.def("conv_fwd", &conv_fwd, "NHWC implicit-GEMM conv + bias + ReLU (bf16 MFMA)", py::arg("x"), py::arg("wb"),
        py::arg("bias"), py::arg("stride"), py::arg("in_scale") = 1.0, py::arg("relu") = true);
  m.def("conv_wgrad", &conv_wgrad, "NHWC conv weight/bias gradient (deterministic block reduction)");
  m.def("conv_dgrad", &conv_dgrad, "NHWC conv data gradient with fused ReLU masks");
}

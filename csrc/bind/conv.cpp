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

ia::ConvGeo geo(const torch::Tensor& x, int64_t N, int64_t KH, int64_t KW, int64_t S, int64_t P = 0) {
  TORCH_CHECK(x.dim() == 4, "x must be NHWC [B, H, W, C]");
  ia::ConvGeo g{};
  g.B = (int)x.size(0);
  g.H = (int)x.size(1);
  g.W = (int)x.size(2);
  g.C = (int)x.size(3);
  g.KH = (int)KH;
  g.KW = (int)KW;
  g.S = (int)S;
  g.P = (int)P;
  g.OH = (g.H + 2 * g.P - g.KH) / g.S + 1;
  g.OW = (g.W + 2 * g.P - g.KW) / g.S + 1;
  g.N = (int)N;
  g.Kp = (g.KH * g.KW * g.C + 31) & ~31;
  TORCH_CHECK(ia::conv_geo_ok(g),
              "conv geometry outside the kernel (valid: KW*C % 8; padded / K % 32 != 0: C % 8, stride 1; N in {16,32,48,64})");
  return g;
}

// [N, KH, KW, C] -> [N, Kp] with zero columns past K (no copy when K == Kp)
torch::Tensor pad_k(const torch::Tensor& w, int Kp) {
  const int64_t N = w.size(0), K = w.numel() / N;
  if (K == Kp) return w;
  auto out = torch::zeros({N, (int64_t)Kp}, w.options());
  out.narrow(1, 0, K).copy_(w.reshape({N, K}));
  return out;
}

// x NHWC, wb bf16 [N][KH][KW][C] -> y bf16 [B, OH, OW, N]
torch::Tensor conv_fwd(torch::Tensor x, torch::Tensor wb, c10::optional<torch::Tensor> bias, int64_t stride,
                       double in_scale, bool relu, int64_t pad, bool splitk) {
  IA_CHECK_CUDA(x);
  IA_CHECK_CONTIG(x);
  IA_CHECK_CUDA(wb);
  IA_CHECK_CONTIG(wb);
  TORCH_CHECK(wb.scalar_type() == torch::kBFloat16 && wb.dim() == 4, "wb must be bf16 [N, KH, KW, C]");
  auto g = geo(x, wb.size(0), wb.size(1), wb.size(2), stride, pad);
  TORCH_CHECK(wb.size(3) == g.C, "channel mismatch");
  auto wk = pad_k(wb, g.Kp);
  const float* b = nullptr;
  if (bias.has_value() && bias->defined()) {
    IA_CHECK_GPU_F32(*bias);
    TORCH_CHECK(bias->numel() == g.N, "bias size");
    b = bias->data_ptr<float>();
  }
  auto y = torch::empty({g.B, g.OH, g.OW, g.N}, x.options().dtype(torch::kBFloat16));
  if (splitk && ia::conv_forward_sk_ok(g)) {  // (else the default form)
    IA_HIP_CHECK3(ia::conv_forward_sk(in_kind(x), x.data_ptr(), wk.data_ptr(), b, y.data_ptr(), g, (float)in_scale,
                                      relu ? 1 : 0, ia_stream()));
    return y;
  }
  IA_HIP_CHECK3(ia::conv_forward(in_kind(x), x.data_ptr(), wk.data_ptr(), b, y.data_ptr(), g, (float)in_scale, relu ? 1 : 0,
                                 ia_stream()));
  return y;
}

// (dW fp32 [N][C][KH][KW] (torch layout), db fp32 [N]); dZ = dy * [y > 0] if relu_out
// the wgrad block partials only (reduction deferred to conv_reduce_multi): returns the slab
torch::Tensor conv_wgrad_partials(torch::Tensor x, torch::Tensor dy, torch::Tensor y, int64_t KH, int64_t KW,
                                  int64_t stride, double in_scale, bool relu_out, int64_t pad) {
  IA_CHECK_CUDA(x);
  IA_CHECK_CONTIG(x);
  IA_CHECK_CUDA(dy);
  IA_CHECK_CONTIG(dy);
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16, "dy must be bf16 NHWC");
  auto g = geo(x, dy.size(3), KH, KW, stride, pad);
  TORCH_CHECK(dy.size(0) == g.B && dy.size(1) == g.OH && dy.size(2) == g.OW, "dy shape");
  if (relu_out) {
    IA_CHECK_CUDA(y);
    IA_CHECK_CONTIG(y);
    TORCH_CHECK(y.sizes() == dy.sizes() && y.scalar_type() == torch::kBFloat16, "y must match dy");
  }
  auto slab = torch::empty({(int64_t)ia::conv_wgrad_slab_floats(g)}, x.options().dtype(torch::kFloat32));
  IA_HIP_CHECK3(ia::conv_wgrad(in_kind(x), x.data_ptr(), dy.data_ptr(), relu_out ? y.data_ptr() : nullptr,
                               slab.data_ptr<float>(), nullptr, nullptr, g, (float)in_scale, relu_out ? 1 : 0, ia_stream()));
  return slab;
}

}  // namespace

// every layer's deferred reduction (slab of conv_wgrad_partials) into dW [N, C, KH, KW] / db [N]
// slots; geometry from the same x / dy / kernel / stride / pad as the partials call. (External:
// the fused Adam launch takes the same reductions, kernels.cpp.)
ia::ConvReduceMulti conv_reduce_args(const std::vector<torch::Tensor>& xs, const std::vector<torch::Tensor>& dys,
                                     const std::vector<int64_t>& KHs, const std::vector<int64_t>& KWs,
                                     const std::vector<int64_t>& strides, const std::vector<int64_t>& pads,
                                     const std::vector<torch::Tensor>& slabs, const std::vector<torch::Tensor>& dWs,
                                     const std::vector<torch::Tensor>& dbs) {
  const size_t n = xs.size();
  TORCH_CHECK(n > 0 && n <= (size_t)ia::kMaxPack && dys.size() == n && KHs.size() == n && KWs.size() == n &&
                  strides.size() == n && pads.size() == n && slabs.size() == n && dWs.size() == n && dbs.size() == n,
              "conv_reduce_multi: one entry per layer (<= 8)");
  ia::ConvReduceMulti r{};
  r.n = (int)n;
  for (size_t l = 0; l < n; ++l) {
    auto g = geo(xs[l], dys[l].size(3), KHs[l], KWs[l], strides[l], pads[l]);
    IA_CHECK_GPU_F32(slabs[l]);
    IA_CHECK_GPU_F32(dWs[l]);
    IA_CHECK_GPU_F32(dbs[l]);
    TORCH_CHECK((size_t)slabs[l].numel() >= ia::conv_wgrad_slab_floats(g), "conv_reduce_multi: slab size");
    TORCH_CHECK(dWs[l].numel() == (int64_t)g.N * g.C * g.KH * g.KW && dbs[l].numel() == g.N, "conv_reduce_multi: dW / db");
    r.g[l] = g;
    r.slab[l] = slabs[l].data_ptr<float>();
    r.dW[l] = dWs[l].data_ptr<float>();
    r.db[l] = dbs[l].data_ptr<float>();
  }
  return r;
}

namespace {

void conv_reduce_multi(std::vector<torch::Tensor> xs, std::vector<torch::Tensor> dys, std::vector<int64_t> KHs,
                       std::vector<int64_t> KWs, std::vector<int64_t> strides, std::vector<int64_t> pads,
                       std::vector<torch::Tensor> slabs, std::vector<torch::Tensor> dWs, std::vector<torch::Tensor> dbs) {
  const ia::ConvReduceMulti r = conv_reduce_args(xs, dys, KHs, KWs, strides, pads, slabs, dWs, dbs);
  IA_HIP_CHECK3(ia::conv_reduce_multi(r, ia_stream()));
}

py::tuple conv_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor y, int64_t KH, int64_t KW, int64_t stride,
                     double in_scale, bool relu_out, int64_t pad, c10::optional<torch::Tensor> dW_out,
                     c10::optional<torch::Tensor> db_out) {
  IA_CHECK_CUDA(x);
  IA_CHECK_CONTIG(x);
  IA_CHECK_CUDA(dy);
  IA_CHECK_CONTIG(dy);
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16, "dy must be bf16 NHWC");
  auto g = geo(x, dy.size(3), KH, KW, stride, pad);
  TORCH_CHECK(dy.size(0) == g.B && dy.size(1) == g.OH && dy.size(2) == g.OW, "dy shape");
  if (relu_out) {
    IA_CHECK_CUDA(y);
    IA_CHECK_CONTIG(y);
    TORCH_CHECK(y.sizes() == dy.sizes() && y.scalar_type() == torch::kBFloat16, "y must match dy");
  }
  auto f32 = x.options().dtype(torch::kFloat32);
  auto slab = torch::empty({(int64_t)ia::conv_wgrad_slab_floats(g)}, f32);
  // torch layout, written by the reduction (optionally straight into caller slots, e.g. views
  // of an optimizer's flat gradient bucket)
  torch::Tensor dW, db;
  if (dW_out && dW_out->defined()) {
    IA_CHECK_GPU_F32(*dW_out);
    IA_CHECK_CONTIG(*dW_out);
    TORCH_CHECK(dW_out->numel() == (int64_t)g.N * g.C * g.KH * g.KW, "conv_wgrad: dW_out size");
    dW = *dW_out;
  } else {
    dW = torch::empty({g.N, g.C, g.KH, g.KW}, f32);
  }
  if (db_out && db_out->defined()) {
    IA_CHECK_GPU_F32(*db_out);
    IA_CHECK_CONTIG(*db_out);
    TORCH_CHECK(db_out->numel() == g.N, "conv_wgrad: db_out size");
    db = *db_out;
  } else {
    db = torch::empty({g.N}, f32);
  }
  IA_HIP_CHECK3(ia::conv_wgrad(in_kind(x), x.data_ptr(), dy.data_ptr(), relu_out ? y.data_ptr() : nullptr,
                               slab.data_ptr<float>(), dW.data_ptr<float>(), db.data_ptr<float>(), g, (float)in_scale,
                               relu_out ? 1 : 0, ia_stream()));
  return py::make_tuple(dW, db);
}

// dZp bf16 [B, H, W, C] = [xp > 0] * conv^T(dy * [y > 0]); wt bf16 [C][KH][KW][N]
torch::Tensor conv_dgrad(torch::Tensor dy, torch::Tensor y, torch::Tensor wt, torch::Tensor xp, int64_t stride,
                         bool relu_out, bool relu_in, int64_t pad, int64_t form) {
  IA_CHECK_CUDA(dy);
  IA_CHECK_CONTIG(dy);
  IA_CHECK_CUDA(wt);
  IA_CHECK_CONTIG(wt);
  IA_CHECK_CUDA(xp);
  IA_CHECK_CONTIG(xp);
  TORCH_CHECK(dy.scalar_type() == torch::kBFloat16 && wt.scalar_type() == torch::kBFloat16 &&
                  xp.scalar_type() == torch::kBFloat16, "dy, wt, xp must be bf16");
  TORCH_CHECK(wt.dim() == 4, "wt must be [C, KH, KW, N]");
  auto g = geo(xp, dy.size(3), wt.size(1), wt.size(2), stride, pad);
  TORCH_CHECK(wt.size(0) == g.C && wt.size(3) == g.N, "wt shape");
  TORCH_CHECK(dy.size(0) == g.B && dy.size(1) == g.OH && dy.size(2) == g.OW, "dy shape");
  if (relu_out) {
    IA_CHECK_CUDA(y);
    IA_CHECK_CONTIG(y);
    TORCH_CHECK(y.sizes() == dy.sizes() && y.scalar_type() == torch::kBFloat16, "y must match dy");
  }
  auto dz = torch::empty({g.B, g.H, g.W, g.C}, xp.options());
  IA_HIP_CHECK3(ia::conv_dgrad(dy.data_ptr(), relu_out ? y.data_ptr() : nullptr, wt.data_ptr(), xp.data_ptr(),
                               dz.data_ptr(), g, relu_out ? 1 : 0, relu_in ? 1 : 0, ia_stream(), (int)form));
  return dz;
}

// One layer's backward in one launch (BC-size batches): (wgrad block partials slab -- reduce with
// conv_reduce_multi --, dZ of the layer input bf16 [B, H, W, C] = [x > 0] * conv^T(dy * [y > 0]))
py::tuple conv_backward_pair(torch::Tensor x, torch::Tensor dy, torch::Tensor y, torch::Tensor wt, int64_t stride,
                             bool relu_out) {
  for (auto* t : {&x, &dy, &wt}) {
    IA_CHECK_CUDA((*t));
    IA_CHECK_CONTIG((*t));
  }
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && dy.scalar_type() == torch::kBFloat16 &&
                  wt.scalar_type() == torch::kBFloat16, "conv_backward_pair: bf16 x, dy, wt");
  TORCH_CHECK(wt.dim() == 4, "wt must be [C, KH, KW, N]");
  auto g = geo(x, dy.size(3), wt.size(1), wt.size(2), stride, 0);
  TORCH_CHECK(wt.size(0) == g.C && wt.size(3) == g.N, "wt shape");
  TORCH_CHECK(dy.size(0) == g.B && dy.size(1) == g.OH && dy.size(2) == g.OW, "dy shape");
  if (relu_out) {
    IA_CHECK_CUDA(y);
    IA_CHECK_CONTIG(y);
    TORCH_CHECK(y.sizes() == dy.sizes() && y.scalar_type() == torch::kBFloat16, "y must match dy");
  }
  TORCH_CHECK(ia::conv_back_pair_ok(g), "conv_backward_pair: geometry outside the paired kernel");
  auto slab = torch::empty({(int64_t)ia::conv_wgrad_slab_floats(g)}, x.options().dtype(torch::kFloat32));
  auto dz = torch::empty({g.B, g.H, g.W, g.C}, x.options());
  IA_HIP_CHECK3(ia::conv_back_pair(x.data_ptr(), dy.data_ptr(), relu_out ? y.data_ptr() : nullptr, slab.data_ptr<float>(),
                                   wt.data_ptr(), dz.data_ptr(), g, relu_out ? 1 : 0, 1, ia_stream()));
  return py::make_tuple(slab, dz);
}

bool conv_backward_pair_ok(torch::Tensor x, int64_t N, int64_t KH, int64_t KW, int64_t stride) {
  if (x.dim() != 4 || x.scalar_type() != torch::kBFloat16) return false;
  ia::ConvGeo g{};
  g.B = (int)x.size(0);
  g.H = (int)x.size(1);
  g.W = (int)x.size(2);
  g.C = (int)x.size(3);
  g.KH = (int)KH;
  g.KW = (int)KW;
  g.S = (int)stride;
  g.P = 0;
  if (g.H < g.KH || g.W < g.KW || g.S <= 0) return false;
  g.OH = (g.H - g.KH) / g.S + 1;
  g.OW = (g.W - g.KW) / g.S + 1;
  g.N = (int)N;
  g.Kp = (g.KH * g.KW * g.C + 31) & ~31;
  return ia::conv_back_pair_ok(g);
}

// fp32 conv weights [N, C, KH, KW] -> (bf16 [N, KH, KW, C] each, bf16 [C, KH, KW, N] where want_t)
// gather (optional): (srcs, perm, cursor, n, dst, inc) of gather_rows_cursor, run in the same launch
py::tuple conv_pack_weights(std::vector<torch::Tensor> ws, std::vector<bool> want_t, std::vector<bool> t_hwc,
                            py::object gather) {
  TORCH_CHECK(ws.size() == want_t.size() && (int)ws.size() <= ia::kMaxPack, "conv_pack_weights: layer count");
  ia::ConvPackArgs a{};
  a.n = (int)ws.size();
  std::vector<torch::Tensor> wbs, wts;
  for (size_t i = 0; i < ws.size(); ++i) {
    auto& w = ws[i];
    IA_CHECK_GPU_F32(w);
    IA_CHECK_CONTIG(w);
    TORCH_CHECK(w.dim() == 4, "conv weight must be [N, C, KH, KW]");
    const int64_t N = w.size(0), C = w.size(1), KH = w.size(2), KW = w.size(3);
    auto wb = torch::empty({N, KH, KW, C}, w.options().dtype(torch::kBFloat16));
    torch::Tensor wt;
    const bool hwc = i < t_hwc.size() && t_hwc[i];
    if (want_t[i])
      wt = hwc ? torch::empty({KH, KW, C, N}, w.options().dtype(torch::kBFloat16))
               : torch::empty({C, KH, KW, N}, w.options().dtype(torch::kBFloat16));
    a.layer[i] = ia::ConvPackLayer{w.data_ptr<float>(), wb.data_ptr(), want_t[i] ? wt.data_ptr() : nullptr, (int)N,
                                   (int)C, (int)KH, (int)KW, hwc ? 1 : 0};
    wbs.push_back(wb);
    wts.push_back(wt);
  }
  if (gather.is_none()) {
    IA_HIP_CHECK3(ia::conv_pack_weights(a, ia_stream()));
  } else {
    auto g = gather.cast<py::tuple>();
    TORCH_CHECK(g.size() == 6, "conv_pack_weights: gather = (srcs, perm, cursor, n, dst, inc)");
    auto srcs = g[0].cast<std::vector<torch::Tensor>>();
    auto perm = g[1].cast<torch::Tensor>();
    auto cursor = g[2].cast<torch::Tensor>();
    const int64_t n = g[3].cast<int64_t>();
    auto dst = g[4].cast<std::vector<torch::Tensor>>();
    c10::optional<torch::Tensor> inc;
    if (!g[5].is_none()) inc = g[5].cast<torch::Tensor>();
    float* incp = nullptr;
    const ia::GatherArgs ga = gather_cursor_args(srcs, perm, cursor, n, dst, inc, &incp);
    IA_HIP_CHECK3(ia::conv_pack_weights(a, ia_stream(), &ga, perm.data_ptr<int>(), cursor.data_ptr<int>(), (int)n, incp));
  }
  py::list lb, lt;
  for (size_t i = 0; i < ws.size(); ++i) {
    lb.append(wbs[i]);
    if (want_t[i]) lt.append(wts[i]);
    else lt.append(py::none());
  }
  return py::make_tuple(lb, lt);
}

// h fp32 [B, NH] = relu(x [B, K] . w [NH, K]^T + b); x, w bf16
torch::Tensor cnn_fc(torch::Tensor x, torch::Tensor w, torch::Tensor b) {
  IA_CHECK_CUDA(x);
  IA_CHECK_CONTIG(x);
  IA_CHECK_CUDA(w);
  IA_CHECK_CONTIG(w);
  IA_CHECK_GPU_F32(b);
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16, "x, w must be bf16");
  const int B = (int)x.size(0);
  const int64_t K = x.numel() / std::max<int64_t>(1, B);
  TORCH_CHECK(w.dim() == 2 && w.size(1) == K, "w must be [NH, K] with K = x.numel() / B");
  const int NH = (int)w.size(0);
  TORCH_CHECK(b.numel() == NH && K % 32 == 0 && NH % 16 == 0, "cnn_fc: K % 32, NH % 16, bias [NH]");
  auto h = torch::empty({B, NH}, x.options().dtype(torch::kFloat32));
  IA_HIP_CHECK3(ia::cnn_fc(x.data_ptr(), w.data_ptr(), b.data_ptr<float>(), h.data_ptr<float>(), B, (int)K, NH, ia_stream()));
  return h;
}

// Linear + ReLU backward over the NHWC-flattened conv output: (dW fp32 [NH, C*HW] torch (c, h, w)
// columns, db fp32 [NH], dX bf16 [M, K] or None)
py::tuple fc_backward(torch::Tensor x, torch::Tensor dh, torch::Tensor h, torch::Tensor wt, int64_t C, bool need_dx,
                      c10::optional<torch::Tensor> dW_out, c10::optional<torch::Tensor> db_out, bool mask_dx) {
  IA_CHECK_CUDA(x);
  IA_CHECK_CONTIG(x);
  IA_CHECK_CUDA(wt);
  IA_CHECK_CONTIG(wt);
  IA_CHECK_GPU_F32(h);
  IA_CHECK_CONTIG(h);
  auto dhc = dh.contiguous().to(torch::kFloat32);
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && wt.scalar_type() == torch::kBFloat16, "fc_backward: bf16 x / wt");
  const int M = (int)x.size(0);
  const int64_t K = x.numel() / std::max<int64_t>(1, M);
  const int NH = (int)h.size(1);
  TORCH_CHECK(h.dim() == 2 && h.size(0) == M && dhc.sizes() == h.sizes() && wt.numel() == K * NH && C > 0 && K % C == 0,
              "fc_backward: shapes");
  TORCH_CHECK(ia::fc_train_ok(M, (int)K, NH, (int)C, (int)(K / C)), "fc_backward: K % 64, NH % 64");
  torch::Tensor dW, db;
  if (dW_out && dW_out->defined()) {
    IA_CHECK_GPU_F32(*dW_out);
    IA_CHECK_CONTIG(*dW_out);
    TORCH_CHECK(dW_out->numel() == (int64_t)NH * K, "fc_backward: dW_out size");
    dW = *dW_out;
  } else {
    dW = torch::empty({NH, K}, h.options());
  }
  if (db_out && db_out->defined()) {
    IA_CHECK_GPU_F32(*db_out);
    IA_CHECK_CONTIG(*db_out);
    TORCH_CHECK(db_out->numel() == NH, "fc_backward: db_out size");
    db = *db_out;
  } else {
    db = torch::empty({NH}, h.options());
  }
  torch::Tensor dx;
  if (need_dx) dx = torch::empty({M, K}, x.options());
  auto dzb = torch::empty({M, NH}, x.options());  // bf16 dZ, fc_wgrad -> fc_dgrad
  IA_HIP_CHECK3(ia::fc_backward(x.data_ptr(), dhc.data_ptr<float>(), h.data_ptr<float>(), wt.data_ptr(),
                                dW.data_ptr<float>(), db.data_ptr<float>(), need_dx ? dx.data_ptr() : nullptr, dzb.data_ptr(), M,
                                (int)K, NH, (int)C, (int)(K / C), ia_stream(), mask_dx));
  return py::make_tuple(dW, db, need_dx ? py::cast(dx) : py::none());
}

// Two same-shape unpadded convs (+ bias + ReLU) in one launch: the collector's expert and
// learner layers. Returns (y1, y2).
py::tuple conv_fwd_pair(torch::Tensor x1, torch::Tensor x2, torch::Tensor w1, torch::Tensor w2, torch::Tensor b1,
                        torch::Tensor b2, int64_t stride, double in_scale, bool relu) {
  for (auto* t : {&x1, &x2, &w1, &w2}) {
    IA_CHECK_CUDA((*t));
    IA_CHECK_CONTIG((*t));
  }
  IA_CHECK_GPU_F32(b1);
  IA_CHECK_GPU_F32(b2);
  TORCH_CHECK(x1.sizes() == x2.sizes() && x1.scalar_type() == x2.scalar_type(), "conv_fwd_pair: inputs differ");
  TORCH_CHECK(w1.sizes() == w2.sizes() && w1.scalar_type() == torch::kBFloat16 && w2.scalar_type() == torch::kBFloat16 &&
                  w1.dim() == 4,
              "conv_fwd_pair: weights must be same-shape bf16 [N, KH, KW, C]");
  auto g = geo(x1, w1.size(0), w1.size(1), w1.size(2), stride, 0);
  TORCH_CHECK(w1.size(3) == g.C && g.Kp == g.KH * g.KW * g.C && g.N % 16 == 0 && b1.numel() == g.N && b2.numel() == g.N,
              "conv_fwd_pair: K = KH*KW*C must be a multiple of 32, N of 16, bias [N]");
  auto y1 = torch::empty({g.B, g.OH, g.OW, g.N}, x1.options().dtype(torch::kBFloat16));
  auto y2 = torch::empty_like(y1);
  ia::ConvPair p{{x1.data_ptr(), x2.data_ptr()}, {w1.data_ptr(), w2.data_ptr()}, {b1.data_ptr<float>(), b2.data_ptr<float>()},
                 {y1.data_ptr(), y2.data_ptr()}};
  IA_HIP_CHECK3(ia::conv_fwd_pair(in_kind(x1), p, g, (float)in_scale, relu ? 1 : 0, ia_stream()));
  return py::make_tuple(y1, y2);
}

// cnn_fc of two same-shape networks in one launch; returns (h1, h2)
py::tuple cnn_fc_pair(torch::Tensor x1, torch::Tensor x2, torch::Tensor w1, torch::Tensor w2, torch::Tensor b1,
                      torch::Tensor b2) {
  for (auto* t : {&x1, &x2, &w1, &w2}) {
    IA_CHECK_CUDA((*t));
    IA_CHECK_CONTIG((*t));
    TORCH_CHECK(t->scalar_type() == torch::kBFloat16, "cnn_fc_pair: x, w must be bf16");
  }
  IA_CHECK_GPU_F32(b1);
  IA_CHECK_GPU_F32(b2);
  TORCH_CHECK(x1.sizes() == x2.sizes() && w1.sizes() == w2.sizes(), "cnn_fc_pair: shapes differ");
  const int B = (int)x1.size(0);
  const int64_t K = x1.numel() / std::max<int64_t>(1, B);
  TORCH_CHECK(w1.dim() == 2 && w1.size(1) == K, "w must be [NH, K] with K = x.numel() / B");
  const int NH = (int)w1.size(0);
  TORCH_CHECK(b1.numel() == NH && b2.numel() == NH && K % 32 == 0 && NH % 16 == 0, "cnn_fc_pair: K % 32, NH % 16");
  auto h1 = torch::empty({B, NH}, x1.options().dtype(torch::kFloat32));
  auto h2 = torch::empty_like(h1);
  ia::CnnFcPair p{{x1.data_ptr(), x2.data_ptr()}, {w1.data_ptr(), w2.data_ptr()}, {b1.data_ptr<float>(), b2.data_ptr<float>()},
                  {h1.data_ptr<float>(), h2.data_ptr<float>()}};
  IA_HIP_CHECK3(ia::cnn_fc_pair(p, B, (int)K, NH, ia_stream()));
  return py::make_tuple(h1, h2);
}

// Action head + choice (+ beta-mix); see cnn_infer.hip. All outputs are preallocated int64 [B].
ia::CnnHeadArgs head_args(torch::Tensor h, torch::Tensor w2, torch::Tensor b2, int64_t mode, int64_t seed,
                          c10::optional<torch::Tensor> counter, torch::Tensor out, c10::optional<torch::Tensor> rec_out,
                          c10::optional<torch::Tensor> mix_expert, c10::optional<torch::Tensor> beta,
                          c10::optional<torch::Tensor> exec_out) {
  IA_CHECK_GPU_F32(h);
  IA_CHECK_GPU_F32(w2);
  IA_CHECK_GPU_F32(b2);
  ia::CnnHeadArgs a{};
  a.B = (int)h.size(0);
  a.NH = (int)h.size(1);
  a.A = (int)w2.size(0);
  TORCH_CHECK(w2.dim() == 2 && w2.size(1) == a.NH && b2.numel() == a.A, "head shapes");
  auto i64 = [&](const torch::Tensor& t, const char* k) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kInt64 && t.numel() == a.B, k,
                " must be a contiguous int64 GPU tensor of B elements");
    return t.data_ptr<int64_t>();
  };
  a.h = h.data_ptr<float>();
  a.W2 = w2.data_ptr<float>();
  a.b2 = b2.data_ptr<float>();
  a.mode = (int)mode;
  a.seed = (uint64_t)seed;
  if (counter.has_value() && counter->defined()) {
    TORCH_CHECK(counter->is_cuda() && counter->scalar_type() == torch::kInt64 && counter->numel() == 1, "counter");
    a.counter = reinterpret_cast<uint64_t*>(counter->data_ptr<int64_t>());
  }
  a.out = i64(out, "out");
  if (rec_out.has_value() && rec_out->defined()) a.rec_out = i64(*rec_out, "rec_out");
  if (exec_out.has_value() && exec_out->defined()) {
    TORCH_CHECK(mix_expert.has_value() && beta.has_value(), "exec_out needs mix_expert and beta");
    a.exec_out = i64(*exec_out, "exec_out");
    a.mix_expert = i64(*mix_expert, "mix_expert");
    IA_CHECK_GPU_F32(*beta);
    a.beta = beta->data_ptr<float>();
  }
  return a;
}

void cnn_head(torch::Tensor h, torch::Tensor w2, torch::Tensor b2, int64_t mode, int64_t seed,
              c10::optional<torch::Tensor> counter, torch::Tensor out, c10::optional<torch::Tensor> rec_out,
              c10::optional<torch::Tensor> mix_expert, c10::optional<torch::Tensor> beta,
              c10::optional<torch::Tensor> exec_out) {
  const ia::CnnHeadArgs a = head_args(h, w2, b2, mode, seed, counter, out, rec_out, mix_expert, beta, exec_out);
  IA_HIP_CHECK3(ia::cnn_head(a, ia_stream()));
}

// DAgger's expert argmax (-> out_e, rec_out_e) and learner Gumbel sample (-> out_l, and
// exec_out = u > beta ? learner : expert) in one launch: the same results as the two cnn_head
// calls (expert, then learner with mix_expert = out_e).
void cnn_head_pair(torch::Tensor h_e, torch::Tensor w_e, torch::Tensor b_e, torch::Tensor out_e,
                   c10::optional<torch::Tensor> rec_out_e, torch::Tensor h_l, torch::Tensor w_l, torch::Tensor b_l,
                   int64_t seed, torch::Tensor counter, torch::Tensor out_l, torch::Tensor beta, torch::Tensor exec_out) {
  const ia::CnnHeadArgs e = head_args(h_e, w_e, b_e, 0, 0, c10::nullopt, out_e, rec_out_e, c10::nullopt, c10::nullopt,
                                      c10::nullopt);
  const ia::CnnHeadArgs r = head_args(h_l, w_l, b_l, 1, seed, counter, out_l, c10::nullopt, out_e, beta, exec_out);
  TORCH_CHECK(e.B == r.B && e.NH == r.NH, "cnn_head_pair: the two heads' batch / hidden sizes differ");
  IA_HIP_CHECK3(ia::cnn_head_pair(e, r, ia_stream()));
}

}  // namespace

void register_conv(py::module& m) {
  m.def("cnn_fc", &cnn_fc, "NatureCNN actor FC: relu(x . w^T + b), bf16 MFMA", py::arg("x"), py::arg("w"), py::arg("b"));
  m.def("cnn_head", &cnn_head, "actor head + argmax / Gumbel sample (+ beta mix)", py::arg("h"), py::arg("w2"),
        py::arg("b2"), py::arg("mode"), py::arg("seed"), py::arg("counter"), py::arg("out"), py::arg("rec_out") = py::none(),
        py::arg("mix_expert") = py::none(), py::arg("beta") = py::none(), py::arg("exec_out") = py::none());
  m.def("cnn_head_pair", &cnn_head_pair, "expert argmax + learner sample + beta mix in one launch", py::arg("h_e"),
        py::arg("w_e"), py::arg("b_e"), py::arg("out_e"), py::arg("rec_out_e"), py::arg("h_l"), py::arg("w_l"), py::arg("b_l"),
        py::arg("seed"), py::arg("counter"), py::arg("out_l"), py::arg("beta"), py::arg("exec_out"));
  m.def("conv_fwd", &conv_fwd, "NHWC implicit-GEMM conv + bias + ReLU (bf16 MFMA)", py::arg("x"), py::arg("wb"),
        py::arg("bias"), py::arg("stride"), py::arg("in_scale") = 1.0, py::arg("relu") = true, py::arg("pad") = 0,
        py::arg("splitk") = false);
  m.def("conv_fwd_pair", &conv_fwd_pair, "two same-shape convs (expert + learner) in one launch");
  m.def("cnn_fc_pair", &cnn_fc_pair, "two same-shape cnn_fc layers in one launch");
  m.def("conv_pack_weights", &conv_pack_weights, "fp32 conv weights -> bf16 GEMM layouts (+ a minibatch gather), one launch",
        py::arg("ws"), py::arg("want_t"), py::arg("t_hwc") = std::vector<bool>{}, py::arg("gather") = py::none());
  m.def("fc_backward", &fc_backward, "NatureCNN feature-layer backward (dW torch layout, db, dX NHWC bf16)", py::arg("x"),
        py::arg("dh"), py::arg("h"), py::arg("wt"), py::arg("C"), py::arg("need_dx"), py::arg("dW_out") = py::none(),
        py::arg("db_out") = py::none(), py::arg("mask_dx") = false);
  m.def("conv_wgrad", &conv_wgrad, "NHWC conv weight/bias gradient (deterministic block reduction)", py::arg("x"),
        py::arg("dy"), py::arg("y"), py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("in_scale"),
        py::arg("relu_out"), py::arg("pad") = 0, py::arg("dW_out") = py::none(), py::arg("db_out") = py::none());
  m.def("conv_wgrad_partials", &conv_wgrad_partials, "NHWC conv weight-gradient block partials (deferred reduction)",
        py::arg("x"), py::arg("dy"), py::arg("y"), py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("in_scale"),
        py::arg("relu_out"), py::arg("pad") = 0);
  m.def("conv_reduce_multi", &conv_reduce_multi, "deferred wgrad reductions of several layers, one launch");
  m.def("conv_backward_pair", &conv_backward_pair, "one layer's wgrad partials + data gradient in one launch",
        py::arg("x"), py::arg("dy"), py::arg("y"), py::arg("wt"), py::arg("stride"), py::arg("relu_out"));
  m.def("conv_backward_pair_ok", &conv_backward_pair_ok, "whether conv_backward_pair takes this layer", py::arg("x"),
        py::arg("N"), py::arg("KH"), py::arg("KW"), py::arg("stride"));
  m.def("conv_dgrad", &conv_dgrad, "NHWC conv data gradient with fused ReLU masks", py::arg("dy"), py::arg("y"),
        py::arg("wt"), py::arg("xp"), py::arg("stride"), py::arg("relu_out"), py::arg("relu_in"), py::arg("pad") = 0,
        py::arg("form") = -1);
}

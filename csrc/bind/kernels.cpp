// Torch-facing wrappers for the HIP kernels (tensor checks -> raw pointers).
#include "common.h"
#include "launchers.h"

namespace {

#define IA_HIP_CHECK(expr)                                                            \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e)); \
  } while (0)

ia::MLPDesc make_desc(const std::vector<torch::Tensor>& Ws, const std::vector<torch::Tensor>& bs, int64_t hidden_act,
                      int64_t out_act, const c10::optional<torch::Tensor>& mean, const c10::optional<torch::Tensor>& var,
                      double eps, double clip) {
  TORCH_CHECK(!Ws.empty() && Ws.size() <= (size_t)ia::kMaxLayers, "1..4 layers supported");
  TORCH_CHECK(Ws.size() == bs.size(), "one bias per weight");
  ia::MLPDesc d{};
  d.n_layers = (int)Ws.size();
  d.hidden_act = (int)hidden_act;
  d.out_act = (int)out_act;
  d.dims[0] = (int)Ws[0].size(1);
  for (size_t l = 0; l < Ws.size(); ++l) {
    IA_CHECK_GPU_F32(Ws[l]);
    IA_CHECK_GPU_F32(bs[l]);
    TORCH_CHECK(Ws[l].dim() == 2 && Ws[l].size(1) == d.dims[l], "layer ", l, " input dim mismatch");
    TORCH_CHECK(bs[l].numel() == Ws[l].size(0), "bias size mismatch");
    d.dims[l + 1] = (int)Ws[l].size(0);
    d.W[l] = Ws[l].data_ptr<float>();
    d.b[l] = bs[l].data_ptr<float>();
  }
  for (int l = 0; l <= d.n_layers; ++l) TORCH_CHECK(d.dims[l] <= ia::kMaxDim, "tmlp width limit is 128");
  if (mean.has_value() && mean->defined()) {
    IA_CHECK_GPU_F32(*mean);
    IA_CHECK_GPU_F32(*var);
    TORCH_CHECK(mean->numel() == d.dims[0] && var->numel() == d.dims[0], "norm stats size mismatch");
    d.norm_mean = mean->data_ptr<float>();
    d.norm_var = var->data_ptr<float>();
  }
  d.norm_eps = (float)eps;
  d.norm_clip = (float)clip;
  return d;
}

torch::Tensor tmlp_forward(torch::Tensor x, std::vector<torch::Tensor> Ws, std::vector<torch::Tensor> bs,
                           int64_t hidden_act, int64_t out_act, c10::optional<torch::Tensor> mean,
                           c10::optional<torch::Tensor> var, double eps, double clip) {
  IA_CHECK_GPU_F32(x);
  TORCH_CHECK(x.dim() == 2, "x must be [B, D]");
  auto d = make_desc(Ws, bs, hidden_act, out_act, mean, var, eps, clip);
  TORCH_CHECK(x.size(1) == d.dims[0], "input dim mismatch");
  auto y = torch::empty({x.size(0), d.dims[d.n_layers]}, x.options());
  IA_HIP_CHECK(ia::tmlp_forward(d, x.data_ptr<float>(), (int)x.size(0), y.data_ptr<float>(), ia_stream()));
  return y;
}

// Returns (dx or None, [dW...], [db...]).
py::tuple tmlp_backward(torch::Tensor x, torch::Tensor dy, std::vector<torch::Tensor> Ws, std::vector<torch::Tensor> bs,
                        int64_t hidden_act, int64_t out_act, c10::optional<torch::Tensor> mean,
                        c10::optional<torch::Tensor> var, double eps, double clip, bool need_dx) {
  IA_CHECK_GPU_F32(x);
  IA_CHECK_GPU_F32(dy);
  auto d = make_desc(Ws, bs, hidden_act, out_act, mean, var, eps, clip);
  const int B = (int)x.size(0);
  TORCH_CHECK(dy.size(0) == B && dy.size(1) == d.dims[d.n_layers], "dy shape mismatch");
  ia::MLPGrads g{};
  std::vector<torch::Tensor> dWs, dbs;
  for (int l = 0; l < d.n_layers; ++l) {
    dWs.push_back(torch::empty_like(Ws[l]));
    dbs.push_back(torch::empty_like(bs[l]));
    g.dW[l] = dWs.back().data_ptr<float>();
    g.db[l] = dbs.back().data_ptr<float>();
  }
  g.accumulate = 0;
  torch::Tensor dx;
  if (need_dx) dx = torch::empty_like(x);
  const size_t slab_n = ia::tmlp_slab_floats(d, B);
  torch::Tensor slab;
  if (slab_n) slab = torch::empty({(int64_t)slab_n}, x.options());
  IA_HIP_CHECK(ia::tmlp_backward(d, x.data_ptr<float>(), dy.data_ptr<float>(), B, need_dx ? dx.data_ptr<float>() : nullptr,
                                 g, slab_n ? slab.data_ptr<float>() : nullptr, ia_stream()));
  py::object dxo = need_dx ? py::cast(dx) : py::none();
  return py::make_tuple(dxo, dWs, dbs);
}

// Grouped (ensemble) descriptor: Ws[l] [G, out, in], bs[l] [G, out], mean / var [G, din];
// x is [B, din] (shared by every group) or [G, B, din].
ia::MLPDesc make_group_desc(const torch::Tensor& x, const std::vector<torch::Tensor>& Ws, const std::vector<torch::Tensor>& bs,
                            int64_t hidden_act, int64_t out_act, const c10::optional<torch::Tensor>& mean,
                            const c10::optional<torch::Tensor>& var, double eps, int* B_out) {
  TORCH_CHECK(!Ws.empty() && Ws.size() <= (size_t)ia::kMaxLayers && Ws.size() == bs.size(), "1..4 layers");
  const int64_t G = Ws[0].size(0);
  ia::MLPDesc d{};
  d.n_layers = (int)Ws.size();
  d.hidden_act = (int)hidden_act;
  d.out_act = (int)out_act;
  d.dims[0] = (int)Ws[0].size(2);
  d.groups = (int)G;
  for (size_t l = 0; l < Ws.size(); ++l) {
    IA_CHECK_GPU_F32(Ws[l]);
    IA_CHECK_GPU_F32(bs[l]);
    TORCH_CHECK(Ws[l].dim() == 3 && Ws[l].size(0) == G && Ws[l].size(2) == d.dims[l], "layer ", l, " must be [G, out, in]");
    TORCH_CHECK(bs[l].dim() == 2 && bs[l].size(0) == G && bs[l].size(1) == Ws[l].size(1), "bias ", l, " must be [G, out]");
    d.dims[l + 1] = (int)Ws[l].size(1);
    d.W[l] = Ws[l].data_ptr<float>();
    d.b[l] = bs[l].data_ptr<float>();
    d.gs_w[l] = Ws[l].size(1) * Ws[l].size(2);
    d.gs_b[l] = Ws[l].size(1);
  }
  for (int l = 0; l <= d.n_layers; ++l) TORCH_CHECK(d.dims[l] <= ia::kMaxDim, "tmlp width limit is 128");
  if (mean.has_value() && mean->defined()) {
    IA_CHECK_GPU_F32(*mean);
    IA_CHECK_GPU_F32(*var);
    TORCH_CHECK(mean->numel() == G * d.dims[0] && var->numel() == G * d.dims[0], "norm stats must be [G, din]");
    d.norm_mean = mean->data_ptr<float>();
    d.norm_var = var->data_ptr<float>();
    d.gs_norm = d.dims[0];
  }
  d.norm_eps = (float)eps;
  IA_CHECK_GPU_F32(x);
  if (x.dim() == 2) {
    TORCH_CHECK(x.size(1) == d.dims[0], "input dim mismatch");
    *B_out = (int)x.size(0);
    d.gs_x = 0;
  } else {
    TORCH_CHECK(x.dim() == 3 && x.size(0) == G && x.size(2) == d.dims[0], "x must be [B, din] or [G, B, din]");
    *B_out = (int)x.size(1);
    d.gs_x = x.size(1) * x.size(2);
  }
  d.gs_y = (int64_t)(*B_out) * d.dims[d.n_layers];
  return d;
}

// y [G, B, out]: every ensemble member's MLP in ONE launch (grid.y = member)
torch::Tensor tmlp_forward_grouped(torch::Tensor x, std::vector<torch::Tensor> Ws, std::vector<torch::Tensor> bs,
                                   int64_t hidden_act, int64_t out_act, c10::optional<torch::Tensor> mean,
                                   c10::optional<torch::Tensor> var, double eps) {
  int B = 0;
  auto d = make_group_desc(x, Ws, bs, hidden_act, out_act, mean, var, eps, &B);
  auto y = torch::empty({(int64_t)d.groups, B, d.dims[d.n_layers]}, x.options());
  IA_HIP_CHECK(ia::tmlp_forward(d, x.data_ptr<float>(), B, y.data_ptr<float>(), ia_stream()));
  return y;
}

// (dx [G, B, din] or None, [dW [G, out, in]...], [db [G, out]...]) for dy [G, B, out]
py::tuple tmlp_backward_grouped(torch::Tensor x, torch::Tensor dy, std::vector<torch::Tensor> Ws, std::vector<torch::Tensor> bs,
                                int64_t hidden_act, int64_t out_act, c10::optional<torch::Tensor> mean,
                                c10::optional<torch::Tensor> var, double eps, bool need_dx) {
  int B = 0;
  auto d = make_group_desc(x, Ws, bs, hidden_act, out_act, mean, var, eps, &B);
  const int64_t G = d.groups;
  IA_CHECK_GPU_F32(dy);
  TORCH_CHECK(dy.dim() == 3 && dy.size(0) == G && dy.size(1) == B && dy.size(2) == d.dims[d.n_layers], "dy must be [G, B, out]");
  TORCH_CHECK(!need_dx || d.gs_x != 0, "dx of a shared input is not produced");
  ia::MLPGrads g{};
  std::vector<torch::Tensor> dWs, dbs;
  for (int l = 0; l < d.n_layers; ++l) {
    dWs.push_back(torch::empty_like(Ws[l]));
    dbs.push_back(torch::empty_like(bs[l]));
    g.dW[l] = dWs.back().data_ptr<float>();
    g.db[l] = dbs.back().data_ptr<float>();
  }
  torch::Tensor dx;
  if (need_dx) dx = torch::empty_like(x);
  const size_t slab_n = ia::tmlp_slab_floats(d, B);
  torch::Tensor slab;
  if (slab_n) slab = torch::empty({(int64_t)(slab_n * G)}, x.options());
  IA_HIP_CHECK(ia::tmlp_backward(d, x.data_ptr<float>(), dy.data_ptr<float>(), B, need_dx ? dx.data_ptr<float>() : nullptr, g,
                                 slab_n ? slab.data_ptr<float>() : nullptr, ia_stream()));
  py::object dxo = need_dx ? py::cast(dx) : py::none();
  return py::make_tuple(dxo, dWs, dbs);
}

py::tuple gae(torch::Tensor rew, torch::Tensor val, torch::Tensor starts, torch::Tensor last_val, torch::Tensor dones,
              double gamma, double lam, c10::optional<torch::Tensor> moments) {
  IA_CHECK_GPU_F32(rew);
  IA_CHECK_GPU_F32(val);
  IA_CHECK_GPU_F32(starts);
  IA_CHECK_GPU_F32(last_val);
  IA_CHECK_GPU_F32(dones);
  TORCH_CHECK(rew.dim() == 2, "rewards must be [T, N]");
  const int T = (int)rew.size(0), N = (int)rew.size(1);
  TORCH_CHECK(val.sizes() == rew.sizes() && starts.sizes() == rew.sizes(), "shape mismatch");
  TORCH_CHECK(last_val.numel() == N && dones.numel() == N, "bootstrap shape mismatch");
  auto adv = torch::empty_like(rew);
  auto ret = torch::empty_like(rew);
  float* mom = nullptr;
  if (moments && moments->defined()) {
    IA_CHECK_GPU_F32(*moments);
    TORCH_CHECK(moments->is_contiguous() && moments->numel() >= 4 * (int64_t)N, "moments must hold [N][4] floats");
    mom = moments->data_ptr<float>();
  }
  IA_HIP_CHECK(ia::gae_launch(rew.data_ptr<float>(), val.data_ptr<float>(), starts.data_ptr<float>(),
                              last_val.data_ptr<float>(), dones.data_ptr<float>(), T, N, (float)gamma, (float)lam,
                              adv.data_ptr<float>(), ret.data_ptr<float>(), ia_stream(), mom));
  return py::make_tuple(adv, ret);
}

// One fused Adam / AdamW step over flat fp32 buffers (ops/optim.py FusedAdam).
void adam_flat(torch::Tensor params, torch::Tensor grads, torch::Tensor exp_avg, torch::Tensor exp_avg_sq,
               torch::Tensor step, double lr, double beta1, double beta2, double eps, double weight_decay, bool decoupled,
               bool maximize, bool zero_grad, c10::optional<torch::Tensor> step_cnt,
               c10::optional<torch::Tensor> append_src, c10::optional<torch::Tensor> append_all,
               c10::optional<torch::Tensor> append_cursor, py::object reduce) {
  for (auto* t : {&params, &grads, &exp_avg, &exp_avg_sq}) {
    IA_CHECK_GPU_F32(*t);
    TORCH_CHECK(t->numel() == params.numel(), "flat Adam buffers must have equal sizes");
  }
  IA_CHECK_GPU_F32(step);
  TORCH_CHECK(step.numel() == 1, "step must be a 1-element device tensor");
  ia::AdamArgs a{};
  a.params = params.data_ptr<float>();
  a.grads = grads.data_ptr<float>();
  a.exp_avg = exp_avg.data_ptr<float>();
  a.exp_avg_sq = exp_avg_sq.data_ptr<float>();
  a.step = step.data_ptr<float>();
  a.n = params.numel();
  a.lr = (float)lr;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.weight_decay = (float)weight_decay;
  a.decoupled = decoupled ? 1 : 0;
  a.maximize = maximize ? 1 : 0;
  a.zero_grad = zero_grad ? 1 : 0;
  if (step_cnt && step_cnt->defined()) {  // the kernel increments `step` itself
    IA_CHECK_CUDA(*step_cnt);
    TORCH_CHECK(step_cnt->scalar_type() == torch::kInt32 && step_cnt->numel() == 1, "step_cnt: int32 scalar (zero)");
    a.cnt = reinterpret_cast<unsigned*>(step_cnt->data_ptr<int>());
  }
  if (append_cursor && append_cursor->defined()) {  // + the graphed epoch's metrics append
    TORCH_CHECK(append_src && append_src->defined() && append_all && append_all->defined(), "append: src, all, cursor");
    const auto& src = *append_src;
    const auto& all = *append_all;
    const auto& cur = *append_cursor;
    IA_CHECK_CUDA(src);
    IA_CHECK_CUDA(all);
    IA_CHECK_CUDA(cur);
    TORCH_CHECK(src.scalar_type() == torch::kFloat32 && all.scalar_type() == torch::kFloat32 && src.is_contiguous() &&
                    all.is_contiguous() && all.numel() % src.numel() == 0 && cur.scalar_type() == torch::kInt32,
                "append: fp32 src [n], all [m, n], int32 cursor");
    a.app_src = src.data_ptr<float>();
    a.app_all = all.data_ptr<float>();
    a.app_cursor = cur.data_ptr<int>();
    a.app_n = (int)src.numel();
  }
  if (!reduce.is_none()) {  // conv_reduce_multi's arguments: those reductions run in this launch
    const auto t = reduce.cast<py::tuple>();
    TORCH_CHECK(t.size() == 9, "reduce: the 9 conv_reduce_multi argument lists");
    const ia::ConvReduceMulti r = conv_reduce_args(
        t[0].cast<std::vector<torch::Tensor>>(), t[1].cast<std::vector<torch::Tensor>>(), t[2].cast<std::vector<int64_t>>(),
        t[3].cast<std::vector<int64_t>>(), t[4].cast<std::vector<int64_t>>(), t[5].cast<std::vector<int64_t>>(),
        t[6].cast<std::vector<torch::Tensor>>(), t[7].cast<std::vector<torch::Tensor>>(),
        t[8].cast<std::vector<torch::Tensor>>());
    IA_HIP_CHECK(ia::adam_flat(a, ia_stream(), &r));
    return;
  }
  IA_HIP_CHECK(ia::adam_flat(a, ia_stream()));
}

// categorical evaluate_actions: (log pi(a), entropy) from raw logits z [B, A] fp32, acts [B] int64
py::tuple cat_eval_fwd(torch::Tensor z, torch::Tensor acts) {
  IA_CHECK_GPU_F32(z);
  IA_CHECK_CONTIG(z);
  IA_CHECK_CUDA(acts);
  IA_CHECK_CONTIG(acts);
  TORCH_CHECK(z.dim() == 2 && acts.scalar_type() == torch::kInt64 && acts.numel() == z.size(0), "cat_eval shapes");
  TORCH_CHECK(z.size(1) <= 64, "cat_eval: at most 64 actions");
  auto logp = torch::empty({z.size(0)}, z.options());
  auto ent = torch::empty({z.size(0)}, z.options());
  IA_HIP_CHECK(ia::cat_eval_fwd(z.data_ptr<float>(), acts.data_ptr<int64_t>(), (int)z.size(0), (int)z.size(1),
                                 logp.data_ptr<float>(), ent.data_ptr<float>(), ia_stream()));
  return py::make_tuple(logp, ent);
}

torch::Tensor cat_eval_bwd(torch::Tensor z, torch::Tensor acts, c10::optional<torch::Tensor> g_lp,
                           c10::optional<torch::Tensor> g_ent) {
  IA_CHECK_GPU_F32(z);
  IA_CHECK_CONTIG(z);
  const float* gl = nullptr;
  const float* ge = nullptr;
  torch::Tensor glc, gec;
  if (g_lp.has_value() && g_lp->defined()) {
    glc = g_lp->contiguous().to(torch::kFloat32);
    gl = glc.data_ptr<float>();
  }
  if (g_ent.has_value() && g_ent->defined()) {
    gec = g_ent->contiguous().to(torch::kFloat32);
    ge = gec.data_ptr<float>();
  }
  auto dz = torch::empty_like(z);
  IA_HIP_CHECK(ia::cat_eval_bwd(z.data_ptr<float>(), acts.data_ptr<int64_t>(), (int)z.size(0), (int)z.size(1), gl, ge,
                                 dz.data_ptr<float>(), ia_stream()));
  return dz;
}

// BC loss on a categorical head: metric vector [7] (see rl.hip) from raw logits z [B, A] fp32,
// acts [B] int64 and (optionally) the flat fp32 parameter buffer for l2_norm
py::tuple bc_cat_loss_fwd(torch::Tensor z, torch::Tensor acts, c10::optional<torch::Tensor> flat, double ent_w,
                          double l2_w) {
  IA_CHECK_GPU_F32(z);
  IA_CHECK_CONTIG(z);
  IA_CHECK_CUDA(acts);
  IA_CHECK_CONTIG(acts);
  TORCH_CHECK(z.dim() == 2 && acts.scalar_type() == torch::kInt64 && acts.numel() == z.size(0), "bc_cat_loss shapes");
  TORCH_CHECK(z.size(0) > 0 && z.size(1) <= 64, "bc_cat_loss: 1..64 actions, B > 0");
  const float* fp = nullptr;
  long n = 0;
  if (flat.has_value() && flat->defined()) {
    IA_CHECK_GPU_F32((*flat));
    IA_CHECK_CONTIG((*flat));
    TORCH_CHECK(reinterpret_cast<uintptr_t>(flat->data_ptr()) % 16 == 0, "flat parameter buffer must be 16-B aligned");
    fp = flat->data_ptr<float>();
    n = (long)flat->numel();
  }
  auto out = torch::empty({7}, z.options());
  auto loss = torch::empty({}, z.options());
  auto part = torch::empty({fp ? ia::sumsq_nparts(n) : 1}, z.options());
  IA_HIP_CHECK(ia::bc_cat_loss_fwd(z.data_ptr<float>(), acts.data_ptr<int64_t>(), (int)z.size(0), (int)z.size(1), fp, n,
                                   part.data_ptr<float>(), (float)ent_w, (float)l2_w, out.data_ptr<float>(),
                                   loss.data_ptr<float>(), ia_stream()));
  return py::make_tuple(out, loss);
}

torch::Tensor bc_cat_loss_bwd(torch::Tensor z, torch::Tensor acts, c10::optional<torch::Tensor> g,
                              c10::optional<torch::Tensor> g_loss, double ent_w) {
  IA_CHECK_GPU_F32(z);
  IA_CHECK_CONTIG(z);
  torch::Tensor gc, glc;
  const float* gp = nullptr;
  const float* glp = nullptr;
  if (g.has_value() && g->defined()) {
    gc = g->contiguous().to(torch::kFloat32);
    TORCH_CHECK(gc.numel() == 7 && gc.is_cuda(), "bc_cat_loss_bwd: g must be the [7] metric gradient");
    gp = gc.data_ptr<float>();
  }
  if (g_loss.has_value() && g_loss->defined()) {
    glc = g_loss->contiguous().to(torch::kFloat32);
    TORCH_CHECK(glc.numel() == 1 && glc.is_cuda(), "bc_cat_loss_bwd: g_loss must be a scalar");
    glp = glc.data_ptr<float>();
  }
  auto dz = torch::empty_like(z);
  IA_HIP_CHECK(ia::bc_cat_loss_bwd(z.data_ptr<float>(), acts.data_ptr<int64_t>(), (int)z.size(0), (int)z.size(1), gp, glp,
                                   (float)ent_w, dz.data_ptr<float>(), ia_stream()));
  return dz;
}

// MCE-IRL soft value iteration: T [S, A, S] fp64, R [S] fp64 -> (V [H, S], Q [H, S, A], pi [H, S, A])
py::tuple soft_value_iteration(torch::Tensor T, torch::Tensor R, int64_t H, double gamma) {
  IA_CHECK_CUDA(T);
  IA_CHECK_CONTIG(T);
  IA_CHECK_CUDA(R);
  IA_CHECK_CONTIG(R);
  TORCH_CHECK(T.scalar_type() == torch::kFloat64 && R.scalar_type() == torch::kFloat64, "fp64 T / R");
  TORCH_CHECK(T.dim() == 3 && T.size(0) == T.size(2) && R.dim() == 1 && R.size(0) == T.size(0), "T [S, A, S], R [S]");
  const int S = (int)T.size(0), A = (int)T.size(1);
  TORCH_CHECK(ia::soft_vi_fits(S, A) && H > 0, "soft_value_iteration: S * (A + 1) doubles must fit LDS");
  auto V = torch::empty({H, S}, T.options());
  auto Q = torch::empty({H, S, A}, T.options());
  auto P = torch::empty({H, S, A}, T.options());
  IA_HIP_CHECK(ia::soft_value_iteration(T.data_ptr<double>(), R.data_ptr<double>(), S, A, (int)H, gamma,
                                        V.data_ptr<double>(), Q.data_ptr<double>(), P.data_ptr<double>(), ia_stream()));
  return py::make_tuple(V, Q, P);
}

// MCE-IRL occupancy: T [S, A, S], pi [H, S, A], D0 [S] (fp64) -> D [H + 1, S]
torch::Tensor occupancy_measures(torch::Tensor T, torch::Tensor P, torch::Tensor D0) {
  for (auto* t : {&T, &P, &D0}) {
    IA_CHECK_CUDA((*t));
    IA_CHECK_CONTIG((*t));
    TORCH_CHECK(t->scalar_type() == torch::kFloat64, "occupancy_measures: fp64 inputs");
  }
  TORCH_CHECK(T.dim() == 3 && T.size(0) == T.size(2) && P.dim() == 3 && P.size(1) == T.size(0) && P.size(2) == T.size(1) &&
                  D0.numel() == T.size(0),
              "T [S, A, S], pi [H, S, A], D0 [S]");
  const int S = (int)T.size(0), A = (int)T.size(1), H = (int)P.size(0);
  TORCH_CHECK(ia::soft_vi_fits(S, A), "occupancy_measures: S * (A + 1) doubles must fit LDS");
  auto D = torch::empty({H + 1, S}, T.options());
  IA_HIP_CHECK(ia::occupancy_measures(T.data_ptr<double>(), P.data_ptr<double>(), D0.data_ptr<double>(), S, A, H,
                                      D.data_ptr<double>(), ia_stream()));
  return D;
}

// KDE: q [NQ, d], x [N, d] fp64 -> logsumexp_j log k(|q - x_j| / h) + offset, [NQ]
torch::Tensor kde_score(torch::Tensor q, torch::Tensor x, double bandwidth, int64_t kind, double offset) {
  IA_CHECK_CUDA(q);
  IA_CHECK_CONTIG(q);
  IA_CHECK_CUDA(x);
  IA_CHECK_CONTIG(x);
  TORCH_CHECK(q.scalar_type() == torch::kFloat64 && x.scalar_type() == torch::kFloat64, "kde_score: fp64 inputs");
  TORCH_CHECK(q.dim() == 2 && x.dim() == 2 && q.size(1) == x.size(1), "kde_score: q [NQ, d], x [N, d]");
  const int NQ = (int)q.size(0), N = (int)x.size(0), d = (int)q.size(1);
  TORCH_CHECK(N > 0 && d > 0 && d <= ia::kKdeMaxDim && kind >= 0 && kind <= 5 && bandwidth > 0, "kde_score args");
  auto out = torch::empty({NQ}, q.options());
  if (NQ == 0) return out;
  const int ns = ia::kde_splits(NQ, N);
  auto pm = torch::empty({(int64_t)ns * NQ}, q.options());
  auto ps = torch::empty({(int64_t)ns * NQ}, q.options());
  IA_HIP_CHECK(ia::kde_score(q.data_ptr<double>(), x.data_ptr<double>(), NQ, N, d, 1.0 / bandwidth, (int)kind, offset,
                             pm.data_ptr<double>(), ps.data_ptr<double>(), out.data_ptr<double>(), ia_stream()));
  return out;
}

// rows b (x n_envs + e) of every source [R, ...] -> new [n, ...] tensors, one launch
std::vector<torch::Tensor> gather_rows(std::vector<torch::Tensor> srcs, torch::Tensor b, c10::optional<torch::Tensor> e,
                                       int64_t n_envs, c10::optional<std::vector<torch::Tensor>> dst) {
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= ia::kGatherMax, "gather_rows: 1..8 fields");
  IA_CHECK_CUDA(b);
  IA_CHECK_CONTIG(b);
  TORCH_CHECK(b.scalar_type() == torch::kInt64 && b.dim() == 1, "gather_rows: b int64 [n]");
  const int64_t n = b.numel();
  const int64_t* ep = nullptr;
  if (e.has_value() && e->defined()) {
    IA_CHECK_CUDA((*e));
    IA_CHECK_CONTIG((*e));
    TORCH_CHECK(e->scalar_type() == torch::kInt64 && e->numel() == n && n_envs >= 1, "gather_rows: e int64 [n]");
    ep = e->data_ptr<int64_t>();
  }
  ia::GatherArgs a{};
  a.k = (int)srcs.size();
  std::vector<torch::Tensor> outs;
  for (int i = 0; i < a.k; ++i) {
    auto& t = srcs[i];
    IA_CHECK_CUDA(t);
    IA_CHECK_CONTIG(t);
    TORCH_CHECK(t.dim() >= 1 && t.device() == b.device(), "gather_rows: sources [R, ...] on b's device");
    auto sizes = t.sizes().vec();
    const int64_t rows = sizes[0];
    TORCH_CHECK(rows % (ep ? n_envs : 1) == 0, "gather_rows: rows must be a multiple of n_envs");
    sizes[0] = n;
    torch::Tensor o;
    if (dst.has_value()) {  // caller-owned outputs (persistent buffers, e.g. a graph's static inputs)
      TORCH_CHECK((int)dst->size() == a.k, "gather_rows: one dst per source");
      o = (*dst)[i];
      IA_CHECK_CONTIG(o);
      TORCH_CHECK(o.sizes().vec() == sizes && o.scalar_type() == t.scalar_type() && o.device() == t.device(),
                  "gather_rows: dst ", i, " shape / dtype / device");
    } else {
      o = torch::empty(sizes, t.options());
    }
    a.f[i] = ia::GatherField{t.data_ptr(), o.data_ptr(), rows ? (int64_t)(t.nbytes() / rows) : 0, rows};
    outs.push_back(o);
  }
  IA_HIP_CHECK(ia::gather_rows(a, b.data_ptr<int64_t>(), ep, (int)n_envs, (int)n, ia_stream()));
  return outs;
}

}  // namespace

// (external: conv.cpp's weight-packing launch carries the same gather)
ia::GatherArgs gather_cursor_args(const std::vector<torch::Tensor>& srcs, const torch::Tensor& perm,
                                  const torch::Tensor& cursor, int64_t n, const std::vector<torch::Tensor>& dst,
                                  const c10::optional<torch::Tensor>& inc, float** incp) {
  TORCH_CHECK(!srcs.empty() && (int)srcs.size() <= ia::kGatherMax && dst.size() == srcs.size(), "gather_rows_cursor: 1..8 fields");
  IA_CHECK_CUDA(perm);
  IA_CHECK_CONTIG(perm);
  IA_CHECK_CUDA(cursor);
  TORCH_CHECK(perm.scalar_type() == torch::kInt32 && cursor.scalar_type() == torch::kInt32 && cursor.numel() >= 1,
              "gather_rows_cursor: int32 perm / cursor");
  ia::GatherArgs a{};
  a.k = (int)srcs.size();
  for (int i = 0; i < a.k; ++i) {
    auto& t = srcs[i];
    auto& o = dst[i];
    IA_CHECK_CUDA(t);
    IA_CHECK_CONTIG(t);
    IA_CHECK_CONTIG(o);
    const int64_t rows = t.size(0);
    auto sizes = t.sizes().vec();
    sizes[0] = n;
    TORCH_CHECK(o.sizes().vec() == sizes && o.scalar_type() == t.scalar_type() && o.device() == t.device(),
                "gather_rows_cursor: dst ", i, " shape / dtype / device");
    a.f[i] = ia::GatherField{t.data_ptr(), o.data_ptr(), rows ? (int64_t)(t.nbytes() / rows) : 0, rows};
  }
  *incp = nullptr;
  if (inc && inc->defined()) {
    IA_CHECK_GPU_F32(*inc);
    TORCH_CHECK(inc->numel() == 1, "gather_rows_cursor: inc must be a 1-element fp32 tensor");
    *incp = inc->data_ptr<float>();
  }
  return a;
}

namespace {

// rows perm[*cursor * n + r] of every source into the caller-owned dst tensors (one launch,
// no host arguments per minibatch: HIP-graph epochs)
void gather_rows_cursor(std::vector<torch::Tensor> srcs, torch::Tensor perm, torch::Tensor cursor, int64_t n,
                        std::vector<torch::Tensor> dst, c10::optional<torch::Tensor> inc) {
  float* incp = nullptr;
  const ia::GatherArgs a = gather_cursor_args(srcs, perm, cursor, n, dst, inc, &incp);
  IA_HIP_CHECK(ia::gather_rows_cursor(a, perm.data_ptr<int>(), cursor.data_ptr<int>(), (int)n, ia_stream(), incp));
}

void append_at_cursor(torch::Tensor src, torch::Tensor all, torch::Tensor cursor) {
  IA_CHECK_CUDA(src);
  IA_CHECK_CUDA(all);
  IA_CHECK_CUDA(cursor);
  TORCH_CHECK(src.scalar_type() == torch::kFloat32 && all.scalar_type() == torch::kFloat32 && src.is_contiguous() &&
                  all.is_contiguous() && all.numel() % src.numel() == 0 && cursor.scalar_type() == torch::kInt32,
              "append_at_cursor: fp32 src [n], all [m, n], int32 cursor");
  IA_HIP_CHECK(ia::append_at_cursor(src.data_ptr<float>(), all.data_ptr<float>(), (int)src.numel(), cursor.data_ptr<int>(),
                                    ia_stream()));
}

// RunningNorm: (optionally) merge x's moments into mean / var / count in place, and return
// the normalised x (or None with want_y = false)
py::object running_norm(torch::Tensor x, torch::Tensor mean, torch::Tensor var, torch::Tensor count, double eps,
                        bool update, bool want_y, c10::optional<torch::Tensor> ema_inv_lr,
                        c10::optional<torch::Tensor> ema_num_batches, double ema_decay) {
  IA_CHECK_GPU_F32(x);
  IA_CHECK_CONTIG(x);
  IA_CHECK_GPU_F32(mean);
  IA_CHECK_GPU_F32(var);
  IA_CHECK_CONTIG(mean);
  IA_CHECK_CONTIG(var);
  IA_CHECK_CUDA(count);
  TORCH_CHECK(count.scalar_type() == torch::kInt32 && count.numel() == 1, "running_norm: int32 scalar count");
  TORCH_CHECK(x.dim() == 2 && mean.numel() == x.size(1) && var.numel() == x.size(1), "running_norm: x [B, D]");
  const int B = (int)x.size(0), D = (int)x.size(1);
  TORCH_CHECK(ia::running_norm_ok(B, D), "running_norm: B * D <= 2^20, D <= 256");
  float* inv_lr = nullptr;
  int* nbat = nullptr;
  if (ema_inv_lr && ema_inv_lr->defined()) {
    TORCH_CHECK(ema_num_batches && ema_num_batches->defined(), "running_norm: EMA needs inv_learning_rate and num_batches");
    IA_CHECK_GPU_F32(*ema_inv_lr);
    IA_CHECK_CUDA(*ema_num_batches);
    TORCH_CHECK(ema_inv_lr->numel() == 1 && ema_num_batches->numel() == 1 &&
                    ema_num_batches->scalar_type() == torch::kInt32,
                "running_norm: scalar fp32 inv_learning_rate, int32 num_batches");
    TORCH_CHECK(ema_decay > 0.0 && ema_decay < 1.0, "running_norm: EMA decay in (0, 1)");
    inv_lr = ema_inv_lr->data_ptr<float>();
    nbat = ema_num_batches->data_ptr<int>();
  }
  torch::Tensor y;
  if (want_y) y = torch::empty_like(x);
  // block partials of the multi-workgroup path (caching allocator: graph-capture safe)
  const size_t wsn = update ? ia::running_norm_ws_floats(B, D) : 0;
  torch::Tensor ws;
  if (wsn) ws = torch::empty({(int64_t)wsn}, x.options());
  IA_HIP_CHECK(ia::running_norm(x.data_ptr<float>(), B, D, mean.data_ptr<float>(), var.data_ptr<float>(),
                                count.data_ptr<int>(), (float)eps, update ? 1 : 0, want_y ? y.data_ptr<float>() : nullptr,
                                wsn ? ws.data_ptr<float>() : nullptr, ia_stream(), inv_lr, nbat, (float)ema_decay));
  return want_y ? py::cast(y) : py::none();
}

// Categorical BC head of a CNN policy, fused (bc_head.hip): metrics [7] (BC_METRICS order)
// into `metrics`, dW / db into the gradient slots (written), dh [B, NH] returned.
torch::Tensor bc_head_train(torch::Tensor h, torch::Tensor W, torch::Tensor b, torch::Tensor acts, torch::Tensor params,
                            torch::Tensor dW, torch::Tensor db, torch::Tensor metrics, torch::Tensor ws, double ent_w,
                            double l2_w, c10::optional<torch::Tensor> prof) {
  for (auto* t : {&h, &W, &b, &params, &dW, &db, &metrics, &ws}) {
    IA_CHECK_GPU_F32((*t));
    IA_CHECK_CONTIG((*t));
  }
  IA_CHECK_CUDA(acts);
  TORCH_CHECK(acts.scalar_type() == torch::kInt64 && acts.is_contiguous(), "bc_head_train: int64 actions");
  TORCH_CHECK(h.dim() == 2 && W.dim() == 2 && W.size(1) == h.size(1) && b.numel() == W.size(0) &&
                  acts.numel() == h.size(0) && dW.numel() == W.numel() && db.numel() == b.numel() && metrics.numel() >= 7,
              "bc_head_train: shapes");
  const int B = (int)h.size(0), NH = (int)h.size(1), A = (int)W.size(0);
  TORCH_CHECK(ia::bc_head_ok(B, NH, A), "bc_head_train: B <= 64, NH 256 or 512, A <= 8");
  const long n = (long)params.numel();
  const int nb = ia::bc_head_sumsq_blocks(n);
  TORCH_CHECK(ws.numel() >= nb + 1, "bc_head_train: workspace of bc_head_workspace(n_params) floats");
  TORCH_CHECK(((uintptr_t)h.data_ptr() | (uintptr_t)W.data_ptr() | (uintptr_t)params.data_ptr()) % 16 == 0,
              "bc_head_train: h / W / params 16-B aligned");
  auto dh = torch::empty_like(h);
  ia::BcHeadArgs a{};
  a.h = h.data_ptr<float>();
  a.W = W.data_ptr<float>();
  a.b = b.data_ptr<float>();
  a.acts = acts.data_ptr<int64_t>();
  a.B = B;
  a.NH = NH;
  a.A = A;
  a.ent_w = (float)ent_w;
  a.l2_w = (float)l2_w;
  a.params = params.data_ptr<float>();
  a.n_params = n;
  a.dW = dW.data_ptr<float>();
  a.db = db.data_ptr<float>();
  a.dh = dh.data_ptr<float>();
  a.metrics = metrics.data_ptr<float>();
  a.cnt = reinterpret_cast<unsigned*>(ws.data_ptr<float>());  // word 0: counter (zeroed by the caller once)
  a.partials = ws.data_ptr<float>() + 1;
  if (prof && prof->defined()) {
    TORCH_CHECK(prof->is_cuda() && prof->scalar_type() == torch::kInt64 && prof->numel() >= 8, "prof: int64 [8]");
    a.prof = reinterpret_cast<long long*>(prof->data_ptr<int64_t>());
  }
  IA_HIP_CHECK(ia::bc_head_train(a, ia_stream()));
  return dh;
}

// [E, n] int32: row e is a pseudo-random permutation of 0..n-1 keyed by (seed, e).
torch::Tensor random_permutations(int64_t E, int64_t n, int64_t seed, torch::Device device) {
  TORCH_CHECK(device.is_cuda(), "random_permutations runs on the GPU");
  TORCH_CHECK(E >= 0 && n >= 0 && n <= (1ll << 30), "bad permutation shape");
  auto out = torch::empty({E, n}, torch::TensorOptions().dtype(torch::kInt32).device(device));
  IA_HIP_CHECK(ia::perm_feistel((int)E, (int)n, (uint64_t)seed, out.data_ptr<int>(), ia_stream()));
  return out;
}

// Returns (probs [P], losses [P], coef [P]).
py::tuple pref_loss_fwd(torch::Tensor r1, torch::Tensor r2, torch::Tensor prefs, double discount, double threshold,
                        double noise) {
  IA_CHECK_GPU_F32(r1);
  IA_CHECK_GPU_F32(r2);
  IA_CHECK_GPU_F32(prefs);
  TORCH_CHECK(r1.dim() == 2 && r1.sizes() == r2.sizes(), "r1/r2 must be [P, L] of equal shape");
  const int P = (int)r1.size(0), L = (int)r1.size(1);
  TORCH_CHECK(prefs.numel() == P, "one preference per pair");
  auto probs = torch::empty({P}, r1.options());
  auto losses = torch::empty({P}, r1.options());
  auto coef = torch::empty({P}, r1.options());
  IA_HIP_CHECK(ia::pref_loss_fwd(r1.data_ptr<float>(), r2.data_ptr<float>(), prefs.data_ptr<float>(), P, L,
                                 (float)discount, (float)threshold, (float)noise, probs.data_ptr<float>(),
                                 losses.data_ptr<float>(), coef.data_ptr<float>(), ia_stream()));
  return py::make_tuple(probs, losses, coef);
}

py::tuple pref_loss_bwd(torch::Tensor coef, torch::Tensor gout, int64_t L, double discount) {
  IA_CHECK_GPU_F32(coef);
  IA_CHECK_GPU_F32(gout);
  const int P = (int)coef.numel();
  auto d1 = torch::empty({P, L}, coef.options());
  auto d2 = torch::empty({P, L}, coef.options());
  IA_HIP_CHECK(ia::pref_loss_bwd(coef.data_ptr<float>(), gout.data_ptr<float>(), P, (int)L, (float)discount,
                                 d1.data_ptr<float>(), d2.data_ptr<float>(), ia_stream()));
  return py::make_tuple(d1, d2);
}

}  // namespace

void register_kernels(py::module& m) {
  m.def("pref_loss_fwd", &pref_loss_fwd, py::arg("r1"), py::arg("r2"), py::arg("prefs"), py::arg("discount"),
        py::arg("threshold"), py::arg("noise"));
  m.def("pref_loss_bwd", &pref_loss_bwd, py::arg("coef"), py::arg("gout"), py::arg("L"), py::arg("discount"));
  m.def("tmlp_forward", &tmlp_forward, py::arg("x"), py::arg("weights"), py::arg("biases"), py::arg("hidden_act"),
        py::arg("out_act"), py::arg("norm_mean") = py::none(), py::arg("norm_var") = py::none(),
        py::arg("norm_eps") = 1e-5, py::arg("norm_clip") = 0.0);
  m.def("tmlp_backward", &tmlp_backward, py::arg("x"), py::arg("dy"), py::arg("weights"), py::arg("biases"),
        py::arg("hidden_act"), py::arg("out_act"), py::arg("norm_mean") = py::none(), py::arg("norm_var") = py::none(),
        py::arg("norm_eps") = 1e-5, py::arg("norm_clip") = 0.0, py::arg("need_dx") = false);
  m.def("tmlp_forward_grouped", &tmlp_forward_grouped, py::arg("x"), py::arg("weights"), py::arg("biases"),
        py::arg("hidden_act"), py::arg("out_act"), py::arg("norm_mean") = py::none(), py::arg("norm_var") = py::none(),
        py::arg("norm_eps") = 1e-5);
  m.def("tmlp_backward_grouped", &tmlp_backward_grouped, py::arg("x"), py::arg("dy"), py::arg("weights"), py::arg("biases"),
        py::arg("hidden_act"), py::arg("out_act"), py::arg("norm_mean") = py::none(), py::arg("norm_var") = py::none(),
        py::arg("norm_eps") = 1e-5, py::arg("need_dx") = false);
  m.def("gae", &gae, py::arg("rewards"), py::arg("values"), py::arg("episode_starts"), py::arg("last_values"),
        py::arg("dones"), py::arg("gamma"), py::arg("lam"), py::arg("moments") = py::none());
  m.def("adam_flat", &adam_flat, py::arg("params"), py::arg("grads"), py::arg("exp_avg"), py::arg("exp_avg_sq"),
        py::arg("step"), py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"),
        py::arg("decoupled"), py::arg("maximize"), py::arg("zero_grad"), py::arg("step_cnt") = py::none(),
        py::arg("append_src") = py::none(), py::arg("append_all") = py::none(), py::arg("append_cursor") = py::none(),
        py::arg("reduce") = py::none());
  m.def("random_permutations", &random_permutations, py::arg("E"), py::arg("n"), py::arg("seed"), py::arg("device"));
  m.def("running_norm", &running_norm, py::arg("x"), py::arg("mean"), py::arg("var"), py::arg("count"), py::arg("eps"),
        py::arg("update"), py::arg("want_y"), py::arg("ema_inv_lr") = py::none(), py::arg("ema_num_batches") = py::none(),
        py::arg("ema_decay") = 0.0);
  m.def("gather_rows_cursor", &gather_rows_cursor, "rows perm[*cursor * n ..] of every source into dst (graph epochs)",
        py::arg("srcs"), py::arg("perm"), py::arg("cursor"), py::arg("n"), py::arg("dst"), py::arg("inc") = py::none());
  m.def("append_at_cursor", &append_at_cursor, "all[*cursor] = src; ++*cursor");
  m.def("gather_rows", &gather_rows, py::arg("srcs"), py::arg("b"), py::arg("e") = py::none(), py::arg("n_envs") = 1,
        py::arg("dst") = py::none());
  m.def("soft_value_iteration", &soft_value_iteration, py::arg("T"), py::arg("R"), py::arg("H"), py::arg("gamma"));
  m.def("occupancy_measures", &occupancy_measures, py::arg("T"), py::arg("P"), py::arg("D0"));
  m.def("kde_score", &kde_score, py::arg("q"), py::arg("x"), py::arg("bandwidth"), py::arg("kind"), py::arg("offset"));
  m.def("bc_cat_loss_fwd", &bc_cat_loss_fwd, py::arg("z"), py::arg("acts"), py::arg("flat"), py::arg("ent_w"),
        py::arg("l2_w"));
  m.def("bc_cat_loss_bwd", &bc_cat_loss_bwd, py::arg("z"), py::arg("acts"), py::arg("g"), py::arg("g_loss"),
        py::arg("ent_w"));
  m.def("bc_head_train", &bc_head_train, py::arg("h"), py::arg("W"), py::arg("b"), py::arg("acts"), py::arg("params"),
        py::arg("dW"), py::arg("db"), py::arg("metrics"), py::arg("ws"), py::arg("ent_w"), py::arg("l2_w"), py::arg("prof") = py::none());
  m.def("bc_head_workspace", [](int64_t n) { return (int64_t)ia::bc_head_sumsq_blocks((long)n) + 1; });
  m.def("cat_eval_fwd", &cat_eval_fwd, py::arg("z"), py::arg("acts"));
  m.def("cat_eval_bwd", &cat_eval_bwd, py::arg("z"), py::arg("acts"), py::arg("g_lp"), py::arg("g_ent"));
}

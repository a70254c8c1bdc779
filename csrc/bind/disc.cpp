// DiscPlan: the fused discriminator update of the device adversarial engine
// (csrc/kernels/disc.hip + tmlp_disc_fwd_bwd). Built once per trainer from a dict of
// persistent tensors (expert set, replay ring, flat reward-net params / Adam moments,
// running-norm buffers, workspaces); each update then only passes the sampled indices
// and the two Adam scalars, so the per-update host cost is one pybind call.
#include "common.h"
#include "launchers.h"

namespace {

#define IA_HIP_CHECK3(expr)                                                           \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e)); \
  } while (0)

class DiscPlan {
 public:
  explicit DiscPlan(py::dict d) {
    auto keep = [&](const char* k, bool optional = false) -> torch::Tensor {
      if (!d.contains(k) || d[k].is_none()) {
        TORCH_CHECK(optional, "disc plan arg missing: ", k);
        return torch::Tensor();
      }
      auto t = d[k].cast<torch::Tensor>();
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "disc plan arg ", k, " must be a contiguous GPU tensor");
      held_.push_back(t);
      return t;
    };
    auto fptr = [&](const char* k, bool optional = false) -> float* {
      auto t = keep(k, optional);
      if (!t.defined()) return nullptr;
      TORCH_CHECK(t.scalar_type() == torch::kFloat32, k, " must be float32");
      return t.data_ptr<float>();
    };
    auto iptr = [&](const char* k, bool optional = false) -> int* {
      auto t = keep(k, optional);
      if (!t.defined()) return nullptr;
      TORCH_CHECK(t.scalar_type() == torch::kInt32, k, " must be int32");
      return t.data_ptr<int>();
    };
    B_ = d["batch"].cast<int>();
    mb_ = d["minibatch"].cast<int>();
    TORCH_CHECK(mb_ > 0 && B_ % mb_ == 0, "batch must be a multiple of the minibatch");
    n_mb_ = B_ / mb_;

    // MLP (weights are views into the flat parameter buffer)
    auto Ws = d["W"].cast<std::vector<torch::Tensor>>();
    auto bs = d["b"].cast<std::vector<torch::Tensor>>();
    TORCH_CHECK(!Ws.empty() && Ws.size() <= (size_t)ia::kMaxLayers && Ws.size() == bs.size(), "1..4 layers");
    desc_ = ia::MLPDesc{};
    desc_.n_layers = (int)Ws.size();
    desc_.dims[0] = (int)Ws[0].size(1);
    for (size_t l = 0; l < Ws.size(); ++l) {
      held_.push_back(Ws[l]);
      held_.push_back(bs[l]);
      desc_.dims[l + 1] = (int)Ws[l].size(0);
      desc_.W[l] = Ws[l].data_ptr<float>();
      desc_.b[l] = bs[l].data_ptr<float>();
    }
    for (int l = 0; l <= desc_.n_layers; ++l) TORCH_CHECK(desc_.dims[l] <= ia::kMaxDim, "width <= 128");
    TORCH_CHECK(desc_.dims[desc_.n_layers] == 1, "discriminator must output one logit");
    desc_.hidden_act = d["hidden_act"].cast<int>();
    desc_.out_act = 0;
    desc_.norm_mean = fptr("rew_mean", true);
    desc_.norm_var = fptr("rew_var", true);
    desc_.norm_eps = (float)d["rew_eps"].cast<double>();
    desc_.norm_clip = 0.f;

    // gather
    g_ = ia::DiscGatherArgs{};
    g_.mb = mb_;
    g_.din = desc_.dims[0];
    g_.obs_dim = d["obs_dim"].cast<int>();
    g_.act_width = d["act_width"].cast<int>();
    g_.use_state = d["use_state"].cast<int>();
    g_.use_action = d["use_action"].cast<int>();
    g_.use_next_state = d["use_next_state"].cast<int>();
    g_.use_done = d["use_done"].cast<int>();
    g_.act_discrete = d["act_discrete"].cast<int>();
    const int din = g_.use_state * g_.obs_dim + g_.use_action * g_.act_width + g_.use_next_state * g_.obs_dim + g_.use_done;
    TORCH_CHECK(din == g_.din, "reward-net input width ", g_.din, " != gathered width ", din);
    g_.e_obs = fptr("e_obs");
    g_.e_next_obs = fptr("e_next_obs");
    g_.e_dones = reinterpret_cast<const bool*>(keep("e_dones").data_ptr());
    g_.g_obs = fptr("g_obs");
    g_.g_next_obs = fptr("g_next_obs");
    g_.g_dones = reinterpret_cast<const bool*>(keep("g_dones").data_ptr());
    if (g_.act_discrete) {
      g_.e_acts_i = keep("e_acts").data_ptr<int64_t>();
      g_.g_acts_i = keep("g_acts").data_ptr<int64_t>();
    } else {
      g_.e_acts = fptr("e_acts");
      g_.g_acts = fptr("g_acts");
    }
    g_.shift = desc_.norm_mean;
    g_.X = fptr("X");
    g_.partials = fptr("partials");
    TORCH_CHECK(held_.back().numel() >= (int64_t)ia::disc_gather_blocks(mb_) * 2 * g_.din, "partials too small");

    // norms
    n_ = ia::DiscNormArgs{};
    n_.mb = mb_;
    n_.din = g_.din;
    n_.nblk = ia::disc_gather_blocks(mb_);
    n_.partials = g_.partials;
    n_.shift = desc_.norm_mean;
    n_.rew_mean = const_cast<float*>(desc_.norm_mean);
    n_.rew_var = const_cast<float*>(desc_.norm_var);
    n_.rew_count = iptr("rew_count", true);
    n_.pol_mean = fptr("pol_mean", true);
    n_.pol_var = fptr("pol_var", true);
    n_.pol_count = iptr("pol_count", true);
    n_.pol_cols = g_.use_state ? g_.obs_dim : 0;
    auto sums = keep("sums", true);
    n_.sums = sums.defined() ? sums.data_ptr<double>() : nullptr;

    // fwd/bwd + Adam
    fb_blocks_ = ia::tmlp_disc_blocks(desc_, 2 * mb_);
    slab_ = fptr("slab");
    stats_slab_ = fptr("stats_slab");
    const ia::TmlpPlan p = ia::plan_tmlp(desc_, 4);
    n_params_ = p.n_params;
    TORCH_CHECK(held_[held_.size() - 2].numel() >= (int64_t)n_mb_ * fb_blocks_ * n_params_, "slab too small");
    TORCH_CHECK(held_.back().numel() >= (int64_t)n_mb_ * fb_blocks_ * ia::kDiscStats, "stats slab too small");
    a_ = ia::DiscAdamArgs{};
    a_.n_params = n_params_;
    a_.nblk = n_mb_ * fb_blocks_;
    a_.stats_nblk = fb_blocks_;
    a_.slab = slab_;
    a_.stats_slab = stats_slab_ + (size_t)(n_mb_ - 1) * fb_blocks_ * ia::kDiscStats;
    a_.grads = fptr("grads");
    a_.params = fptr("params");
    TORCH_CHECK(held_.back().numel() == n_params_, "flat params size ", held_.back().numel(), " != ", n_params_);
    a_.exp_avg = fptr("exp_avg");
    a_.exp_avg_sq = fptr("exp_avg_sq");
    a_.beta1 = (float)d["beta1"].cast<double>();
    a_.beta2 = (float)d["beta2"].cast<double>();
    a_.eps = (float)d["eps"].cast<double>();
    a_.weight_decay = (float)d["weight_decay"].cast<double>();
    scale_ = (float)((double)mb_ / (double)B_ / (double)(2 * mb_));  // mean BCE * mb / B
  }

  int n_params() const { return n_params_; }
  int n_minibatches() const { return n_mb_; }
  int pol_cols() const { return n_.pol_cols; }
  // [slots, 2 * pol_cols + 1] float32 record buffer for deferred policy-norm merges
  void set_pol_defer(torch::Tensor t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kFloat32 && t.dim() == 2 &&
                    t.size(1) == 2 * n_.pol_cols + 1,
                "pol_defer must be a contiguous float32 GPU tensor [slots, 2 * pol_cols + 1]");
    defer_ = t;
    defer_slots_ = (int)t.size(0);
  }
  // apply slots [0, n_slots) of the deferred records to the policy RunningNorm, in order
  void pol_norm_merge(int n_slots) {
    TORCH_CHECK(defer_.defined() && n_slots <= defer_slots_, "pol_norm_merge: bad slot count");
    TORCH_CHECK(n_.pol_mean && n_.pol_count, "plan has no policy norm");
    IA_HIP_CHECK3(ia::pol_norm_merge(n_.pol_mean, n_.pol_var, n_.pol_count, defer_.data_ptr<float>(), n_slots,
                                     n_.pol_cols, ia_stream()));
  }

  // One minibatch: gather + (local) moments + norm merge, or DP split via `sums`.
  void gather(int k, torch::Tensor e_idx, torch::Tensor g_idx) {
    check_idx(e_idx);
    check_idx(g_idx);
    ia::DiscGatherArgs g = g_;
    g.e_idx = e_idx.data_ptr<int64_t>() + (size_t)k * mb_;
    g.g_idx = g_idx.data_ptr<int64_t>() + (size_t)k * mb_;
    IA_HIP_CHECK3(ia::disc_gather(g, ia_stream()));
  }
  // merge_rew / merge_pol: whether each RunningNorm is in training mode (updates its stats)
  // pol_defer_slot >= 0: the policy-norm merge is recorded into slot k of the buffer set by
  // set_pol_defer (applied later by pol_norm_merge) instead of done in place
  void norm(int mode, int n_total, bool merge_rew, bool merge_pol, int pol_defer_slot = -1) {
    ia::DiscNormArgs n = n_;
    n.pol_defer = nullptr;
    if (merge_pol && pol_defer_slot >= 0) {
      TORCH_CHECK(defer_.defined() && pol_defer_slot < defer_slots_, "pol_defer slot ", pol_defer_slot, " out of range");
      n.pol_defer = defer_.data_ptr<float>() + (size_t)pol_defer_slot * (2 * n_.pol_cols + 1);
    }
    n.mode = mode;
    n.n_total = n_total;
    if (!merge_rew) {
      n.rew_mean = n.rew_var = nullptr;
      n.rew_count = nullptr;
    }
    if (!merge_pol) {
      n.pol_mean = n.pol_var = nullptr;
      n.pol_count = nullptr;
    }
    TORCH_CHECK(mode == 0 || n.sums != nullptr, "DP norm modes need the sums buffer");
    IA_HIP_CHECK3(ia::disc_norm(n, ia_stream()));
  }
  void fwd_bwd(int k) {
    ia::DiscLoss dl{mb_, scale_, stats_slab_ + (size_t)k * fb_blocks_ * ia::kDiscStats};
    IA_HIP_CHECK3(ia::tmlp_disc_fwd_bwd(desc_, g_.X, 2 * mb_, dl, slab_ + (size_t)k * fb_blocks_ * n_params_, ia_stream()));
  }
  // reduce=1: slab -> grads (adam=0) or straight into Adam (adam=1); reduce=0: Adam from grads.
  void adam(int reduce, int do_adam, double step_size, double bc2_sqrt, c10::optional<torch::Tensor> stats_out) {
    ia::DiscAdamArgs a = a_;
    a.reduce = reduce;
    a.adam = do_adam;
    a.step_size = (float)step_size;
    a.bc2_sqrt = (float)bc2_sqrt;
    a.stats_out = nullptr;
    if (stats_out.has_value() && stats_out->defined()) {
      TORCH_CHECK(stats_out->is_cuda() && stats_out->scalar_type() == torch::kFloat32 &&
                      stats_out->numel() >= ia::kDiscStats && stats_out->is_contiguous(),
                  "stats_out must be a float32 GPU tensor of >= 8 elements");
      a.stats_out = stats_out->data_ptr<float>();
    }
    IA_HIP_CHECK3(ia::disc_adam(a, ia_stream()));
  }
  // Whole single-rank update: all minibatches + Adam, 3 launches per minibatch + 1.
  void update(torch::Tensor e_idx, torch::Tensor g_idx, double step_size, double bc2_sqrt, bool merge_rew, bool merge_pol,
              c10::optional<torch::Tensor> stats_out, int pol_defer_base = -1) {
    for (int k = 0; k < n_mb_; ++k) {
      gather(k, e_idx, g_idx);
      if (merge_rew || merge_pol) norm(0, 0, merge_rew, merge_pol, pol_defer_base < 0 ? -1 : pol_defer_base + k);
      fwd_bwd(k);
    }
    adam(1, 1, step_size, bc2_sqrt, stats_out);
  }

 private:
  void check_idx(const torch::Tensor& t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kInt64 && t.numel() >= B_,
                "indices must be int64 GPU tensors of >= batch entries");
  }
  std::vector<torch::Tensor> held_;
  torch::Tensor defer_;
  int defer_slots_ = 0;
  ia::MLPDesc desc_{};
  ia::DiscGatherArgs g_{};
  ia::DiscNormArgs n_{};
  ia::DiscAdamArgs a_{};
  float* slab_ = nullptr;
  float* stats_slab_ = nullptr;
  int B_ = 0, mb_ = 0, n_mb_ = 0, fb_blocks_ = 0, n_params_ = 0;
  float scale_ = 0.f;
};

// Workspace sizes for a configuration: (gather blocks, fwd/bwd blocks per minibatch, n_params).
py::tuple disc_plan_sizes(std::vector<int> dims, int minibatch) {
  ia::MLPDesc d{};
  d.n_layers = (int)dims.size() - 1;
  TORCH_CHECK(d.n_layers >= 1 && d.n_layers <= ia::kMaxLayers, "1..4 layers");
  for (int l = 0; l <= d.n_layers; ++l) d.dims[l] = dims[l];
  const ia::TmlpPlan p = ia::plan_tmlp(d, 4);
  return py::make_tuple(ia::disc_gather_blocks(minibatch), ia::tmlp_disc_blocks(d, 2 * minibatch), p.n_params);
}

}  // namespace

void register_disc(py::module& m) {
  py::class_<DiscPlan>(m, "DiscPlan")
      .def(py::init<py::dict>())
      .def_property_readonly("n_params", &DiscPlan::n_params)
      .def("gather", &DiscPlan::gather)
      .def_property_readonly("n_minibatches", &DiscPlan::n_minibatches)
      .def_property_readonly("pol_cols", &DiscPlan::pol_cols)
      .def("set_pol_defer", &DiscPlan::set_pol_defer)
      .def("pol_norm_merge", &DiscPlan::pol_norm_merge, py::arg("n_slots"))
      .def("norm", &DiscPlan::norm, py::arg("mode"), py::arg("n_total"), py::arg("merge_rew"), py::arg("merge_pol"),
           py::arg("pol_defer_slot") = -1)
      .def("fwd_bwd", &DiscPlan::fwd_bwd)
      .def("adam", &DiscPlan::adam, py::arg("reduce"), py::arg("do_adam"), py::arg("step_size"), py::arg("bc2_sqrt"),
           py::arg("stats_out") = py::none())
      .def("update", &DiscPlan::update, py::arg("e_idx"), py::arg("g_idx"), py::arg("step_size"), py::arg("bc2_sqrt"),
           py::arg("merge_rew"), py::arg("merge_pol"), py::arg("stats_out") = py::none(), py::arg("pol_defer_base") = -1);
  m.def("disc_plan_sizes", &disc_plan_sizes, py::arg("dims"), py::arg("minibatch"));
}

// AirlDiscPlan: the fused AIRL discriminator update (csrc/kernels/airl_disc.hip + the Adam of
// disc.hip). Built once per trainer from a dict of persistent tensors (expert set, replay
// ring, policy / base / potential weights, running-norm buffers, flat reward parameters and
// Adam moments, workspaces); an update then passes only the sampled indices and the two Adam
// scalars: one pybind call, 3 launches per minibatch + 1.
#include "common.h"
#include "launchers.h"

namespace {

#define IA_HIP_CHECK_A(expr)                                                          \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e)); \
  } while (0)

class AirlDiscPlan {
 public:
  explicit AirlDiscPlan(py::dict d) {
    auto keep = [&](py::dict& src, const char* k, bool optional = false) -> torch::Tensor {
      if (!src.contains(k) || src[k].is_none()) {
        TORCH_CHECK(optional, "airl plan arg missing: ", k);
        return torch::Tensor();
      }
      auto t = src[k].cast<torch::Tensor>();
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "airl plan arg ", k, " must be a contiguous GPU tensor");
      held_.push_back(t);
      return t;
    };
    auto fptr = [&](const char* k, bool optional = false) -> float* {
      auto t = keep(d, k, optional);
      if (!t.defined()) return nullptr;
      TORCH_CHECK(t.scalar_type() == torch::kFloat32, k, " must be float32");
      return t.data_ptr<float>();
    };
    auto iptr = [&](const char* k, bool optional = false) -> int* {
      auto t = keep(d, k, optional);
      if (!t.defined()) return nullptr;
      TORCH_CHECK(t.scalar_type() == torch::kInt32, k, " must be int32");
      return t.data_ptr<int>();
    };
    auto net = [&](const char* k, int* off) -> ia::AirlNet {
      py::dict nd = d[k].cast<py::dict>();
      auto Ws = nd["W"].cast<std::vector<torch::Tensor>>();
      auto bs = nd["b"].cast<std::vector<torch::Tensor>>();
      TORCH_CHECK(!Ws.empty() && Ws.size() <= (size_t)ia::kAirlMaxLayers && Ws.size() == bs.size(), k, ": 1..4 layers");
      ia::AirlNet n{};
      n.n_layers = (int)Ws.size();
      n.dims[0] = (int)Ws[0].size(1);
      n.hidden_act = nd["hidden_act"].cast<int>();
      n.param_off = off ? *off : 0;
      int o = 0;
      for (size_t l = 0; l < Ws.size(); ++l) {
        TORCH_CHECK(Ws[l].is_cuda() && Ws[l].is_contiguous() && Ws[l].scalar_type() == torch::kFloat32, k, " weights");
        TORCH_CHECK(l == 0 || Ws[l].size(1) == Ws[l - 1].size(0), k, ": layer widths do not chain");
        held_.push_back(Ws[l]);
        held_.push_back(bs[l]);
        n.dims[l + 1] = (int)Ws[l].size(0);
        n.W[l] = Ws[l].data_ptr<float>();
        n.b[l] = bs[l].data_ptr<float>();
        n.w_off[l] = o;
        o += (int)Ws[l].numel();
        n.b_off[l] = o;
        o += (int)bs[l].numel();
      }
      if (off) *off += o;
      return n;
    };
    B_ = d["batch"].cast<int>();
    mb_ = d["minibatch"].cast<int>();
    TORCH_CHECK(mb_ > 0 && B_ % mb_ == 0, "batch must be a multiple of the minibatch");
    n_mb_ = B_ / mb_;
    a_ = ia::AirlDiscArgs{};
    a_.mb = mb_;
    a_.D = d["obs_dim"].cast<int>();
    a_.A = d["act_dim"].cast<int>();
    a_.act_discrete = d["act_discrete"].cast<int>();
    a_.aw = a_.A;  // Box width, or n_actions (one-hot in the base input)
    a_.aw_pi = a_.act_discrete ? 1 : a_.A;
    a_.use_state = d["use_state"].cast<int>();
    a_.use_action = d["use_action"].cast<int>();
    a_.use_next_state = d["use_next_state"].cast<int>();
    a_.use_done = d["use_done"].cast<int>();
    a_.din_b = a_.use_state * a_.D + a_.use_action * a_.aw + a_.use_next_state * a_.D + a_.use_done;
    a_.e_obs = fptr("e_obs");
    a_.e_next_obs = fptr("e_next_obs");
    a_.e_dones = reinterpret_cast<const bool*>(keep(d, "e_dones").data_ptr());
    a_.g_obs = fptr("g_obs");
    a_.g_next_obs = fptr("g_next_obs");
    a_.g_dones = reinterpret_cast<const bool*>(keep(d, "g_dones").data_ptr());
    if (a_.act_discrete) {
      a_.e_acts_i = keep(d, "e_acts").data_ptr<int64_t>();
      a_.g_acts_i = keep(d, "g_acts").data_ptr<int64_t>();
    } else {
      a_.e_acts = fptr("e_acts");
      a_.g_acts = fptr("g_acts");
    }
    // nets: the flat reward parameter order is base (W0, b0, W1, b1, ...) then potential
    int off = 0;
    a_.pol = net("pol", nullptr);
    a_.base = net("base", &off);
    a_.pot = net("pot", &off);
    a_.n_params = off;
    TORCH_CHECK(a_.base.dims[0] == a_.din_b, "base-net input width ", a_.base.dims[0], " != gathered width ", a_.din_b);
    TORCH_CHECK(a_.pot.dims[0] == a_.D && a_.pol.dims[0] == a_.D, "potential / policy input must be the observation");
    a_.log_std = fptr("log_std", true);
    TORCH_CHECK(a_.act_discrete || a_.log_std != nullptr, "Gaussian policy needs log_std");
    a_.gamma = (float)d["gamma"].cast<double>();
    // norms
    a_.b_mean = fptr("b_mean", true);
    a_.b_var = fptr("b_var", true);
    a_.b_count = iptr("b_count", true);
    a_.p_mean = fptr("p_mean", true);
    a_.p_var = fptr("p_var", true);
    a_.p_count = iptr("p_count", true);
    a_.q_mean = fptr("q_mean", true);
    a_.q_var = fptr("q_var", true);
    a_.q_count = iptr("q_count", true);
    a_.eps_b = (float)d["eps_b"].cast<double>();
    a_.eps_p = (float)d["eps_p"].cast<double>();
    a_.eps_q = (float)d["eps_q"].cast<double>();
    // workspaces
    const int n = 2 * mb_, ncol = a_.din_b + 2 * a_.D;
    auto need = [&](const char* k, int64_t numel) {
      TORCH_CHECK(held_.back().numel() >= numel, k, " too small: ", held_.back().numel(), " < ", numel);
    };
    a_.Xb = fptr("Xb");
    need("Xb", (int64_t)n * a_.din_b);
    a_.S = fptr("S");
    need("S", (int64_t)n * a_.D);
    a_.S2 = fptr("S2");
    need("S2", (int64_t)n * a_.D);
    a_.Act = fptr("Act");
    need("Act", (int64_t)n * a_.aw_pi);
    a_.Done = fptr("Done");
    need("Done", n);
    a_.gather_blocks = ia::airl_gather_blocks(mb_);
    a_.partials = fptr("partials");
    need("partials", (int64_t)a_.gather_blocks * 2 * ncol);
    auto sums = keep(d, "sums", true);
    if (sums.defined()) {
      TORCH_CHECK(sums.scalar_type() == torch::kFloat64 && sums.numel() >= 2 * ncol, "sums: float64 [2 * cols]");
      a_.sums = sums.data_ptr<double>();
    }
    a_.nrm = fptr("nrm");
    need("nrm", 4 * 256);
    fb_blocks_ = ia::airl_fwd_blocks(mb_);
    a_.slab = fptr("slab");
    need("slab", (int64_t)n_mb_ * fb_blocks_ * a_.n_params);
    a_.stats_slab = fptr("stats_slab");
    need("stats_slab", (int64_t)n_mb_ * fb_blocks_ * ia::kDiscStats);
    a_.scale = (float)((double)mb_ / (double)B_ / (double)(2 * mb_));
    TORCH_CHECK(ia::airl_plan(a_, plan_), "AIRL discriminator outside the fused kernel's limits (widths <= 64, <= 4 "
                                          "layers, <= 16 actions, din + 2 obs <= 128)");
    // Adam (disc.hip)
    ad_ = ia::DiscAdamArgs{};
    ad_.n_params = a_.n_params;
    ad_.nblk = n_mb_ * fb_blocks_;
    ad_.stats_nblk = fb_blocks_;
    ad_.slab = a_.slab;
    ad_.stats_slab = a_.stats_slab + (size_t)(n_mb_ - 1) * fb_blocks_ * ia::kDiscStats;
    ad_.grads = fptr("grads");
    need("grads", a_.n_params);
    ad_.params = fptr("params");
    TORCH_CHECK(held_.back().numel() == a_.n_params, "flat params size ", held_.back().numel(), " != ", a_.n_params);
    ad_.exp_avg = fptr("exp_avg");
    ad_.exp_avg_sq = fptr("exp_avg_sq");
    ad_.beta1 = (float)d["beta1"].cast<double>();
    ad_.beta2 = (float)d["beta2"].cast<double>();
    ad_.eps = (float)d["eps"].cast<double>();
    ad_.weight_decay = (float)d["weight_decay"].cast<double>();
  }

  int n_params() const { return a_.n_params; }
  int n_minibatches() const { return n_mb_; }
  int lds_bytes() const { return plan_.lds_bytes; }
  // phase cycle counters of the fwd/bwd kernel (block 0): int64 GPU tensor [8] or None
  void set_prof(c10::optional<torch::Tensor> t) {
    if (!t.has_value() || !t->defined()) {
      a_.prof = nullptr;
      return;
    }
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == torch::kInt64 && t->numel() >= 8, "prof: int64 GPU tensor [8]");
    prof_ = *t;
    a_.prof = reinterpret_cast<unsigned long long*>(prof_.data_ptr<int64_t>());
  }

  void gather(int k, torch::Tensor e_idx, torch::Tensor g_idx) {
    check_idx(e_idx);
    check_idx(g_idx);
    ia::AirlDiscArgs a = a_;
    a.e_idx = e_idx.data_ptr<int64_t>();
    a.g_idx = g_idx.data_ptr<int64_t>();
    IA_HIP_CHECK_A(ia::airl_gather(a, k, ia_stream()));
  }
  // mode 0: local moments + merges; 1: moments -> sums (all-reduce them); 2: merges from sums
  void norm(int mode, int n_total, bool merge_b, bool merge_p, bool merge_q) {
    ia::AirlDiscArgs a = a_;
    a.merge_b = merge_b;
    a.merge_p = merge_p;
    a.merge_q = merge_q;
    TORCH_CHECK(mode == 0 || a.sums != nullptr, "DP norm modes need the sums buffer");
    IA_HIP_CHECK_A(ia::airl_norm(a, mode, n_total, ia_stream()));
  }
  void fwd_bwd(int k) { IA_HIP_CHECK_A(ia::airl_fwd_bwd(a_, plan_, k, ia_stream())); }
  void adam(int reduce, int do_adam, double step_size, double bc2_sqrt, c10::optional<torch::Tensor> stats_out) {
    ia::DiscAdamArgs a = ad_;
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
    IA_HIP_CHECK_A(ia::disc_adam(a, ia_stream()));
  }
  // Split update (single rank): stage(i) runs update i's gathers and norm merges -- the only
  // part of an update that touches the running norms, none of it depends on the disc weights --
  // into per-(update, minibatch) workspaces; apply(i) then runs the fwd/bwd passes and the Adam
  // step from them. All stages of a round followed by all applies are the same launches on the
  // same data as update() x n (bitwise), but the policy norm (q, merged as a side effect of the
  // log pi pass, as the reference's training-mode evaluate_actions does) is final after the
  // stages: the next rollout's step chain can run concurrently with the applies.
  //
  // defer_q: the policy-norm merges are left to q_merge(n) (one launch after PPO for the round's
  // n staged updates); the stages then leave the policy norm untouched and can run concurrently
  // with the PPO update that reads it.
  void stage(int slot, torch::Tensor e_idx, torch::Tensor g_idx, bool merge_b, bool merge_p, bool merge_q,
             bool defer_q) {
    TORCH_CHECK(slot >= 0 && slot < n_slots_, "stage: slot ", slot, " outside the reserved ", n_slots_);
    for (int k = 0; k < n_mb_; ++k) {
      ia::AirlDiscArgs a = slot_args(slot, k);
      check_idx(e_idx);
      check_idx(g_idx);
      a.e_idx = e_idx.data_ptr<int64_t>();
      a.g_idx = g_idx.data_ptr<int64_t>();
      IA_HIP_CHECK_A(ia::airl_gather(a, k, ia_stream()));
      a.merge_b = merge_b;
      a.merge_p = merge_p;
      a.merge_q = merge_q;
      if (!(defer_q && merge_q && a.q_mean)) a.q_defer = nullptr;
      IA_HIP_CHECK_A(ia::airl_norm(a, 0, 0, ia_stream()));
    }
  }
  // the deferred policy-norm merges of staged updates [0, n), in update order; rows: rows per
  // minibatch merge (0: 2 mb; data parallel with synced norms: 2 mb x world)
  void q_merge(int n, int rows) {
    TORCH_CHECK(n >= 0 && n <= n_slots_, "q_merge: ", n, " updates, ", n_slots_, " staged");
    TORCH_CHECK(a_.q_mean != nullptr && a_.q_count != nullptr, "q_merge: no policy norm");
    if (n == 0) return;
    ia::AirlDiscArgs a = slot_args(0, 0);
    IA_HIP_CHECK_A(ia::airl_q_merge(a, n * n_mb_, (long long)slot_floats(), rows > 0 ? rows : 2 * mb_, ia_stream()));
  }
  // Split update under data parallelism: the staging of update `slot`, minibatch k, in the two
  // halves around the normaliser all-reduce -- mode 1: gather + local moments into `sums` (the
  // caller all-reduces them), mode 2: the merges from the all-reduced sums (n_total rows) into
  // the slot's normaliser rows. apply_grads(slot) runs the slot's fwd/bwd passes and the gradient
  // / stats reduction only (the caller all-reduces `grads`, then adam(0, 1, ...)). Same launches,
  // same data as the non-split DP update (bitwise).
  void stage_part(int slot, int k, torch::Tensor e_idx, torch::Tensor g_idx, int mode, int n_total, bool merge_b,
                  bool merge_p, bool merge_q, bool defer_q) {
    TORCH_CHECK(slot >= 0 && slot < n_slots_, "stage_part: slot ", slot, " outside the reserved ", n_slots_);
    TORCH_CHECK(k >= 0 && k < n_mb_, "stage_part: minibatch ", k);
    TORCH_CHECK(mode == 1 || mode == 2, "stage_part: mode 1 (gather + moments) or 2 (merges)");
    TORCH_CHECK(a_.sums != nullptr, "stage_part needs the sums buffer");
    ia::AirlDiscArgs a = slot_args(slot, k);
    a.merge_b = merge_b;
    a.merge_p = merge_p;
    a.merge_q = merge_q;
    if (!(defer_q && merge_q && a.q_mean) || mode == 1) a.q_defer = nullptr;
    if (mode == 1) {
      check_idx(e_idx);
      check_idx(g_idx);
      a.e_idx = e_idx.data_ptr<int64_t>();
      a.g_idx = g_idx.data_ptr<int64_t>();
      IA_HIP_CHECK_A(ia::airl_gather(a, k, ia_stream()));
      IA_HIP_CHECK_A(ia::airl_norm(a, 1, 0, ia_stream()));
    } else {
      IA_HIP_CHECK_A(ia::airl_norm(a, 2, n_total, ia_stream()));
    }
  }
  void apply_grads(int slot, c10::optional<torch::Tensor> stats_out) {
    TORCH_CHECK(slot >= 0 && slot < n_slots_, "apply_grads: slot ", slot, " was not staged");
    for (int k = 0; k < n_mb_; ++k) IA_HIP_CHECK_A(ia::airl_fwd_bwd(slot_args(slot, k), plan_, k, ia_stream()));
    adam(1, 0, 0.0, 1.0, stats_out);
  }
  // stage / apply workspaces for n updates per round (grow only when no apply is pending)
  void reserve(int n) {
    if (n <= n_slots_) return;
    auto opts = torch::TensorOptions().dtype(torch::kFloat32).device(held_.front().device());
    slots_ = torch::zeros({(int64_t)n * n_mb_ * slot_floats()}, opts);
    n_slots_ = n;
  }
  void apply(int slot, double step_size, double bc2_sqrt, c10::optional<torch::Tensor> stats_out) {
    TORCH_CHECK(slot >= 0 && slot < n_slots_, "apply: slot ", slot, " was not staged");
    for (int k = 0; k < n_mb_; ++k) IA_HIP_CHECK_A(ia::airl_fwd_bwd(slot_args(slot, k), plan_, k, ia_stream()));
    adam(1, 1, step_size, bc2_sqrt, stats_out);
  }

  // whole single-rank update: 3 launches per minibatch + Adam
  void update(torch::Tensor e_idx, torch::Tensor g_idx, double step_size, double bc2_sqrt, bool merge_b, bool merge_p,
              bool merge_q, c10::optional<torch::Tensor> stats_out) {
    for (int k = 0; k < n_mb_; ++k) {
      gather(k, e_idx, g_idx);
      norm(0, 0, merge_b, merge_p, merge_q);
      fwd_bwd(k);
    }
    adam(1, 1, step_size, bc2_sqrt, stats_out);
  }

 private:
  void check_idx(const torch::Tensor& t) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kInt64 && t.numel() >= B_,
                "indices must be int64 GPU tensors of >= batch entries");
  }
  // per-(slot, minibatch) copies of the gathered rows (Xb, S, S2, Act, Done) and of the
  // normaliser rows (nrm) for stage / apply; grown on demand
  int64_t slot_floats() const {
    const int64_t n = 2 * mb_;
    const int64_t f = n * (a_.din_b + 2 * a_.D + a_.aw_pi + 1) + 5 * 256;  // nrm rows + q_defer
    return (f + 63) & ~int64_t(63);
  }

  ia::AirlDiscArgs slot_args(int slot, int k) const {
    ia::AirlDiscArgs a = a_;
    const int64_t n = 2 * mb_;
    float* base = slots_.data_ptr<float>() + ((int64_t)slot * n_mb_ + k) * slot_floats();
    a.Xb = base;
    a.S = a.Xb + n * a_.din_b;
    a.S2 = a.S + n * a_.D;
    a.Act = a.S2 + n * a_.D;
    a.Done = a.Act + n * a_.aw_pi;
    a.nrm = a.Done + n;
    a.q_defer = a.nrm + 4 * 256;
    return a;
  }
  std::vector<torch::Tensor> held_;
  torch::Tensor slots_;
  int n_slots_ = 0;
  torch::Tensor prof_;
  ia::AirlDiscArgs a_{};
  ia::AirlPlan plan_{};
  ia::DiscAdamArgs ad_{};
  int B_ = 0, mb_ = 0, n_mb_ = 0, fb_blocks_ = 0;
};

// Workspace sizes: (gather blocks, fwd/bwd blocks per minibatch).
py::tuple airl_plan_sizes(int minibatch) {
  return py::make_tuple(ia::airl_gather_blocks(minibatch), ia::airl_fwd_blocks(minibatch));
}

}  // namespace

void register_airl(py::module& m) {
  py::class_<AirlDiscPlan>(m, "AirlDiscPlan")
      .def(py::init<py::dict>())
      .def_property_readonly("n_params", &AirlDiscPlan::n_params)
      .def_property_readonly("n_minibatches", &AirlDiscPlan::n_minibatches)
      .def_property_readonly("lds_bytes", &AirlDiscPlan::lds_bytes)
      .def("set_prof", &AirlDiscPlan::set_prof)
      .def("gather", &AirlDiscPlan::gather)
      .def("norm", &AirlDiscPlan::norm, py::arg("mode"), py::arg("n_total"), py::arg("merge_b"), py::arg("merge_p"),
           py::arg("merge_q"))
      .def("fwd_bwd", &AirlDiscPlan::fwd_bwd)
      .def("adam", &AirlDiscPlan::adam, py::arg("reduce"), py::arg("do_adam"), py::arg("step_size"), py::arg("bc2_sqrt"),
           py::arg("stats_out") = py::none())
      .def("reserve", &AirlDiscPlan::reserve)
      .def("stage_part", &AirlDiscPlan::stage_part, py::arg("slot"), py::arg("k"), py::arg("e_idx"), py::arg("g_idx"),
           py::arg("mode"), py::arg("n_total"), py::arg("merge_b"), py::arg("merge_p"), py::arg("merge_q"),
           py::arg("defer_q") = false)
      .def("apply_grads", &AirlDiscPlan::apply_grads, py::arg("slot"), py::arg("stats_out") = py::none())
      .def("stage", &AirlDiscPlan::stage, py::arg("slot"), py::arg("e_idx"), py::arg("g_idx"), py::arg("merge_b"),
           py::arg("merge_p"), py::arg("merge_q"), py::arg("defer_q") = false)
      .def("q_merge", &AirlDiscPlan::q_merge, py::arg("n"), py::arg("rows") = 0)
      .def("apply", &AirlDiscPlan::apply, py::arg("slot"), py::arg("step_size"), py::arg("bc2_sqrt"),
           py::arg("stats_out") = py::none())
      .def("update", &AirlDiscPlan::update, py::arg("e_idx"), py::arg("g_idx"), py::arg("step_size"), py::arg("bc2_sqrt"),
           py::arg("merge_b"), py::arg("merge_p"), py::arg("merge_q"), py::arg("stats_out") = py::none());
  m.def("airl_plan_sizes", &airl_plan_sizes, py::arg("minibatch"));
}

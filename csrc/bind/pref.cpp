// PrefRmPlan: the fused preference reward-model minibatch (csrc/kernels/pref_rm.hip + the
// AdamW of disc.hip). Built once per trainer / dataset store from a dict of persistent
// tensors (device-resident fragment dataset, reward-net weights and RunningNorm buffers, the
// FusedAdam flat parameters, moments and device step counter); a minibatch then passes only
// its pair ids: one pybind call, four launches, no host sync, HIP-graph capturable.
#include "common.h"
#include "launchers.h"

#include <algorithm>

namespace {

#define IA_HIP_CHECK_P(expr)                                                          \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e)); \
  } while (0)

class PrefRmPlan {
 public:
  explicit PrefRmPlan(py::dict d) {
    auto keep = [&](const char* k, bool optional = false) -> torch::Tensor {
      if (!d.contains(k) || d[k].is_none()) {
        TORCH_CHECK(optional, "pref plan arg missing: ", k);
        return torch::Tensor();
      }
      auto t = d[k].cast<torch::Tensor>();
      TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "pref plan arg ", k, " must be a contiguous GPU tensor");
      held_.push_back(t);
      return t;
    };
    auto fptr = [&](const char* k, bool optional = false) -> float* {
      auto t = keep(k, optional);
      if (!t.defined()) return nullptr;
      TORCH_CHECK(t.scalar_type() == torch::kFloat32, k, " must be float32");
      return t.data_ptr<float>();
    };
    a_ = ia::PrefRmArgs{};
    a_.L = d["L"].cast<int>();
    B_ = d["batch"].cast<int>();
    cap_ = d["capacity"].cast<int>();
    TORCH_CHECK(a_.L > 0 && B_ > 0 && cap_ >= B_, "fragment length, batch and capacity");
    a_.ds = d["ds"].cast<int>();
    a_.da = d["da"].cast<int>();
    a_.dns = d["dns"].cast<int>();
    const int use_done = d["use_done"].cast<int>();
    a_.din = a_.ds + a_.da + a_.dns + use_done;
    a_.s_all = fptr("s_all", a_.ds == 0);
    a_.a_all = fptr("a_all", a_.da == 0);
    a_.ns_all = fptr("ns_all", a_.dns == 0);
    a_.d_all = fptr("d_all", use_done == 0);
    a_.prefs_all = fptr("prefs_all");
    a_.gt_all = fptr("gt_all", true);
    // reward MLP: flat parameter order W0, b0, W1, b1, ... (the optimizer's flat buffer)
    py::dict nd = d["net"].cast<py::dict>();
    auto Ws = nd["W"].cast<std::vector<torch::Tensor>>();
    auto bs = nd["b"].cast<std::vector<torch::Tensor>>();
    TORCH_CHECK(!Ws.empty() && Ws.size() <= (size_t)ia::kAirlMaxLayers && Ws.size() == bs.size(), "net: 1..4 layers");
    ia::AirlNet& n = a_.net;
    n.n_layers = (int)Ws.size();
    n.dims[0] = (int)Ws[0].size(1);
    n.hidden_act = nd["hidden_act"].cast<int>();
    n.param_off = 0;
    int o = 0;
    for (size_t l = 0; l < Ws.size(); ++l) {
      TORCH_CHECK(Ws[l].is_cuda() && Ws[l].is_contiguous() && Ws[l].scalar_type() == torch::kFloat32, "net weights");
      TORCH_CHECK(l == 0 || Ws[l].size(1) == Ws[l - 1].size(0), "net: layer widths do not chain");
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
    a_.n_params = o;
    TORCH_CHECK(n.dims[0] == a_.din, "reward-net input width ", n.dims[0], " != gathered width ", a_.din);
    a_.rmean = fptr("rmean", true);
    a_.rvar = fptr("rvar", true);
    if (a_.rmean) {
      auto c = keep("rcount");
      TORCH_CHECK(c.scalar_type() == torch::kInt32, "rcount must be int32");
      a_.rcount = c.data_ptr<int>();
    }
    a_.eps = (float)d["eps"].cast<double>();
    a_.discount = (float)d["discount"].cast<double>();
    a_.threshold = (float)d["threshold"].cast<double>();
    a_.noise = (float)d["noise"].cast<double>();
    a_.gscale = (float)(1.0 / (double)B_);
    TORCH_CHECK(ia::pref_rm_plan(a_, plan_), "reward net outside the fused kernel's limits (widths <= 64, <= 4 layers, "
                                             "scalar head, <= 128 input columns)");
    // workspaces, sized for `capacity` pairs per minibatch
    const auto fo = torch::TensorOptions().dtype(torch::kFloat32).device(held_[0].device());
    const int64_t rows = (int64_t)cap_ * 2 * a_.L;
    const int blocks = ia::pref_rm_blocks(cap_, a_.L);
    ws_.push_back(torch::empty({rows * a_.din}, fo));
    a_.X = ws_.back().data_ptr<float>();
    ws_.push_back(torch::empty({(int64_t)blocks * 2 * a_.din}, fo));
    a_.partials = ws_.back().data_ptr<float>();
    sums_ = torch::zeros({2 * a_.din}, fo.dtype(torch::kFloat64));
    a_.sums = sums_.data_ptr<double>();
    ws_.push_back(torch::zeros({1}, fo.dtype(torch::kInt32)));
    a_.cnt = reinterpret_cast<unsigned*>(ws_.back().data_ptr<int>());
    ws_.push_back(torch::zeros({256}, fo));
    a_.old_mv = ws_.back().data_ptr<float>();
    ws_.push_back(torch::zeros({1}, fo.dtype(torch::kInt32)));
    a_.old_cnt = ws_.back().data_ptr<int>();
    ws_.push_back(torch::zeros({256}, fo));
    a_.nrm = ws_.back().data_ptr<float>();
    ws_.push_back(torch::empty({rows}, fo));
    a_.r = ws_.back().data_ptr<float>();
    ws_.push_back(torch::empty({(int64_t)blocks * a_.n_params}, fo));
    a_.slab = ws_.back().data_ptr<float>();
    ws_.push_back(torch::zeros({(int64_t)cap_ * 8}, fo));
    a_.pstats = ws_.back().data_ptr<float>();
    grads_ = torch::zeros({a_.n_params}, fo);
    metrics_ = torch::zeros({8}, fo);
    // AdamW (disc.hip) on the optimizer's flat buffers, bias corrections from its device step
    ad_ = ia::DiscAdamArgs{};
    ad_.n_params = a_.n_params;
    ad_.params = fptr("params");
    TORCH_CHECK(held_.back().numel() >= a_.n_params, "flat params smaller than the net");
    ad_.exp_avg = fptr("exp_avg");
    ad_.exp_avg_sq = fptr("exp_avg_sq");
    a_.step = fptr("step");
    ad_.step = a_.step;
    ad_.lr = (float)d["lr"].cast<double>();
    ad_.beta1 = (float)d["beta1"].cast<double>();
    ad_.beta2 = (float)d["beta2"].cast<double>();
    ad_.eps = (float)d["adam_eps"].cast<double>();
    ad_.weight_decay = (float)d["weight_decay"].cast<double>();
    ad_.decoupled = d["decoupled"].cast<bool>() ? 1 : 0;
    ad_.grads = grads_.data_ptr<float>();
    ad_.slab = a_.slab;
    ad_.stats_slab = a_.pstats;
  }

  int n_params() const { return a_.n_params; }
  int lds_bytes() const { return plan_.lds_bytes; }
  torch::Tensor sums() const { return sums_; }
  torch::Tensor grads() const { return grads_; }
  torch::Tensor metrics() const { return metrics_; }

  // single rank: gather, forward (+ RunningNorm merge), backward, AdamW -> metrics()
  // ([loss, accuracy, ground-truth loss] minibatch means)
  torch::Tensor step(torch::Tensor idx, bool merge) {
    ia::PrefRmArgs a = args(idx, merge);
    IA_HIP_CHECK_P(ia::pref_rm_gather(a, ia_stream()));
    IA_HIP_CHECK_P(ia::pref_rm_fwd(a, plan_, 0, ia_stream()));
    IA_HIP_CHECK_P(ia::pref_rm_bwd(a, plan_, ia_stream()));
    adam_launch(a, 1, 1);
    return metrics_;
  }
  // data-parallel pieces: gather (+ block sums -> sums()), forward from the all-reduced
  // sums of n_total rows, backward + slab reduction into grads() (all-reduce them), AdamW
  // gather (+ the column sums -> sums(): all-reduce them before forward(n_total > 0))
  void gather(torch::Tensor idx, bool merge) {
    ia::PrefRmArgs a = args(idx, merge);
    IA_HIP_CHECK_P(ia::pref_rm_gather(a, ia_stream()));
  }
  // moments from sums() over n_total rows (0: this rank's rows)
  void forward(torch::Tensor idx, bool merge, int n_total) {
    ia::PrefRmArgs a = args(idx, merge);
    IA_HIP_CHECK_P(ia::pref_rm_fwd(a, plan_, n_total, ia_stream()));
  }
  void backward(torch::Tensor idx, bool merge) {
    ia::PrefRmArgs a = args(idx, merge);
    IA_HIP_CHECK_P(ia::pref_rm_bwd(a, plan_, ia_stream()));
    adam_launch(a, 1, 0);
  }
  void apply(torch::Tensor idx) {
    ia::PrefRmArgs a = args(idx, false);
    adam_launch(a, 0, 1);
  }
  // One epoch (single rank) in one call -- capturable as ONE graph that is replayed per
  // epoch: minibatch mb takes pairs order[*cursor * P + mb * B, ...) (P pairs, batch B; the
  // last minibatch may be partial), its metrics go to ep[mb * 8 ...]; the epoch end copies
  // ep to all[*cursor] and advances the device cursor.
  void epoch(torch::Tensor order, int P, torch::Tensor cursor, torch::Tensor ep, torch::Tensor all, bool merge) {
    TORCH_CHECK(order.is_cuda() && order.is_contiguous() && order.scalar_type() == torch::kInt64, "order: int64 GPU");
    TORCH_CHECK(cursor.is_cuda() && cursor.scalar_type() == torch::kInt32 && cursor.numel() == 1, "cursor: int32 GPU [1]");
    const int n_mb = (P + B_ - 1) / B_;
    TORCH_CHECK(P > 0 && order.numel() >= P, "order holds fewer than P pairs");
    TORCH_CHECK(ep.is_cuda() && ep.scalar_type() == torch::kFloat32 && ep.numel() >= (int64_t)n_mb * 8, "ep: float32 [n_mb * 8]");
    TORCH_CHECK(all.is_cuda() && all.scalar_type() == torch::kFloat32 && all.numel() % ((int64_t)n_mb * 8) == 0,
                "all: float32 [epochs * n_mb * 8]");
    for (int mb = 0; mb < n_mb; ++mb) {
      ia::PrefRmArgs a = a_;
      a.n = std::min(B_, P - mb * B_);
      TORCH_CHECK(a.n <= cap_, "minibatch above capacity");
      a.idx = order.data_ptr<int64_t>() + (int64_t)mb * B_;
      a.cursor = cursor.data_ptr<int>();
      a.idx_stride = P;
      a.merge = merge ? 1 : 0;
      IA_HIP_CHECK_P(ia::pref_rm_gather(a, ia_stream()));
      IA_HIP_CHECK_P(ia::pref_rm_fwd(a, plan_, 0, ia_stream()));
      IA_HIP_CHECK_P(ia::pref_rm_bwd(a, plan_, ia_stream()));
      adam_launch(a, 1, 1, ep.data_ptr<float>() + (int64_t)mb * 8);
    }
    IA_HIP_CHECK_P(ia::pref_rm_epoch_end(ep.data_ptr<float>(), all.data_ptr<float>(), n_mb * 8, cursor.data_ptr<int>(),
                                         ia_stream()));
  }

 private:
  ia::PrefRmArgs args(const torch::Tensor& idx, bool merge) {
    TORCH_CHECK(idx.is_cuda() && idx.is_contiguous() && idx.scalar_type() == torch::kInt64 && idx.dim() == 1,
                "idx: int64 GPU vector");
    TORCH_CHECK(idx.numel() > 0 && idx.numel() <= cap_, "minibatch of ", idx.numel(), " pairs (capacity ", cap_, ")");
    ia::PrefRmArgs a = a_;
    a.n = (int)idx.numel();
    a.idx = idx.data_ptr<int64_t>();
    a.merge = merge ? 1 : 0;
    return a;
  }
  void adam_launch(const ia::PrefRmArgs& a, int reduce, int do_adam, float* stats_out = nullptr) {
    ia::DiscAdamArgs d = ad_;
    d.reduce = reduce;
    d.adam = do_adam;
    d.nblk = ia::pref_rm_blocks(a.n, a.L);
    d.stats_nblk = a.n;
    d.stats_scale = 1.f / (float)a.n;
    d.stats_out = reduce ? (stats_out ? stats_out : metrics_.data_ptr<float>()) : nullptr;
    IA_HIP_CHECK_P(ia::disc_adam(d, ia_stream()));
  }
  std::vector<torch::Tensor> held_, ws_;
  torch::Tensor sums_, grads_, metrics_;
  ia::PrefRmArgs a_{};
  ia::PrefPlan plan_{};
  ia::DiscAdamArgs ad_{};
  int B_ = 0, cap_ = 0;
};

}  // namespace

void register_pref(py::module& m) {
  py::class_<PrefRmPlan>(m, "PrefRmPlan")
      .def(py::init<py::dict>())
      .def_property_readonly("n_params", &PrefRmPlan::n_params)
      .def_property_readonly("lds_bytes", &PrefRmPlan::lds_bytes)
      .def_property_readonly("sums", &PrefRmPlan::sums)
      .def_property_readonly("grads", &PrefRmPlan::grads)
      .def_property_readonly("metrics", &PrefRmPlan::metrics)
      .def("step", &PrefRmPlan::step, py::arg("idx"), py::arg("merge"))
      .def("gather", &PrefRmPlan::gather, py::arg("idx"), py::arg("merge"))
      .def("forward", &PrefRmPlan::forward, py::arg("idx"), py::arg("merge"), py::arg("n_total"))
      .def("backward", &PrefRmPlan::backward, py::arg("idx"), py::arg("merge"))
      .def("apply", &PrefRmPlan::apply, py::arg("idx"))
      .def("epoch", &PrefRmPlan::epoch, py::arg("order"), py::arg("P"), py::arg("cursor"), py::arg("ep"), py::arg("all"),
           py::arg("merge"));
}

// Torch-facing bindings of the device engine kernels (rollout, PPO update).
// Arguments arrive as a Python dict of tensors / numbers, so the engine's Python
// side (imitation_amd/engine/*.py) owns the layout and this file only validates
// devices/dtypes and forwards raw pointers.
#include "common.h"
#include "launchers.h"
#include "vec_env.h"

namespace {

#define IA_HIP_CHECK2(expr)                                                           \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    TORCH_CHECK(_e == hipSuccess, "HIP error in " #expr ": ", hipGetErrorString(_e)); \
  } while (0)

template <typename T>
T* tptr(const py::dict& d, const char* k, bool optional = false) {
  if (!d.contains(k) || d[k].is_none()) {
    TORCH_CHECK(optional, "engine arg missing: ", k);
    return nullptr;
  }
  auto t = d[k].cast<torch::Tensor>();
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "engine arg ", k, " must be a contiguous GPU tensor");
  return reinterpret_cast<T*>(t.data_ptr());
}

int ival(const py::dict& d, const char* k, int def = 0) { return d.contains(k) ? d[k].cast<int>() : def; }
double fval(const py::dict& d, const char* k, double def = 0.0) { return d.contains(k) ? d[k].cast<double>() : def; }

ia::WaveMLP wave_mlp(const py::dict& d) {
  ia::WaveMLP m{};
  auto Ws = d["W"].cast<std::vector<torch::Tensor>>();
  auto bs = d["b"].cast<std::vector<torch::Tensor>>();
  TORCH_CHECK(!Ws.empty() && Ws.size() <= (size_t)ia::kWaveMaxLayers, "1..4 layers");
  m.n_layers = (int)Ws.size();
  m.dims[0] = (int)Ws[0].size(1);
  for (size_t l = 0; l < Ws.size(); ++l) {
    TORCH_CHECK(Ws[l].is_cuda() && Ws[l].is_contiguous() && Ws[l].scalar_type() == torch::kFloat32, "W");
    m.dims[l + 1] = (int)Ws[l].size(0);
    TORCH_CHECK(m.dims[l + 1] <= ia::kWaveMaxDim && m.dims[l] <= ia::kWaveMaxDim, "engine MLP width <= 64");
    m.W[l] = Ws[l].data_ptr<float>();
    m.b[l] = bs[l].data_ptr<float>();
  }
  m.hidden_act = d["hidden_act"].cast<int>();
  m.out_act = d["out_act"].cast<int>();
  m.norm_mean = tptr<const float>(d, "norm_mean", true);
  m.norm_var = tptr<const float>(d, "norm_var", true);
  m.norm_eps = (float)fval(d, "norm_eps", 1e-5);
  return m;
}

void rollout(py::dict d) {
  ia::RolloutArgs a{};
  std::string env = d["env"].cast<std::string>();
  int ms = 0;
  TORCH_CHECK(ia::make_env_params(env, &a.P, &ms), "unknown native env ", env);
  TORCH_CHECK(a.P.kind != ia::ENV_PONG, "image envs are not supported by the device rollout");
  a.max_steps = ival(d, "max_steps", ms);
  a.T = ival(d, "T");
  a.N = ival(d, "N");
  a.seed = (uint64_t)d["seed"].cast<long long>();
  a.step0 = d["step0"].cast<long long>();
  a.state = tptr<float>(d, "state");
  a.rng = tptr<uint64_t>(d, "rng");
  a.elapsed = tptr<int>(d, "elapsed");
  a.ep_ret = tptr<float>(d, "ep_ret");
  a.cur_obs = tptr<float>(d, "cur_obs");
  a.cur_start = tptr<float>(d, "cur_start");
  a.pi = wave_mlp(d["pi"].cast<py::dict>());
  a.log_std = tptr<const float>(d, "log_std", true);
  a.act_low = tptr<const float>(d, "act_low", true);
  a.act_high = tptr<const float>(d, "act_high", true);
  a.n_actions = ival(d, "n_actions", 0);
  TORCH_CHECK(a.n_actions > 0 || (a.act_low && a.act_high && a.log_std), "Gaussian policy needs log_std and Box bounds");
  TORCH_CHECK(a.n_actions <= 64, "Categorical over more than 64 actions");
  TORCH_CHECK(a.pi.dims[0] == a.P.obs_dim, "actor input dim != obs dim");
  TORCH_CHECK(a.pi.dims[a.pi.n_layers] == (a.n_actions > 0 ? a.n_actions : a.P.act_dim), "actor head width");
  a.explore_mode = tptr<const int>(d, "explore_mode", true);
  a.deterministic = ival(d, "deterministic", 0);
  TORCH_CHECK(a.P.obs_dim <= ia::kEngineMaxObs, "obs dim too large for the device rollout");
  a.obs_buf = tptr<float>(d, "obs_buf");
  a.act_raw = tptr<float>(d, "act_raw");
  a.act_env = tptr<float>(d, "act_env");
  a.env_rew = tptr<float>(d, "env_rew");
  a.starts = tptr<float>(d, "starts");
  a.dones = tptr<float>(d, "dones");
  a.trunc = tptr<float>(d, "trunc");
  a.next_obs = tptr<float>(d, "next_obs");
  a.ep_ret_out = tptr<float>(d, "ep_ret_out");
  if (d.contains("prof") && !d["prof"].is_none()) {
    auto t = d["prof"].cast<torch::Tensor>();
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == torch::kInt64 && t.numel() == (int64_t)a.N * 5,
                "prof must be a contiguous int64 GPU tensor of N x 5");
    a.prof = reinterpret_cast<long long*>(t.data_ptr());
  }
  a.lds_actor = ival(d, "lds_actor", 0);
  IA_HIP_CHECK2(ia::rollout_launch(a, ia_stream()));
}

void rollout_post(py::dict d) {
  ia::RolloutPostArgs a{};
  a.T = ival(d, "T");
  a.N = ival(d, "N");
  a.D = ival(d, "D");
  a.A = ival(d, "A");
  a.n_actions = ival(d, "n_actions", 0);
  a.gamma = (float)fval(d, "gamma", 0.99);
  a.obs = tptr<const float>(d, "obs_buf");
  a.act_raw = tptr<const float>(d, "act_raw");
  a.act_env = tptr<const float>(d, "act_env");
  a.next_obs = tptr<const float>(d, "next_obs");
  a.dones = tptr<const float>(d, "dones");
  a.trunc = tptr<const float>(d, "trunc");
  a.env_rew = tptr<const float>(d, "env_rew");
  a.cur_obs = tptr<const float>(d, "cur_obs");
  a.vf = wave_mlp(d["vf"].cast<py::dict>());
  TORCH_CHECK(a.vf.dims[0] == a.D && a.vf.dims[a.vf.n_layers] == 1, "critic shape");
  a.logp = tptr<float>(d, "logp", true);
  if (a.logp) {
    a.pi = wave_mlp(d["pi"].cast<py::dict>());
    TORCH_CHECK(a.pi.dims[0] == a.D, "actor input dim");
    a.log_std = tptr<const float>(d, "log_std", true);
    TORCH_CHECK(a.n_actions > 0 || a.log_std, "Gaussian log-prob needs log_std");
  }
  a.rew_enabled = ival(d, "rew_enabled", 0);
  if (a.rew_enabled) {
    a.rew = wave_mlp(d["rew"].cast<py::dict>());
    a.use_state = ival(d, "use_state", 1);
    a.use_action = ival(d, "use_action", 1);
    a.use_next_state = ival(d, "use_next_state", 0);
    a.use_done = ival(d, "use_done", 0);
    a.rew_transform = ival(d, "rew_transform", 0);
    a.shaped = ival(d, "shaped", 0);
    if (a.shaped) {
      a.pot = wave_mlp(d["pot"].cast<py::dict>());
      a.shaping_gamma = (float)fval(d, "shaping_gamma", 0.99);
      TORCH_CHECK(a.pot.dims[0] == a.D, "potential input dim");
    }
    const int din = (a.use_state ? a.D : 0) + (a.use_action ? (a.n_actions > 0 ? a.n_actions : a.A) : 0) +
                    (a.use_next_state ? a.D : 0) + (a.use_done ? 1 : 0);
    TORCH_CHECK(a.rew.dims[0] == din, "reward MLP input dim ", a.rew.dims[0], " != ", din);
    TORCH_CHECK(din <= ia::kWaveMaxDim, "reward input wider than a wave");
  }
  a.values = tptr<float>(d, "values");
  a.boot = tptr<float>(d, "boot");
  a.rewards = tptr<float>(d, "rewards");
  a.rew_raw = tptr<float>(d, "rew_raw", true);
  a.last_values = tptr<float>(d, "last_values");
  IA_HIP_CHECK2(ia::rollout_post_launch(a, ia_stream()));
}

void reward_outnorm(py::dict d) {
  ia::OutNormArgs a{};
  a.T = ival(d, "T");
  a.N = ival(d, "N");
  a.rew_raw = tptr<const float>(d, "rew_raw");
  a.boot = tptr<const float>(d, "boot");
  a.rewards = tptr<float>(d, "rewards");
  a.mean = tptr<float>(d, "mean");
  a.var = tptr<float>(d, "var");
  a.count_i = tptr<int>(d, "count_i", true);
  if (a.count_i) TORCH_CHECK(py::cast<torch::Tensor>(d["count_i"]).scalar_type() == torch::kInt32, "count_i: int32");
  a.count = tptr<float>(d, "count", a.count_i != nullptr);
  a.eps = (float)fval(d, "eps", 1e-5);
  a.step_stats = tptr<const float>(d, "step_stats", true);
  IA_HIP_CHECK2(ia::reward_outnorm_launch(a, ia_stream()));
}

void ppo_update(py::dict d) {
  ia::PPOArgs a{};
  a.D = ival(d, "D");
  a.A = ival(d, "A");
  a.discrete = ival(d, "discrete");
  auto pid = d["pi_dims"].cast<std::vector<int>>();
  auto vid = d["vf_dims"].cast<std::vector<int>>();
  TORCH_CHECK(pid.size() >= 2 && pid.size() <= (size_t)ia::kWaveMaxLayers + 1, "pi dims");
  TORCH_CHECK(vid.size() >= 2 && vid.size() <= (size_t)ia::kWaveMaxLayers + 1, "vf dims");
  a.n_pi = (int)pid.size() - 1;
  a.n_vf = (int)vid.size() - 1;
  for (size_t i = 0; i < pid.size(); ++i) a.pi_dims[i] = pid[i];
  for (size_t i = 0; i < vid.size(); ++i) a.vf_dims[i] = vid[i];
  auto pw = d["pi_w_off"].cast<std::vector<int>>();
  auto pb = d["pi_b_off"].cast<std::vector<int>>();
  auto vw = d["vf_w_off"].cast<std::vector<int>>();
  auto vb = d["vf_b_off"].cast<std::vector<int>>();
  for (int l = 0; l < a.n_pi; ++l) { a.pi_w_off[l] = pw[l]; a.pi_b_off[l] = pb[l]; }
  for (int l = 0; l < a.n_vf; ++l) { a.vf_w_off[l] = vw[l]; a.vf_b_off[l] = vb[l]; }
  a.log_std_off = ival(d, "log_std_off", -1);
  a.hidden_act = ival(d, "hidden_act");
  a.params = tptr<float>(d, "params");
  a.grads = tptr<float>(d, "grads");
  a.exp_avg = tptr<float>(d, "exp_avg");
  a.exp_avg_sq = tptr<float>(d, "exp_avg_sq");
  a.n_params = ival(d, "n_params");
  a.has_norm = ival(d, "has_norm");
  a.norm_mean = tptr<float>(d, "norm_mean", true);
  a.norm_var = tptr<float>(d, "norm_var", true);
  a.norm_count = tptr<float>(d, "norm_count", true);
  a.norm_count_i = tptr<int>(d, "norm_count_i", true);
  if (a.norm_count_i)
    TORCH_CHECK(py::cast<torch::Tensor>(d["norm_count_i"]).scalar_type() == torch::kInt32, "norm_count_i: int32");
  a.norm_eps = (float)fval(d, "norm_eps", 1e-5);
  a.obs = tptr<const float>(d, "obs");
  a.acts = tptr<const float>(d, "acts");
  a.old_logp = tptr<const float>(d, "old_logp");
  a.adv = tptr<const float>(d, "adv");
  a.returns = tptr<const float>(d, "returns");
  a.perm = tptr<const int>(d, "perm");
  a.rows = ival(d, "rows");
  a.batch = ival(d, "batch");
  a.n_epochs = ival(d, "n_epochs");
  a.clip_range = (float)fval(d, "clip_range");
  a.ent_coef = (float)fval(d, "ent_coef");
  a.vf_coef = (float)fval(d, "vf_coef");
  a.max_grad_norm = (float)fval(d, "max_grad_norm");
  a.lr = (float)fval(d, "lr");
  a.beta1 = (float)fval(d, "beta1", 0.9);
  a.beta2 = (float)fval(d, "beta2", 0.999);
  a.adam_eps = (float)fval(d, "adam_eps", 1e-5);
  a.normalize_advantage = ival(d, "normalize_advantage", 1);
  a.adam_step = tptr<float>(d, "adam_step");
  a.stats = tptr<float>(d, "stats");
  a.zero_stats = ival(d, "zero_stats", 0);
  a.mode = ival(d, "mode", 0);
  a.mb_index = ival(d, "mb_index", 0);
  a.prof = tptr<unsigned long long>(d, "prof", true);
  if (a.prof) TORCH_CHECK(py::cast<torch::Tensor>(d["prof"]).numel() >= 20, "prof: 20 int64 cycle counters (ppo_rc_kernel.h)");
  a.rc_gmax = ival(d, "rc_gmax", 0);
  a.rc_cw = ival(d, "rc_cw", 0);
  a.err = reinterpret_cast<unsigned*>(tptr<int>(d, "err", true));
  a.spin_limit = (unsigned)ival(d, "spin_limit", 0);
  a.debug_stall = ival(d, "debug_stall", 0);
  a.rc_cus = ival(d, "rc_cus", 0);
  TORCH_CHECK(a.D <= 64, "obs dim <= 64");
  ia::PPORcGeo geo;
  size_t rc_lds = 0;
  if (a.mode == 0 && ival(d, "allow_rc", 1) && ia::ppo_rc_plan(a, geo, rc_lds)) {
    auto ws = torch::empty({(int64_t)ia::ppo_rc_workspace_floats(a)},
                           torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, c10::hip::current_device()));
    IA_HIP_CHECK2(ia::ppo_rc_launch(a, ws.data_ptr<float>(), ia_stream()));
    return;
  }
  IA_HIP_CHECK2(ia::ppo_launch(a, ia_stream()));
}

// Which kernel engine_ppo_update(mode 0) runs for this configuration: "rc" or "lds".
std::string ppo_path(py::dict d) {
  ia::PPOArgs a{};
  a.D = ival(d, "D");
  a.A = ival(d, "A");
  a.discrete = ival(d, "discrete");
  auto pid = d["pi_dims"].cast<std::vector<int>>();
  auto vid = d["vf_dims"].cast<std::vector<int>>();
  a.n_pi = (int)pid.size() - 1;
  a.n_vf = (int)vid.size() - 1;
  for (size_t i = 0; i < pid.size(); ++i) a.pi_dims[i] = pid[i];
  for (size_t i = 0; i < vid.size(); ++i) a.vf_dims[i] = vid[i];
  a.batch = ival(d, "batch");
  a.rows = ival(d, "rows");
  a.log_std_off = ival(d, "log_std_off", -1);
  a.rc_gmax = ival(d, "rc_gmax", 0);
  a.rc_cw = ival(d, "rc_cw", 0);
  a.rc_cus = ival(d, "rc_cus", 0);
  a.hidden_act = ival(d, "hidden_act", 0);  // selects the shape-specialised instance family
  ia::PPORcGeo geo;
  size_t lds = 0;
  if (ival(d, "allow_rc", 1) && ia::ppo_rc_plan(a, geo, lds))
    return "rc:g" + std::to_string(geo.G) + "x" + std::to_string(geo.nch) + "x" + std::to_string(geo.cw) + ":kt" +
           std::to_string(geo.kt) + (geo.ns ? ":ns" : "");
  return "lds";
}

size_t ppo_lds(py::dict d) {
  ia::PPOArgs a{};
  a.D = ival(d, "D");
  a.A = ival(d, "A");
  a.discrete = ival(d, "discrete");
  auto pid = d["pi_dims"].cast<std::vector<int>>();
  auto vid = d["vf_dims"].cast<std::vector<int>>();
  a.n_pi = (int)pid.size() - 1;
  a.n_vf = (int)vid.size() - 1;
  for (size_t i = 0; i < pid.size(); ++i) a.pi_dims[i] = pid[i];
  for (size_t i = 0; i < vid.size(); ++i) a.vf_dims[i] = vid[i];
  a.batch = ival(d, "batch");
  return ia::ppo_lds_bytes(a);
}

}  // namespace

// One DAgger-collector env step (mode 0) or reset of every env (mode 1); see dagger.hip.
void dagger_env_step(py::dict d) {
  ia::DaggerEnvArgs a{};
  std::string env = d["env"].cast<std::string>();
  int ms = 0;
  TORCH_CHECK(ia::make_env_params(env, &a.P, &ms), "unknown native env ", env);
  a.N = ival(d, "N");
  a.max_steps = ival(d, "max_steps", ms);
  a.mode = ival(d, "mode", 0);
  a.sdim = ia::state_size(a.P);
  a.state = tptr<float>(d, "state");
  a.rng = tptr<uint64_t>(d, "rng");
  a.elapsed = tptr<int>(d, "elapsed");
  a.ep_ret = tptr<float>(d, "ep_ret");
  auto check_numel = [&](const char* k, int64_t want) {
    if (!d.contains(k) || d[k].is_none()) return;
    auto t = d[k].cast<torch::Tensor>();
    TORCH_CHECK(t.numel() == want, "dagger_env_step: ", k, " has ", t.numel(), " elements, expected ", want);
  };
  check_numel("state", (int64_t)a.N * a.sdim);
  check_numel("rng", a.N);
  check_numel("elapsed", a.N);
  const bool img = a.P.kind == ia::ENV_PONG;
  const int64_t obs_elems = img ? (int64_t)ia::kPongH * ia::kPongW * ia::kPongStack : a.P.obs_dim;
  if (img) {
    a.obs_u8 = tptr<uint8_t>(d, "obs");
    check_numel("obs", a.N * obs_elems);
  } else {
    a.obs_f = tptr<float>(d, "obs");
    check_numel("obs", a.N * obs_elems);
  }
  if (a.mode == 0) {
    if (a.P.n_actions > 0) {
      a.act_i = tptr<const int64_t>(d, "actions");
      check_numel("actions", a.N);
    } else {
      a.act_f = tptr<const float>(d, "actions");
      check_numel("actions", (int64_t)a.N * a.P.act_dim);
    }
    a.rew = tptr<float>(d, "rew");
    a.term = tptr<uint8_t>(d, "term");
    a.trunc = tptr<uint8_t>(d, "trunc");
    if (img) a.term_obs_u8 = tptr<uint8_t>(d, "term_obs");
    else a.term_obs_f = tptr<float>(d, "term_obs");
    check_numel("term_obs", a.N * obs_elems);
    a.ep_ret_out = tptr<float>(d, "ep_ret_out");
    a.ep_len_out = tptr<int>(d, "ep_len_out");
    for (const char* k : {"rew", "term", "trunc", "ep_ret_out", "ep_len_out"}) check_numel(k, a.N);
    if (d.contains("obs_rec") && !d["obs_rec"].is_none()) {
      a.obs_rec = img ? (void*)tptr<uint8_t>(d, "obs_rec") : (void*)tptr<float>(d, "obs_rec");
      check_numel("obs_rec", a.N * obs_elems);
    }
  }
  IA_HIP_CHECK2(ia::dagger_env_step(a, ia_stream()));
}

void register_engine(py::module& m) {
  m.def("dagger_env_step", &dagger_env_step, "DAgger collector: one device env step (mode 0) / reset all (mode 1)");
  m.def("engine_rollout", &rollout, "T-step device rollout (actor sampling + env) for N envs");
  m.def("engine_rollout_post", &rollout_post,
        "values, log-probs, TimeLimit bootstrap and learned reward of a rollout, all transitions in parallel");
  m.def("engine_reward_outnorm", &reward_outnorm, "NormalizedRewardNet output normalisation over a rollout");
  m.def("engine_ppo_update", &ppo_update, "persistent PPO update / DP minibatch grads / apply");
  m.def("engine_ppo_path", &ppo_path, "kernel used by engine_ppo_update mode 0 (rc | lds)");
  m.def("engine_ppo_lds", &ppo_lds, "LDS bytes the PPO kernel needs for a configuration");
}

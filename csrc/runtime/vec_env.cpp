#include "vec_env.h"

#include <string.h>

#include <stdexcept>

namespace ia {

namespace {

LocoParams loco_base(int nq_root, int nv_root, int nj, int obs_skip) {
  LocoParams p{};
  p.nq_root = nq_root;
  p.nv_root = nv_root;
  p.nj = nj;
  p.obs_skip = obs_skip;
  p.frame_skip = 5;
  p.dt = 0.01f;
  p.ctrl_cost = 0.1f;
  p.fwd_weight = 1.0f;
  p.healthy_reward = 0.0f;
  p.drag = 0.4f;
  for (int j = 0; j < kMaxJoints; ++j) {
    // heterogeneous joints so that a gait has to be discovered, not copied
    p.gear[j] = 40.0f + 10.0f * (float)((j * 5) % 3);
    p.stiff[j] = 8.0f + 2.0f * (float)(j % 2);
    p.damp[j] = 2.0f;
    p.thrust[j] = 1.2f + 0.3f * (float)((j * 7) % 4);
    p.pitch_coupling[j] = (j % 2 == 0 ? 1.0f : -1.0f) * 0.8f;
  }
  return p;
}

}  // namespace

bool make_env_params(const std::string& name, EnvParams* P, int* max_steps) {
  EnvParams p{};
  int ms = -1;
  if (name == "CartPole-v0" || name == "CartPole-v1") {
    p.kind = ENV_CARTPOLE; p.obs_dim = 4; p.act_dim = 1; p.n_actions = 2; p.terminates = 1;
    ms = name == "CartPole-v0" ? 200 : 500;
  } else if (name == "seals/CartPole-v0") {
    p.kind = ENV_SEALS_CARTPOLE; p.obs_dim = 4; p.act_dim = 1; p.n_actions = 2; p.terminates = 0; ms = 500;
  } else if (name == "Pendulum-v1") {
    p.kind = ENV_PENDULUM; p.obs_dim = 3; p.act_dim = 1; p.n_actions = 0; p.terminates = 0; ms = 200;
  } else if (name == "MountainCar-v0" || name == "seals/MountainCar-v0") {
    p.kind = ENV_MOUNTAINCAR; p.obs_dim = 2; p.act_dim = 1; p.n_actions = 3;
    p.terminates = name == "MountainCar-v0" ? 1 : 0; ms = 200;
  } else if (name == "Acrobot-v1") {
    p.kind = ENV_ACROBOT; p.obs_dim = 6; p.act_dim = 1; p.n_actions = 3; p.terminates = 1; ms = 500;
  } else if (name == "seals/HalfCheetah-v1" || name == "HalfCheetah-v4" || name == "seals/HalfCheetah-v0") {
    p.kind = ENV_LOCO; p.loco = loco_base(3, 3, 6, 1); p.obs_dim = 17; p.act_dim = 6; ms = 1000;
  } else if (name == "seals/Hopper-v1" || name == "Hopper-v4" || name == "seals/Hopper-v0") {
    p.kind = ENV_LOCO; p.loco = loco_base(3, 3, 3, 1); p.loco.frame_skip = 4; p.loco.ctrl_cost = 1e-3f;
    p.loco.healthy_reward = 1.0f; p.obs_dim = 11; p.act_dim = 3; ms = 1000;
  } else if (name == "seals/Walker2d-v1" || name == "Walker2d-v4" || name == "seals/Walker2d-v0") {
    p.kind = ENV_LOCO; p.loco = loco_base(3, 3, 6, 1); p.loco.frame_skip = 4; p.loco.ctrl_cost = 1e-3f;
    p.loco.healthy_reward = 1.0f; p.obs_dim = 17; p.act_dim = 6; ms = 1000;
  } else if (name == "seals/Swimmer-v1" || name == "Swimmer-v4" || name == "seals/Swimmer-v0") {
    p.kind = ENV_LOCO; p.loco = loco_base(3, 3, 2, 2); p.loco.frame_skip = 4; p.loco.ctrl_cost = 1e-4f;
    p.obs_dim = 8; p.act_dim = 2; ms = 1000;
  } else if (name == "seals/Ant-v1" || name == "Ant-v4" || name == "seals/Ant-v0") {
    p.kind = ENV_LOCO; p.loco = loco_base(7, 6, 8, 2); p.loco.ctrl_cost = 0.5f; p.loco.healthy_reward = 1.0f;
    p.obs_dim = 27; p.act_dim = 8; ms = 1000;
  } else if (name == "PongNoFrameskip-v4" || name == "ALE/Pong-v5" || name == "Pong-synthetic-v0") {
    p.kind = ENV_PONG; p.obs_dim = kPongH * kPongW * kPongStack; p.act_dim = 1; p.n_actions = 6;
    p.terminates = 1; ms = 27000;
  } else {
    return false;
  }
  if (P) *P = p;
  if (max_steps) *max_steps = ms;
  return true;
}

std::vector<std::string> native_env_names() {
  return {"CartPole-v0", "CartPole-v1", "seals/CartPole-v0", "Pendulum-v1", "MountainCar-v0",
          "seals/MountainCar-v0", "Acrobot-v1", "seals/HalfCheetah-v1", "HalfCheetah-v4", "seals/HalfCheetah-v0",
          "seals/Hopper-v1", "Hopper-v4", "seals/Hopper-v0", "seals/Walker2d-v1", "Walker2d-v4",
          "seals/Walker2d-v0", "seals/Swimmer-v1", "Swimmer-v4", "seals/Swimmer-v0", "seals/Ant-v1", "Ant-v4",
          "seals/Ant-v0", "PongNoFrameskip-v4", "ALE/Pong-v5", "Pong-synthetic-v0"};
}

BatchedEnv::BatchedEnv(const std::string& name, int n, int max_steps, uint64_t seed) : name_(name), n_(n) {
  int default_ms = -1;
  if (!make_env_params(name, &params_, &default_ms)) throw std::invalid_argument("unknown native env: " + name);
  if (n <= 0) throw std::invalid_argument("num_envs must be positive");
  max_steps_ = max_steps > 0 ? max_steps : default_ms;
  sdim_ = state_size(params_);
  state_.assign((size_t)n * sdim_, 0.f);
  rng_.resize(n);
  for (int i = 0; i < n; ++i) rng_[i] = seed_stream(seed, (uint64_t)i);
  t_.assign(n, 0);
  ret_acc_.assign(n, 0.0);
  if (is_image()) frames_.assign((size_t)n * kPongH * kPongW * kPongStack, 0);
}

void BatchedEnv::seed(const std::vector<uint64_t>& seeds) {
  if ((int)seeds.size() != n_) throw std::invalid_argument("need one seed per env");
  for (int i = 0; i < n_; ++i) rng_[i] = seed_stream(seeds[i], 0);
}

void BatchedEnv::render_pong(int i, bool reset_stack) {
  uint8_t* fr = frames_.data() + (size_t)i * kPongH * kPongW * kPongStack;
  const float* s = state_.data() + (size_t)i * sdim_;
  for (int r = 0; r < kPongH; ++r) {
    for (int c = 0; c < kPongW; ++c) {
      uint8_t* px = fr + ((size_t)r * kPongW + c) * kPongStack;
      uint8_t v = pong_pixel(s, r, c);
      if (reset_stack) {
        for (int k = 0; k < kPongStack; ++k) px[k] = v;
      } else {
        for (int k = 0; k < kPongStack - 1; ++k) px[k] = px[k + 1];
        px[kPongStack - 1] = v;
      }
    }
  }
}

void BatchedEnv::write_obs(int i, void* obs) {
  if (is_image()) {
    const size_t sz = (size_t)kPongH * kPongW * kPongStack;
    memcpy((uint8_t*)obs + (size_t)i * sz, frames_.data() + (size_t)i * sz, sz);
  } else {
    env_obs(params_, state_.data() + (size_t)i * sdim_, (float*)obs + (size_t)i * params_.obs_dim);
  }
}

void BatchedEnv::reset(void* obs) {
  for (int i = 0; i < n_; ++i) {
    env_reset(params_, state_.data() + (size_t)i * sdim_, rng_[i]);
    t_[i] = 0;
    ret_acc_[i] = 0.0;
    if (is_image()) render_pong(i, true);
    write_obs(i, obs);
  }
}

void BatchedEnv::step(const float* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc,
                      void* terminal_obs, double* ep_ret, int64_t* ep_len) {
  const int ad = params_.act_dim;
  const bool img = is_image();
  // Independent envs: parallelise across envs when the batch is large enough
  // to amortise thread start-up (per-env work is ~100 ns for classic control).
#pragma omp parallel for schedule(static) if (n_ >= 512 || (img && n_ >= 8))
  for (int i = 0; i < n_; ++i) {
    float* s = state_.data() + (size_t)i * sdim_;
    int is_term = 0;
    float r = env_step(params_, s, actions + (size_t)i * ad, &is_term, rng_[i]);
    t_[i] += 1;
    ret_acc_[i] += r;
    bool is_trunc = !is_term && max_steps_ > 0 && t_[i] >= max_steps_;
    rew[i] = r;
    term[i] = (uint8_t)is_term;
    trunc[i] = (uint8_t)is_trunc;
    if (img) render_pong(i, false);
    if (is_term || is_trunc) {
      write_obs(i, terminal_obs);
      ep_ret[i] = ret_acc_[i];
      ep_len[i] = t_[i];
      env_reset(params_, s, rng_[i]);
      t_[i] = 0;
      ret_acc_[i] = 0.0;
      if (img) render_pong(i, true);
    } else {
      ep_ret[i] = 0.0;
      ep_len[i] = 0;
    }
    write_obs(i, obs);
  }
}

}  // namespace ia

// Native batched vector environment (host side).
//
// Replaces the reference's per-env Python objects stepped through SB3
// DummyVecEnv/SubprocVecEnv (src/imitation/util/util.py:158-166): all envs of a
// rank live in one SoA block and are stepped in a single call, with SB3
// auto-reset semantics (the terminal observation is reported separately, as
// info["terminal_observation"] in rollout.py:162-167) and Monitor-style
// episode statistics (info["episode"], util/util.py:150).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "ia/envs.h"

namespace ia {

bool make_env_params(const std::string& name, EnvParams* out, int* default_max_steps);
std::vector<std::string> native_env_names();

class BatchedEnv {
 public:
  BatchedEnv(const std::string& name, int n, int max_steps, uint64_t seed);

  int num_envs() const { return n_; }
  int obs_dim() const { return params_.obs_dim; }
  int act_dim() const { return params_.act_dim; }
  int n_actions() const { return params_.n_actions; }
  int max_steps() const { return max_steps_; }
  bool is_image() const { return params_.kind == ENV_PONG; }
  int obs_numel() const { return is_image() ? kPongH * kPongW * kPongStack : params_.obs_dim; }
  int state_dim() const { return sdim_; }
  const EnvParams& params() const { return params_; }
  const std::string& name() const { return name_; }

  // Reseed env i's stream (used by VecEnv.seed / reset(seed=...)).
  void seed(const std::vector<uint64_t>& seeds);
  // Reset every env; obs is [n, obs_numel] (float32, or uint8 for image envs).
  void reset(void* obs);
  // Step with auto-reset. actions: [n, act_dim] float32 (discrete as float index).
  // Outputs: obs [n, obs_numel]; rew/term/trunc [n]; terminal_obs [n, obs_numel]
  // (valid where term|trunc); ep_ret/ep_len [n] (valid where term|trunc).
  void step(const float* actions, void* obs, float* rew, uint8_t* term, uint8_t* trunc, void* terminal_obs,
            double* ep_ret, int64_t* ep_len);

  // Raw state access for checkpointing / tests.
  std::vector<float>& state() { return state_; }
  std::vector<uint64_t>& rng() { return rng_; }
  std::vector<int64_t>& elapsed() { return t_; }
  std::vector<uint8_t>& frames() { return frames_; }

 private:
  void write_obs(int i, void* obs);
  void render_pong(int i, bool reset_stack);

  std::string name_;
  int n_;
  int max_steps_;
  int sdim_;
  EnvParams params_;
  std::vector<float> state_;
  std::vector<uint64_t> rng_;
  std::vector<int64_t> t_;
  std::vector<double> ret_acc_;
  std::vector<uint8_t> frames_;  // image envs: n * H * W * stack (HWC)
};

}  // namespace ia

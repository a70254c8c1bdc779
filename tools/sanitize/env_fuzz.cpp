// Host-sanitizer harness for the native env runtime: every native env is
// reset and stepped with random / out-of-range actions, its state saved and restored,
// under AddressSanitizer + UBSan. Host code only (no HIP calls, no GPU):
//   tools/sanitize/run.sh
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <vector>

#include "vec_env.h"

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 600;
  std::mt19937_64 gen(7);
  std::uniform_real_distribution<float> u(-2.f, 2.f);
  int n_envs_checked = 0;
  for (const std::string& name : ia::native_env_names()) {
    const int n = 3;
    ia::BatchedEnv env(name, n, 150, 1234);
    const int numel = env.obs_numel();
    const size_t obs_bytes = (size_t)n * numel * (env.is_image() ? 1 : sizeof(float));
    std::vector<uint8_t> obs(obs_bytes), tobs(obs_bytes);
    std::vector<float> rew(n), acts((size_t)n * (env.n_actions() > 0 ? 1 : env.act_dim()));
    std::vector<uint8_t> term(n), trunc(n);
    std::vector<double> ep_ret(n);
    std::vector<int64_t> ep_len(n);
    env.reset(obs.data());
    std::vector<float> saved_state;
    std::vector<uint64_t> saved_rng;
    for (int t = 0; t < steps; ++t) {
      for (size_t i = 0; i < acts.size(); ++i)
        acts[i] = env.n_actions() > 0 ? (float)(gen() % env.n_actions()) : u(gen);
      env.step(acts.data(), obs.data(), rew.data(), term.data(), trunc.data(), tobs.data(), ep_ret.data(), ep_len.data());
      for (int i = 0; i < n; ++i)
        if (!isfinite(rew[i])) { fprintf(stderr, "%s: non-finite reward\n", name.c_str()); return 1; }
      if (t == steps / 2) { saved_state = env.state(); saved_rng = env.rng(); }
    }
    env.state() = saved_state;
    env.rng() = saved_rng;
    env.step(acts.data(), obs.data(), rew.data(), term.data(), trunc.data(), tobs.data(), ep_ret.data(), ep_len.data());
    ++n_envs_checked;
  }
  printf("env_fuzz ok: %d envs x %d steps\n", n_envs_checked, steps);
  return 0;
}

// Device-resident rollout: policy sampling + env physics + learned reward for
// T steps of N envs in ONE launch (replaces the reference's per-step host loop:
// SB3 collect_rollouts -> policy.forward -> VecEnv.step over pipes ->
// RewardVecEnvWrapper -> reward_net.predict_processed with numpy<->device copies,
// SURVEY §3.1 hot loops).
//
// Mapping: one wave64 per env, one env per workgroup, so there is no
// inter-wave synchronisation at all in the T-step loop. Inside a wave an MLP
// layer is "lane j computes unit j": the layer input is broadcast lane->wave with
// v_readlane (SGPR operand, no LDS traffic), weights are read transposed from LDS
// ([din][64], lanes contiguous -> conflict-free ds_read_b32).  These nets are
// 8 rows wide per step, far below an MFMA tile: the VALU is the right unit here;
// the minibatch-sized work (PPO update, discriminator) runs on MFMA.
// Env physics runs on lane 0 from the shared __host__ __device__ headers
// (csrc/include/ia/envs.h) -- bit-for-bit the same model the host runtime steps.
#include <hip/hip_runtime.h>

#include "ia/engine.h"
#include "ia/envs.h"
#include "ia/mfma.h"
#include "ia/rng.h"
#include "launchers.h"

namespace ia {
namespace {

constexpr int kW = 64;  // transposed-weight row stride (one slot per lane)

struct LdsMLP {
  int n_layers;
  int dims[kWaveMaxLayers + 1];
  int hidden_act, out_act;
  float* WT[kWaveMaxLayers];  // [din][kW]
  float* b[kWaveMaxLayers];   // [kW]
  float* mean;                // [kW] or null
  float* rstd;                // [kW]
};

__device__ float* load_mlp(const WaveMLP& m, LdsMLP& out, float* lds) {
  out.n_layers = m.n_layers;
  out.hidden_act = m.hidden_act;
  out.out_act = m.out_act;
  for (int l = 0; l <= m.n_layers; ++l) out.dims[l] = m.dims[l];
  const int lane = threadIdx.x;
  for (int l = 0; l < m.n_layers; ++l) {
    const int din = m.dims[l], dout = m.dims[l + 1];
    out.WT[l] = lds;
    for (int e = lane; e < din * kW; e += 64) {
      const int k = e / kW, j = e - k * kW;
      lds[e] = j < dout ? m.W[l][j * din + k] : 0.f;
    }
    lds += din * kW;
    out.b[l] = lds;
    lds[lane] = lane < dout ? m.b[l][lane] : 0.f;
    lds += kW;
  }
  if (m.norm_mean) {
    out.mean = lds;
    out.rstd = lds + kW;
    const int d0 = m.dims[0];
    lds[lane] = lane < d0 ? m.norm_mean[lane] : 0.f;
    lds[kW + lane] = lane < d0 ? rsqrtf(m.norm_var[lane] + m.norm_eps) : 1.f;
    lds += 2 * kW;
  } else {
    out.mean = nullptr;
    out.rstd = nullptr;
  }
  return lds;
}

__device__ __forceinline__ float bcast(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

// Lane j of x holds input feature j (j < dims[0]); returns lane j = output unit j.
__device__ float wave_mlp(const LdsMLP& m, float x) {
  const int lane = threadIdx.x;
  float h = x;
  if (m.mean) h = lane < m.dims[0] ? (h - m.mean[lane]) * m.rstd[lane] : 0.f;
  for (int l = 0; l < m.n_layers; ++l) {
    const int din = m.dims[l];
    const float* WT = m.WT[l];
    float acc = m.b[l][lane];
    int k = 0;
    for (; k + 4 <= din; k += 4) {
      const float x0 = bcast(h, k), x1 = bcast(h, k + 1), x2 = bcast(h, k + 2), x3 = bcast(h, k + 3);
      acc = fmaf(WT[(k + 0) * kW + lane], x0, acc);
      acc = fmaf(WT[(k + 1) * kW + lane], x1, acc);
      acc = fmaf(WT[(k + 2) * kW + lane], x2, acc);
      acc = fmaf(WT[(k + 3) * kW + lane], x3, acc);
    }
    for (; k < din; ++k) acc = fmaf(WT[k * kW + lane], bcast(h, k), acc);
    const int act = l == m.n_layers - 1 ? m.out_act : m.hidden_act;
    h = lane < m.dims[l + 1] ? apply_act(act, acc) : 0.f;
  }
  return h;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ uint64_t hash3(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t s = a ^ (0x9E3779B97F4A7C15ull * (b + 1)) ^ (0xC2B2AE3D27D4EB4Full * (c + 1));
  splitmix64(s);
  return s;
}

__global__ __launch_bounds__(64) void rollout_kernel(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int n = blockIdx.x;
  const int lane = threadIdx.x;
  const EnvParams& P = a.P;
  const int D = P.obs_dim;
  const int A = a.n_actions > 0 ? 1 : P.act_dim;
  const int S = state_size(P);
  LdsMLP pi, vf, rw;
  float* p = lds;
  p = load_mlp(a.pi, pi, p);
  p = load_mlp(a.vf, vf, p);
  if (a.rew_enabled) p = load_mlp(a.rew, rw, p);
  float* st = p;       // [kMaxState]
  float* ob = st + kMaxState;  // [kEngineMaxObs]
  float* act = ob + kEngineMaxObs;  // [kWaveMaxDim]
  for (int i = lane; i < S; i += 64) st[i] = a.state[(size_t)n * S + i];
  __syncthreads();

  float o = lane < D ? a.cur_obs[(size_t)n * D + lane] : 0.f;
  float start = a.cur_start[n];
  uint64_t rng = a.rng[n];
  int elapsed = a.elapsed[n];
  float ep_ret = a.ep_ret[n];
  const float lstd = (a.log_std && lane < A) ? a.log_std[lane] : 0.f;
  const float half_log2pi = 0.91893853320467274f;

  for (int t = 0; t < a.T; ++t) {
    const size_t row = (size_t)t * a.N + n;
    if (lane < D) a.obs_buf[row * D + lane] = o;
    if (lane == 0) a.starts[row] = start;
    // ---- policy + value
    const float head = wave_mlp(pi, o);
    const float value = bcast(wave_mlp(vf, o), 0);
    const uint64_t key = hash3(a.seed, (uint64_t)n, (uint64_t)(a.step0 + t));
    float a_raw, a_env, logp;
    if (a.n_actions > 0) {
      // Categorical: inverse-CDF sample on the softmax of the logits
      const float lg = lane < a.n_actions ? head : -INFINITY;
      const float mx = wave_max(lg);
      const float ex = lane < a.n_actions ? expf(lg - mx) : 0.f;
      const float z = wave_sum(ex);
      uint64_t s = key;
      const float u = uniform01(s) * z;
      // inclusive prefix over lanes
      float c = ex;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const float y = __shfl_up(c, off);
        if (lane >= off) c += y;
      }
      const unsigned long long m = __ballot(c > u && lane < a.n_actions);
      int k = m ? __builtin_ctzll(m) : a.n_actions - 1;
      const float lp = bcast(lg, k) - mx - logf(z);
      a_raw = (float)k;
      a_env = (float)k;
      logp = lp;
    } else {
      uint64_t s = key ^ (0xD6E8FEB86659FD93ull * (lane + 1));
      const float eps = normal01(s);
      const float std = expf(lstd);
      a_raw = head + std * eps;
      const float lp = lane < A ? (-0.5f * eps * eps - lstd - half_log2pi) : 0.f;
      logp = wave_sum(lp);
      a_env = lane < A ? fminf(fmaxf(a_raw, a.act_low[lane]), a.act_high[lane]) : 0.f;
    }
    if (lane < A) {
      a.act_raw[row * A + lane] = a_raw;
      a.act_env[row * A + lane] = a_env;
      act[lane] = a_env;
    }
    // ---- env step (lane 0), SB3 auto-reset + TimeLimit + Monitor
    __syncthreads();
    int term = 0;
    float r_env = 0.f;
    if (lane == 0) {
      r_env = env_step(P, st, act, &term, rng);
      env_obs(P, st, ob);
    }
    __syncthreads();
    term = __builtin_amdgcn_readfirstlane(term);
    r_env = bcast(r_env, 0);
    elapsed += 1;
    ep_ret += r_env;
    const bool trunc = !term && elapsed >= a.max_steps;
    const bool done = term || trunc;
    const float o_next = lane < D ? ob[lane] : 0.f;  // terminal obs when done
    // ---- learned reward R(s, a, s', d)
    float r = r_env;
    if (a.rew_enabled) {
      float x = 0.f;
      int off = 0;
      if (a.use_state) { if (lane < D) x = o; off += D; }
      if (a.use_action) {
        float av;
        if (a.n_actions > 0) {
          const int k = (int)bcast(a_env, 0);
          av = (lane - off) == k ? 1.f : 0.f;
          if (lane >= off && lane < off + a.n_actions) x = av;
          off += a.n_actions;
        } else {
          av = __shfl(a_env, lane - off);
          if (lane >= off && lane < off + A) x = av;
          off += A;
        }
      }
      if (a.use_next_state) {
        const float v = __shfl(o_next, lane - off);
        if (lane >= off && lane < off + D) x = v;
        off += D;
      }
      if (a.use_done) { if (lane == off) x = done ? 1.f : 0.f; off += 1; }
      float logit = bcast(wave_mlp(rw, x), 0);
      r = a.rew_transform == REW_SOFTPLUS ? (logit > 0.f ? logit + log1pf(expf(-logit)) : log1pf(expf(logit))) : logit;
    }
    if (trunc) {  // SB3: bootstrap the value of the truncated terminal obs into the reward
      r += a.gamma * bcast(wave_mlp(vf, o_next), 0);
    }
    if (lane == 0) {
      a.logp[row] = logp;
      a.values[row] = value;
      a.rewards[row] = r;
      a.env_rew[row] = r_env;
      a.dones[row] = done ? 1.f : 0.f;
      a.ep_ret_out[row] = done ? ep_ret : 0.f;
    }
    if (lane < D) a.next_obs[row * D + lane] = o_next;
    if (done) {
      __syncthreads();
      if (lane == 0) {
        env_reset(P, st, rng);
        env_obs(P, st, ob);
      }
      __syncthreads();
      elapsed = 0;
      ep_ret = 0.f;
      o = lane < D ? ob[lane] : 0.f;
    } else {
      o = o_next;
    }
    start = done ? 1.f : 0.f;
  }
  // bootstrap value of the final observation
  const float lastv = bcast(wave_mlp(vf, o), 0);
  __syncthreads();
  for (int i = lane; i < S; i += 64) a.state[(size_t)n * S + i] = st[i];
  if (lane < D) a.cur_obs[(size_t)n * D + lane] = o;
  if (lane == 0) {
    a.cur_start[n] = start;
    a.last_values[n] = lastv;
    a.elapsed[n] = elapsed;
    a.ep_ret[n] = ep_ret;
  }
  // lane 0's rng advanced inside env_step/env_reset; persist it
  rng = (uint64_t)__builtin_amdgcn_readfirstlane((int)(rng & 0xffffffffu)) |
        ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(rng >> 32)) << 32);
  if (lane == 0) a.rng[n] = rng;
}

int mlp_lds_floats(const WaveMLP& m) {
  int f = 0;
  for (int l = 0; l < m.n_layers; ++l) f += m.dims[l] * kW + kW;
  if (m.norm_mean) f += 2 * kW;
  return f;
}

}  // namespace

size_t rollout_lds_bytes(const RolloutArgs& a) {
  int f = mlp_lds_floats(a.pi) + mlp_lds_floats(a.vf) + (a.rew_enabled ? mlp_lds_floats(a.rew) : 0);
  f += kMaxState + kEngineMaxObs + kWaveMaxDim;
  return (size_t)f * sizeof(float);
}

hipError_t rollout_launch(const RolloutArgs& a, hipStream_t s) {
  if (a.T <= 0 || a.N <= 0) return hipSuccess;
  const size_t lds = rollout_lds_bytes(a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rollout_kernel, dim3(a.N), dim3(64), lds, s, a);
  return hipGetLastError();
}

}  // namespace ia

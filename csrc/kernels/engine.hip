// Device rollout, parallel part: everything a rollout step records but the next step
// does not depend on, recomputed for all T x N transitions at once after the serial
// chain (rollout.hip) -- the value estimate V(s_t), the log-prob of the sampled action,
// the TimeLimit bootstrap gamma V(s_T) on truncation (SB3 collect_rollouts), the
// learned reward R(s, a, s', d) of GAIL / AIRL / preference comparisons (softplus /
// raw, optional potential shaping) and V of the final observations. Plus the
// NormalizedRewardNet output normalisation replay (sequential in t).
//
// Mapping: one wave per row, rows strided over the grid; in a wave an MLP layer is
// "lane j computes unit j", the input is broadcast with v_readlane, the weights are
// read transposed from LDS ([din][64], lanes contiguous -> conflict-free b128 reads),
// staged once per workgroup. 4096-row rounds fill every CU.
#include <hip/hip_runtime.h>

#include "ia/engine.h"
#include "ia/wave.h"
#include "launchers.h"

namespace ia {
namespace {

constexpr int kW = 64;  // one weight slot per lane

__host__ __device__ __forceinline__ int ceil8(int x) { return (x + 7) & ~7; }

// Weight image of one layer: [ceil8(din)/4][64 lanes][4 k] so lane j fetches the
// weights of 4 consecutive inputs of unit j with one ds_read_b128; zero-padded.
struct LdsMLP {
  int n_layers;
  int dims[kWaveMaxLayers + 1];
  int hidden_act, out_act;
  lf* WT[kWaveMaxLayers];
  lf* b[kWaveMaxLayers];  // [kW]
  lf* mean;               // [kW] or null
  lf* rstd;               // [kW]
};

__device__ __forceinline__ int wt_index(int k, int j) { return ((k >> 2) * kW + j) * 4 + (k & 3); }

__device__ lf* load_mlp(const WaveMLP& m, LdsMLP& out, lf* lds) {
  out.n_layers = m.n_layers;
  out.hidden_act = m.hidden_act;
  out.out_act = m.out_act;
#pragma unroll
  for (int l = 0; l <= kWaveMaxLayers; ++l) out.dims[l] = l <= m.n_layers ? m.dims[l] : 0;
  const int lane = threadIdx.x & 63;
  // every thread of the workgroup takes part: element e of the zero-padded [64][dp] weight
  // matrix goes to thread e % blockDim.x, so consecutive threads read consecutive inputs of
  // one unit (coalesced) and 4 loads are in flight per thread before their LDS stores
  const int tid = threadIdx.x, nth = blockDim.x;
#pragma unroll
  for (int l = 0; l < kWaveMaxLayers; ++l) {
    if (l < m.n_layers) {
      const int din = m.dims[l], dout = m.dims[l + 1], dp = ceil8(din);
      const float* W = m.W[l];
      out.WT[l] = lds;
      const int n_el = dp * kW;
#pragma unroll 4
      for (int e = tid; e < n_el; e += nth) {
        const int j = e / dp, k = e - j * dp;
        lds[wt_index(k, j)] = (j < dout && k < din) ? W[j * din + k] : 0.f;
      }
      lds += n_el;
      out.b[l] = lds;
      if (tid < kW) lds[tid] = tid < dout ? m.b[l][tid] : 0.f;
      lds += kW;
    } else {
      out.WT[l] = nullptr;
      out.b[l] = nullptr;
    }
  }
  if (m.norm_mean) {
    out.mean = lds;
    out.rstd = lds + kW;
    const int d0 = m.dims[0];
    if (tid < kW) {
      lds[tid] = tid < d0 ? m.norm_mean[tid] : 0.f;
      lds[kW + tid] = tid < d0 ? rsqrtf(m.norm_var[tid] + m.norm_eps) : 1.f;
    }
    lds += 2 * kW;
  } else {
    out.mean = nullptr;
    out.rstd = nullptr;
  }
  return lds;
}

// acc_j += sum_k W[j][k] * x_k, x_k = readlane(h, k) (k uniform), 8 inputs per step:
// both 16-byte weight fetches are issued before the FMA chain.
// Two interleaved FMA chains (even / odd inputs) halve the dependent-FMA depth.
__device__ __forceinline__ float layer_dot(const lf* WT, int din, float h, float acc) {
  const lf4* w4 = (const lf4*)WT + (threadIdx.x & 63);
  const int dp = ceil8(din);
  float acc1 = 0.f;
  for (int k = 0; k < dp; k += 8) {
    const f32v4 w0 = w4[(k >> 2) * kW], w1 = w4[((k >> 2) + 1) * kW];
    acc = fmaf(w0.x, bcast(h, k + 0), acc);
    acc1 = fmaf(w0.y, bcast(h, k + 1), acc1);
    acc = fmaf(w0.z, bcast(h, k + 2), acc);
    acc1 = fmaf(w0.w, bcast(h, k + 3), acc1);
    acc = fmaf(w1.x, bcast(h, k + 4), acc);
    acc1 = fmaf(w1.y, bcast(h, k + 5), acc1);
    acc = fmaf(w1.z, bcast(h, k + 6), acc);
    acc1 = fmaf(w1.w, bcast(h, k + 7), acc1);
  }
  return acc + acc1;
}

// Lane j of x holds input feature j (j < dims[0]); returns lane j = output unit j.
// Inputs beyond dims[0] must be zero (padded weight rows multiply them).
__device__ float wave_mlp(const LdsMLP& m, float x) {
  const int lane = threadIdx.x & 63;
  float h = x;
  if (m.mean) h = lane < m.dims[0] ? (h - m.mean[lane]) * m.rstd[lane] : 0.f;
#pragma unroll
  for (int l = 0; l < kWaveMaxLayers; ++l) {
    if (l < m.n_layers) {
      const float acc = layer_dot(m.WT[l], m.dims[l], h, m.b[l][lane]);
      const int act = l == m.n_layers - 1 ? m.out_act : m.hidden_act;
      h = lane < m.dims[l + 1] ? act_fast(act, acc) : 0.f;
    }
  }
  return h;
}



int mlp_lds_floats(const WaveMLP& m) {
  int f = 0;
  for (int l = 0; l < m.n_layers; ++l) f += ceil8(m.dims[l]) * kW + kW;
  if (m.norm_mean) f += 2 * kW;
  return f;
}

// Reward-net input [s | a | s' | d] in lane layout (lane k = feature k).
__device__ __forceinline__ float reward_input(const RolloutPostArgs& a, float o, float o_next, float a_env, bool done) {
  const int lane = threadIdx.x & 63;
  const int D = a.D, A = a.A;
  float x = 0.f;
  int off = 0;
  if (a.use_state) { if (lane < D) x = o; off += D; }
  if (a.use_action) {
    if (a.n_actions > 0) {
      const int k = (int)bcast(a_env, 0);
      if (lane >= off && lane < off + a.n_actions) x = (lane - off) == k ? 1.f : 0.f;
      off += a.n_actions;
    } else {
      const float av = __shfl(a_env, lane - off);
      if (lane >= off && lane < off + A) x = av;
      off += A;
    }
  }
  if (a.use_next_state) {
    const float v = __shfl(o_next, lane - off);
    if (lane >= off && lane < off + D) x = v;
    off += D;
  }
  if (a.use_done) { if (lane == off) x = done ? 1.f : 0.f; }
  return x;
}

}  // namespace

// (count, mean, biased var) of a <- a merged with b (Chan et al.; the update of
// RunningNorm.update_stats for b = one step's batch). a empty: b exactly.
__device__ __forceinline__ void chan_merge(float& n, float& m, float& v, float bn, float bm, float bv) {
  if (bn <= 0.f) return;
  if (n <= 0.f) {
    n = bn;
    m = bm;
    v = bv;
    return;
  }
  const float delta = bm - m, tot = n + bn;
  m += delta * bn / tot;
  v = (v * n + bv * bn + delta * delta * n * bn / tot) / tot;
  n = tot;
}

// NormalizedRewardNet output normalisation (see OutNormArgs), sequential in t. Three phases
// instead of one serial wave: (A) every step's batch moments in parallel (they do not depend
// on the running state), (B) the Chan recurrence over the steps as a wave-level scan,
// recording the running (mean, var) each step is normalised with, (C) every reward in
// parallel. Steps go through LDS in chunks of kOutNormChunk. Measured (AIRL Hopper, T = 1024,
// one MI355X): 163 us with (B) on one lane.
constexpr int kOutNormThreads = 256;
constexpr int kOutNormChunk = 4096;

__global__ __launch_bounds__(kOutNormThreads) void reward_outnorm_kernel(OutNormArgs a) {
  __shared__ float sm[kOutNormChunk], sv[kOutNormChunk], sn[kOutNormChunk];
  __shared__ float state[3];
  const int tid = threadIdx.x;
  if (tid == 0) {
    state[0] = a.mean[0];
    state[1] = a.var[0];
    state[2] = a.count_i ? (float)a.count_i[0] : a.count[0];
  }
  for (int t0 = 0; t0 < a.T; t0 += kOutNormChunk) {
    const int nt = min(kOutNormChunk, a.T - t0);
    // (A) batch moments of each step (over the N envs, or the global ones under DP)
    for (int j = tid; j < nt; j += kOutNormThreads) {
      const int t = t0 + j;
      float bm, bv, bn;
      if (a.step_stats) {
        bn = a.step_stats[3 * t];
        bm = a.step_stats[3 * t + 1];
        bv = a.step_stats[3 * t + 2];
      } else {
        bn = (float)a.N;
        const float* x = a.rew_raw + (size_t)t * a.N;
        float s = 0.f;
        for (int n = 0; n < a.N; ++n) s += x[n];
        bm = s / bn;
        float q = 0.f;
        for (int n = 0; n < a.N; ++n) {
          const float d = x[n] - bm;
          q += d * d;
        }
        bv = q / bn;
      }
      sm[j] = bm;
      sv[j] = bv;
      sn[j] = bn;
    }
    __syncthreads();
    // (B) running state before each step (replaces the step's moments in LDS): a Chan merge
    // is associative, so wave 0 scans it -- lane l folds its run of steps, a 6-level prefix
    // scan over the lanes gives each run's carry-in, and each lane replays its run from there
    // (~2 x nt / 64 dependent merges instead of nt on one lane)
    if (tid < 64) {
      const int lane = tid;
      const int per = (nt + 63) >> 6;
      const int j0 = min(lane * per, nt), j1 = min(j0 + per, nt);
      float n = 0.f, m = 0.f, v = 0.f;  // this lane's run, folded (n = 0: identity)
      for (int j = j0; j < j1; ++j) chan_merge(n, m, v, sn[j], sm[j], sv[j]);
#pragma unroll
      for (int k = 1; k < 64; k <<= 1) {  // inclusive prefix over lanes 0..l
        const float on = __shfl_up(n, k, 64), om = __shfl_up(m, k, 64), ov = __shfl_up(v, k, 64);
        if (lane >= k) {
          float pn = on, pm = om, pv = ov;
          chan_merge(pn, pm, pv, n, m, v);
          n = pn;
          m = pm;
          v = pv;
        }
      }
      // carry-in: the running state, then the runs of lanes 0..l-1
      float cn = __shfl_up(n, 1, 64), cm = __shfl_up(m, 1, 64), cv = __shfl_up(v, 1, 64);
      float rn = state[2], rm = state[0], rv = state[1];
      if (lane > 0) chan_merge(rn, rm, rv, cn, cm, cv);
      for (int j = j0; j < j1; ++j) {
        const float bn = sn[j], bm = sm[j], bv = sv[j];
        sm[j] = rm;
        sv[j] = rv;
        chan_merge(rn, rm, rv, bn, bm, bv);
      }
      // the state after the chunk: lane 63's run ends it (runs past nt are empty)
      const int last = nt > 0 ? min((nt - 1) / per, 63) : 0;
      const float fn = __shfl(rn, last, 64), fm = __shfl(rm, last, 64), fv = __shfl(rv, last, 64);
      if (lane == 0) {
        state[0] = fm;
        state[1] = fv;
        state[2] = fn;
      }
    }
    __syncthreads();
    // (C) normalised rewards + TimeLimit bootstrap
    const int n_el = nt * a.N;
    for (int e = tid; e < n_el; e += kOutNormThreads) {
      const int j = e / a.N;
      const size_t i = (size_t)t0 * a.N + e;
      const float rstd = 1.f / sqrtf(sv[j] + a.eps);
      a.rewards[i] = (a.rew_raw[i] - sm[j]) * rstd + a.boot[i];
    }
    __syncthreads();
  }
  if (tid == 0) {
    a.mean[0] = state[0];
    a.var[0] = state[1];
    if (a.count_i) a.count_i[0] = (int)state[2];
    else a.count[0] = state[2];
  }
}
constexpr int kPostWaves = 8;  // waves per workgroup sharing one LDS image of the nets

__global__ __launch_bounds__(64 * kPostWaves) void rollout_post_kernel(RolloutPostArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_raw[];
  lf* p = (lf*)lds_raw;
  const int lane = threadIdx.x & 63;
  LdsMLP pi, vf, rw, pt;
  const bool need_pi = a.logp != nullptr;
  if (need_pi) p = load_mlp(a.pi, pi, p);
  p = load_mlp(a.vf, vf, p);
  if (a.rew_enabled) p = load_mlp(a.rew, rw, p);
  if (a.rew_enabled && a.shaped) p = load_mlp(a.pot, pt, p);
  __syncthreads();
  const int D = a.D, A = a.A;
  const bool discrete = a.n_actions > 0;
  const int rows = a.T * a.N;
  const float lstd = (!discrete && a.log_std && lane < A) ? a.log_std[lane] : 0.f;
  const float inv_sd = expf(-lstd);
  const float half_log2pi = 0.91893853320467274f;
  const int wave = threadIdx.x >> 6;
  for (int row = blockIdx.x * kPostWaves + wave; row < rows + a.N; row += gridDim.x * kPostWaves) {
    if (row >= rows) {  // bootstrap value of the final observations
      const int n = row - rows;
      const float o = lane < D ? a.cur_obs[(size_t)n * D + lane] : 0.f;
      const float v = bcast(wave_mlp(vf, o), 0);
      if (lane == 0) a.last_values[n] = v;
      continue;
    }
    const size_t r64 = (size_t)row;
    const float o = lane < D ? a.obs[r64 * D + lane] : 0.f;
    const float o_next = lane < D ? a.next_obs[r64 * D + lane] : 0.f;
    const float a_raw = lane < A ? a.act_raw[r64 * A + lane] : 0.f;
    const float a_env = lane < A ? a.act_env[r64 * A + lane] : 0.f;
    const bool done = a.dones[r64] > 0.5f;
    const bool trunc = a.trunc[r64] > 0.5f;
    const float value = bcast(wave_mlp(vf, o), 0);
    float logp = 0.f;
    if (need_pi) {  // distribution.log_prob(actions) of the rollout-time policy
      const float head = wave_mlp(pi, o);
      if (discrete) {
        const float lg = lane < a.n_actions ? head : -INFINITY;
        const float mx = wave_max(lg);
        const float z = wave_sum(lane < a.n_actions ? expf(lg - mx) : 0.f);
        logp = bcast(head, (int)bcast(a_raw, 0)) - mx - logf(z);
      } else {
        const float zz = (a_raw - head) * inv_sd;
        logp = wave_sum(lane < A ? (-0.5f * zz * zz - lstd - half_log2pi) : 0.f);
      }
    }
    // SB3: on truncation the value of the terminal observation is bootstrapped into the reward
    const float bt = trunc ? a.gamma * bcast(wave_mlp(vf, o_next), 0) : 0.f;
    float r = 0.f;
    if (a.rew_enabled) {
      const float logit = bcast(wave_mlp(rw, reward_input(a, o, o_next, a_env, done)), 0);
      r = a.rew_transform == REW_SOFTPLUS ? softplus_f(logit) : logit;
      if (a.shaped) {  // AIRL potential shaping (reward_nets.py ShapedRewardNet.forward)
        const float phi_s = bcast(wave_mlp(pt, o), 0);
        const float phi_n = done ? 0.f : bcast(wave_mlp(pt, o_next), 0);
        r += a.shaping_gamma * phi_n - phi_s;
      }
    }
    if (lane == 0) {
      a.values[r64] = value;
      if (need_pi) a.logp[r64] = logp;
      a.boot[r64] = bt;
      if (a.rew_raw && a.rew_enabled) a.rew_raw[r64] = r;
      a.rewards[r64] = (a.rew_enabled ? r : a.env_rew[r64]) + bt;
    }
  }
}

size_t rollout_post_lds_bytes(const RolloutPostArgs& a) {
  int f = (a.logp ? mlp_lds_floats(a.pi) : 0) + mlp_lds_floats(a.vf);
  if (a.rew_enabled) f += mlp_lds_floats(a.rew) + (a.shaped ? mlp_lds_floats(a.pot) : 0);
  return (size_t)f * sizeof(float);
}

hipError_t rollout_post_launch(const RolloutPostArgs& a, hipStream_t s) {
  const int rows = a.T * a.N + a.N;
  if (a.T <= 0 || a.N <= 0) return hipSuccess;
  if (a.D > kEngineMaxObs || a.A > kWaveMaxDim) return hipErrorInvalidValue;
  const size_t lds = rollout_post_lds_bytes(a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  // one transition per wave (the per-row chain of 3-4 small MLPs is latency bound, so the
  // rows go wide: 4096 rows = 512 workgroups, two per CU at this kernel's LDS / VGPR use); the
  // N bootstrap rows are second rows of the first N waves (one value net each).
  // Measured (one MI355X): GAIL HalfCheetah (4104 rows, 3 nets) 78 -> 27 us, AIRL Hopper
  // (8200 rows, 4 nets) 304 -> 104 us, against 4-wave workgroups of 2 rows per wave that
  // loaded the weights wave by wave with strided reads (profiles/r4_rollout_breakdown.md).
  const int grid = (a.T * a.N + kPostWaves - 1) / kPostWaves;
  hipLaunchKernelGGL(rollout_post_kernel, dim3(grid), dim3(64 * kPostWaves), lds, s, a);
  return hipGetLastError();
}

hipError_t reward_outnorm_launch(const OutNormArgs& a, hipStream_t s) {
  if (a.T <= 0 || a.N <= 0) return hipSuccess;
  hipLaunchKernelGGL(reward_outnorm_kernel, dim3(1), dim3(kOutNormThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace ia

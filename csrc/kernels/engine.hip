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

constexpr int kW = 64;  // one weight slot per lane

// LDS pointers typed address_space(3) (32-bit, ds_read/ds_write).
typedef __attribute__((address_space(3))) float lf;
typedef float f32v4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f32v4 lf4;

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
  const int lane = threadIdx.x;
#pragma unroll
  for (int l = 0; l < kWaveMaxLayers; ++l) {
    if (l < m.n_layers) {
      const int din = m.dims[l], dout = m.dims[l + 1], dp = ceil8(din);
      out.WT[l] = lds;
      for (int k = 0; k < dp; ++k) lds[wt_index(k, lane)] = (lane < dout && k < din) ? m.W[l][lane * din + k] : 0.f;
      lds += dp * kW;
      out.b[l] = lds;
      lds[lane] = lane < dout ? m.b[l][lane] : 0.f;
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
    lds[lane] = lane < d0 ? m.norm_mean[lane] : 0.f;
    lds[kW + lane] = lane < d0 ? rsqrtf(m.norm_var[lane] + m.norm_eps) : 1.f;
    lds += 2 * kW;
  } else {
    out.mean = nullptr;
    out.rstd = nullptr;
  }
  return lds;
}

// The rollout / reward kernels run ONE wave per workgroup: lanes exchange data through
// LDS, and a wave's LDS accesses complete in issue order, so a wavefront-scope fence (a
// compiler ordering point) replaces __syncthreads(). The workgroup-scope release of
// __syncthreads() would also wait for every outstanding global store of the step
// (vmcnt(0)) -- an L2 round trip on the serial step chain.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float bcast(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}

// acc_j += sum_k W[j][k] * x_k, x_k = readlane(h, k) (k uniform), 8 inputs per step:
// both 16-byte weight fetches are issued before the FMA chain.
__device__ __forceinline__ float layer_dot(const lf* WT, int din, float h, float acc) {
  const lf4* w4 = (const lf4*)WT + threadIdx.x;
  const int dp = ceil8(din);
  for (int k = 0; k < dp; k += 8) {
    const f32v4 w0 = w4[(k >> 2) * kW], w1 = w4[((k >> 2) + 1) * kW];
    acc = fmaf(w0.x, bcast(h, k + 0), acc);
    acc = fmaf(w0.y, bcast(h, k + 1), acc);
    acc = fmaf(w0.z, bcast(h, k + 2), acc);
    acc = fmaf(w0.w, bcast(h, k + 3), acc);
    acc = fmaf(w1.x, bcast(h, k + 4), acc);
    acc = fmaf(w1.y, bcast(h, k + 5), acc);
    acc = fmaf(w1.z, bcast(h, k + 6), acc);
    acc = fmaf(w1.w, bcast(h, k + 7), acc);
  }
  return acc;
}

// Fast tanh for the rollout policy/reward nets (|err| ~1e-7 abs).
__device__ __forceinline__ float act_fast(int act, float x) {
  if (act == ACT_TANH) {
    const float e = __expf(2.f * fminf(fmaxf(x, -15.f), 15.f));
    return 1.f - 2.f / (e + 1.f);
  }
  return apply_act(act, x);
}

// Lane j of x holds input feature j (j < dims[0]); returns lane j = output unit j.
// Inputs beyond dims[0] must be zero (padded weight rows multiply them).
__device__ float wave_mlp(const LdsMLP& m, float x) {
  const int lane = threadIdx.x;
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

// Actor and critic evaluated together: lanes [0,32) = actor units, [32,64) = critic
// units (both nets <= 32 wide, same depth, shared input normaliser). Halves the
// serial k-loop of the two per-step policy evaluations.
struct PairMLP {
  int n_layers;
  int din[kWaveMaxLayers];  // max(din_pi, din_vf) per layer
  int dpi[kWaveMaxLayers + 1], dvf[kWaveMaxLayers + 1];
  int hidden_act;
  lf* WT[kWaveMaxLayers];
  lf* b[kWaveMaxLayers];  // [64]
  lf* mean;
  lf* rstd;
};

__device__ bool pair_ok(const WaveMLP& pi, const WaveMLP& vf) {
  if (pi.n_layers != vf.n_layers || pi.dims[0] != vf.dims[0] || pi.hidden_act != vf.hidden_act) return false;
  for (int l = 0; l <= pi.n_layers; ++l)
    if (pi.dims[l] > 32 || vf.dims[l] > 32) return false;
  return true;
}

__host__ __device__ inline int pair_lds_floats(const WaveMLP& pi, const WaveMLP& vf) {
  int f = 0;
  for (int l = 0; l < pi.n_layers; ++l) {
    const int din = pi.dims[l] > vf.dims[l] ? pi.dims[l] : vf.dims[l];
    f += ceil8(din) * kW + kW;
  }
  return f + (pi.norm_mean ? 2 * kW : 0);
}

__device__ lf* load_pair(const WaveMLP& pi, const WaveMLP& vf, PairMLP& out, lf* lds) {
  const int lane = threadIdx.x;
  out.n_layers = pi.n_layers;
  out.hidden_act = pi.hidden_act;
#pragma unroll
  for (int l = 0; l <= kWaveMaxLayers; ++l) {
    out.dpi[l] = l <= pi.n_layers ? pi.dims[l] : 0;
    out.dvf[l] = l <= vf.n_layers ? vf.dims[l] : 0;
  }
  const bool hi = lane >= 32;
  const int j = hi ? lane - 32 : lane;
#pragma unroll
  for (int l = 0; l < kWaveMaxLayers; ++l) {
    if (l < pi.n_layers) {
      const int dp = pi.dims[l], dv = vf.dims[l], din = dp > dv ? dp : dv;
      const int op = pi.dims[l + 1], ov = vf.dims[l + 1];
      out.din[l] = din;
      out.WT[l] = lds;
      for (int k = 0; k < ceil8(din); ++k) {
        float v = 0.f;
        if (!hi && j < op && k < dp) v = pi.W[l][j * dp + k];
        if (hi && j < ov && k < dv) v = vf.W[l][j * dv + k];
        lds[wt_index(k, lane)] = v;
      }
      lds += ceil8(din) * kW;
      out.b[l] = lds;
      lds[lane] = !hi ? (j < op ? pi.b[l][j] : 0.f) : (j < ov ? vf.b[l][j] : 0.f);
      lds += kW;
    } else {
      out.din[l] = 0;
      out.WT[l] = nullptr;
      out.b[l] = nullptr;
    }
  }
  if (pi.norm_mean) {
    out.mean = lds;
    out.rstd = lds + kW;
    const int d0 = pi.dims[0];
    lds[lane] = lane < d0 ? pi.norm_mean[lane] : 0.f;
    lds[kW + lane] = lane < d0 ? rsqrtf(pi.norm_var[lane] + pi.norm_eps) : 1.f;
    lds += 2 * kW;
  } else {
    out.mean = nullptr;
    out.rstd = nullptr;
  }
  return lds;
}

// x: lane k < dims[0] holds feature k. Returns lane j<dpi[L]: actor output j; lane 32: value.
__device__ float pair_mlp(const PairMLP& m, float x) {
  const int lane = threadIdx.x;
  const bool hi = lane >= 32;
  float h = x;
  if (m.mean) h = lane < m.dpi[0] ? (h - m.mean[lane]) * m.rstd[lane] : 0.f;
#pragma unroll
  for (int l = 0; l < kWaveMaxLayers; ++l) {
    if (l < m.n_layers) {
      float acc = m.b[l][lane];
      if (l == 0) {
        acc = layer_dot(m.WT[l], m.din[l], h, acc);
      } else {  // actor lanes read actor units (lanes k), critic lanes read critic units (32 + k)
        const lf4* w4 = (const lf4*)m.WT[l] + lane;
        const int dp = ceil8(m.din[l]);
        for (int k = 0; k < dp; k += 8) {
          const f32v4 w0 = w4[(k >> 2) * kW], w1 = w4[((k >> 2) + 1) * kW];
          const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float lo = bcast(h, k + u), up = bcast(h, 32 + k + u);
            acc = fmaf(wv[u], hi ? up : lo, acc);
          }
        }
      }
      const bool last = l == m.n_layers - 1;
      const int dout = hi ? m.dvf[l + 1] : m.dpi[l + 1];
      const int j = hi ? lane - 32 : lane;
      h = j < dout ? (last ? acc : act_fast(m.hidden_act, acc)) : 0.f;
    }
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

// Locomotion model stepped by the whole wave: joint j on lane j, root dynamics
// computed redundantly (uniformly) by every lane, cross-joint sums taken with
// readlane in joint order (the host runtime's summation order). Same equations as
// ia::loco_step (csrc/include/ia/envs.h); the serial per-joint chain of the host
// version is what made the env step the longest part of a rollout step.
// Per-lane joint constants, loaded once per kernel (a lane-indexed kernarg read is a
// vector memory load; inside the step it would wait behind the step's global stores).
struct LocoLane {
  float gear, stiff, damp, thrust;
};

__device__ LocoLane loco_lane(const LocoParams& p) {
  const int lane = threadIdx.x;
  const bool jl = lane < p.nj;
  return {jl ? p.gear[lane] : 0.f, jl ? p.stiff[lane] : 0.f, jl ? p.damp[lane] : 0.f, jl ? p.thrust[lane] : 0.f};
}

// The env state / action scratch live in LDS: accessed through LDS-typed pointers
// (ds_read / ds_write, lgkmcnt) rather than generic ones -- a flat access waits on vmcnt,
// i.e. behind every global store the step has issued (gfx9 counts stores in vmcnt).
__device__ float loco_step_wave(const LocoParams& p, const LocoLane& ll, float* s_gen, const float* a_gen) {
  lf* s = (lf*)s_gen;
  const lf* a_in = (const lf*)a_gen;
  const int lane = threadIdx.x;
  const int nq = loco_nq(p), nj = p.nj, jq = p.nq_root, jv = p.nv_root;
  const bool jl = lane < nj;
  const float a = jl ? fminf(fmaxf(a_in[lane], -1.f), 1.f) : 0.f;
  float q = jl ? s[jq + lane] : 0.f;
  float qd = jl ? s[nq + jv + lane] : 0.f;
  const float gear = ll.gear, stiff = ll.stiff, damp = ll.damp, tc = ll.thrust;
  float ctrl = 0.f, pitch = 0.f;
  for (int j = 0; j < nj; ++j) {
    const float aj = bcast(a, j);
    ctrl += aj * aj;
    pitch += p.pitch_coupling[j] * aj;
  }
  float rq[8], rv[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    rq[i] = i < p.nq_root ? s[i] : 0.f;
    rv[i] = i < p.nv_root ? s[nq + i] : 0.f;
  }
  const float x_before = rq[0];
  const float dt = p.dt;
  for (int sub = 0; sub < p.frame_skip; ++sub) {
    const float qdd = gear * a - stiff * q - damp * qd - 2.0f * IA_SINF(q);
    const float st = stance(q);
    const float th_j = jl ? tc * st * fmaxf(-qd, 0.f) : 0.f;
    qd = qd + dt * qdd;
    float thrust = 0.f, lift = 0.f;
    for (int j = 0; j < nj; ++j) {
      thrust += bcast(th_j, j);
      lift += bcast(st, j);
    }
    const float vx = rv[0];
    rv[0] = vx + dt * (thrust - p.drag * vx * (1.0f + fabsf(vx)));
    if (p.nv_root > 1) rv[1] = rv[1] + dt * (-20.f * rq[1] - 4.f * rv[1] + 0.5f * (lift / (float)nj - 0.5f));
    if (p.nv_root > 2) rv[2] = rv[2] + dt * (-15.f * IA_SINF(rq[2]) - 3.f * rv[2] + pitch);
#pragma unroll
    for (int i = 3; i < 8; ++i)
      if (i < p.nv_root) rv[i] = rv[i] * (1.f - 2.f * dt) + dt * 0.1f * pitch;
    rq[0] += dt * rv[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) {
      if (i < p.nq_root) {
        if (i < p.nv_root) {  // (uniform branch) static register index: no select chain
          rq[i] += dt * rv[i] * 1.f;
        } else {  // free-joint quaternion slots (3D bodies only)
          const int vi = i % p.nv_root;
          float v = 0.f;
#pragma unroll
          for (int u = 0; u < 8; ++u) v = u == vi ? rv[u] : v;
          rq[i] += dt * v * 0.1f;
        }
      }
    }
    float qn = q + dt * qd;
    if (qn > 1.2f) { qn = 1.2f; if (qd > 0) qd = 0.f; }
    if (qn < -1.2f) { qn = -1.2f; if (qd < 0) qd = 0.f; }
    q = qn;
  }
  wave_sync();
  if (jl) {
    s[jq + lane] = q;
    s[nq + jv + lane] = qd;
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i < p.nq_root) s[i] = rq[i];
      if (i < p.nv_root) s[nq + i] = rv[i];
    }
  }
  wave_sync();
  const float dt_total = dt * p.frame_skip;
  return p.fwd_weight * (rq[0] - x_before) / dt_total + p.healthy_reward - p.ctrl_cost * ctrl;
}

// Observation of a locomotion state, one feature per lane.
__device__ float loco_obs_lane(const LocoParams& p, const float* s_gen) {
  const lf* s = (const lf*)s_gen;
  const int lane = threadIdx.x;
  const int nq = loco_nq(p), nv = loco_nv(p);
  const int npos = nq - p.obs_skip;
  if (lane < npos) return s[p.obs_skip + lane];
  if (lane < npos + nv) return s[nq + lane - npos];
  return 0.f;
}

__device__ __forceinline__ uint64_t hash3(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t s = a ^ (0x9E3779B97F4A7C15ull * (b + 1)) ^ (0xC2B2AE3D27D4EB4Full * (c + 1));
  splitmix64(s);
  return s;
}

__global__ __launch_bounds__(64) void rollout_kernel(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_raw[];
  lf* lds = (lf*)lds_raw;
  const int n = blockIdx.x;
  const int lane = threadIdx.x;
  const EnvParams& P = a.P;
  const int D = P.obs_dim;
  const int A = a.n_actions > 0 ? 1 : P.act_dim;
  const int S = state_size(P);
  LdsMLP pi, vf, rw;
  PairMLP pv;
  lf* p = lds;
  const bool paired = pair_ok(a.pi, a.vf);
  if (paired) p = load_pair(a.pi, a.vf, pv, p);
  p = load_mlp(a.pi, pi, p);
  p = load_mlp(a.vf, vf, p);
  if (a.rew_enabled) p = load_mlp(a.rew, rw, p);
  LdsMLP pt;
  if (a.rew_enabled && a.shaped) p = load_mlp(a.pot, pt, p);
  // env state / obs / action scratch stays a generic pointer: the shared host/device
  // env code (ia/envs.h) takes float*
  float* st = (float*)p;       // [kMaxState]
  float* ob = st + kMaxState;  // [kEngineMaxObs]
  float* act = ob + kEngineMaxObs;  // [kWaveMaxDim]
  for (int i = lane; i < S; i += 64) st[i] = a.state[(size_t)n * S + i];
  wave_sync();

  const LocoLane ll = P.kind == ENV_LOCO ? loco_lane(P.loco) : LocoLane{0.f, 0.f, 0.f, 0.f};
  float o = lane < D ? a.cur_obs[(size_t)n * D + lane] : 0.f;
  float start = a.cur_start[n];
  uint64_t rng = a.rng[n];
  int elapsed = a.elapsed[n];
  float ep_ret = a.ep_ret[n];
  const float lstd = (a.log_std && lane < A) ? a.log_std[lane] : 0.f;
  const float half_log2pi = 0.91893853320467274f;

  unsigned long long c_pol = 0, c_env = 0, c_rew = 0, c_all0 = clock64(), c0 = 0;
  for (int t = 0; t < a.T; ++t) {
    const size_t row = (size_t)t * a.N + n;
    c0 = clock64();
    if (lane < D) a.obs_buf[row * D + lane] = o;
    if (lane == 0) a.starts[row] = start;
    // ---- policy + value
    float head, value;
    if (paired) {
      const float out = pair_mlp(pv, o);
      head = out;
      value = bcast(out, 32);
    } else {
      head = wave_mlp(pi, o);
      value = bcast(wave_mlp(vf, o), 0);
    }
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
    if (a.explore_mode && a.explore_mode[t]) {  // ExplorationWrapper's random policy
      uint64_t s = key ^ 0x5851F42D4C957F2Dull;
      if (a.n_actions > 0) {
        s ^= 0x2545F4914F6CDD1Dull;
        const float u = uniform01(s);
        int k = (int)(u * (float)a.n_actions);
        k = k < a.n_actions ? k : a.n_actions - 1;
        a_raw = a_env = (float)k;
      } else {
        s ^= 0xD6E8FEB86659FD93ull * (lane + 1);
        const float u = uniform01(s);
        a_env = lane < A ? a.act_low[lane] + u * (a.act_high[lane] - a.act_low[lane]) : 0.f;
        a_raw = a_env;
      }
    }
    if (lane < A) {
      a.act_raw[row * A + lane] = a_raw;
      a.act_env[row * A + lane] = a_env;
      ((lf*)act)[lane] = a_env;
    }
    // ---- env step (lane 0), SB3 auto-reset + TimeLimit + Monitor
    c_pol += clock64() - c0;
    c0 = clock64();
    wave_sync();
    int term = 0;
    float r_env = 0.f;
    float o_next;  // terminal obs when done
    if (P.kind == ENV_LOCO) {
      r_env = loco_step_wave(P.loco, ll, st, act);
      o_next = loco_obs_lane(P.loco, st);
    } else {
      if (lane == 0) {
        r_env = env_step(P, st, act, &term, rng);
        env_obs(P, st, ob);
      }
      wave_sync();
      term = __builtin_amdgcn_readfirstlane(term);
      r_env = bcast(r_env, 0);
      o_next = lane < D ? ob[lane] : 0.f;
    }
    elapsed += 1;
    ep_ret += r_env;
    const bool trunc = !term && elapsed >= a.max_steps;
    const bool done = term || trunc;
    c_env += clock64() - c0;
    c0 = clock64();
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
      if (a.shaped) {  // AIRL potential shaping (reward_nets.py ShapedRewardNet.forward)
        const float phi_s = bcast(wave_mlp(pt, lane < D ? o : 0.f), 0);
        const float phi_n = done ? 0.f : bcast(wave_mlp(pt, lane < D ? o_next : 0.f), 0);
        r += a.shaping_gamma * phi_n - phi_s;
      }
    }
    c_rew += clock64() - c0;
    float bt = 0.f;
    if (trunc) {  // SB3: bootstrap the value of the truncated terminal obs into the reward
      bt = a.gamma * bcast(wave_mlp(vf, o_next), 0);
    }
    if (a.rew_raw && lane == 0) {
      a.rew_raw[row] = r;
      a.boot[row] = bt;
    }
    r += bt;
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
      wave_sync();
      if (lane == 0) {
        env_reset(P, st, rng);
        env_obs(P, st, ob);
      }
      wave_sync();
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
  wave_sync();
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
  if (a.prof && lane == 0) {
    a.prof[n * 4 + 0] = c_pol;
    a.prof[n * 4 + 1] = c_env;
    a.prof[n * 4 + 2] = c_rew;
    a.prof[n * 4 + 3] = clock64() - c_all0;
  }
}

int mlp_lds_floats(const WaveMLP& m) {
  int f = 0;
  for (int l = 0; l < m.n_layers; ++l) f += ceil8(m.dims[l]) * kW + kW;
  if (m.norm_mean) f += 2 * kW;
  return f;
}

}  // namespace

// NormalizedRewardNet output normalisation (see OutNormArgs): one wave, sequential in t.
__global__ __launch_bounds__(64) void reward_outnorm_kernel(OutNormArgs a) {
  const int lane = threadIdx.x;
  float mean = a.mean[0], var = a.var[0], cnt = a.count[0];
  for (int t = 0; t < a.T; ++t) {
    const float rstd = 1.f / sqrtf(var + a.eps);
    float s = 0.f;
    for (int n = lane; n < a.N; n += 64) {
      const size_t i = (size_t)t * a.N + n;
      const float x = a.rew_raw[i];
      a.rewards[i] = (x - mean) * rstd + a.boot[i];
      s += x;
    }
    float bm, bv, bn;
    if (a.step_stats) {
      bn = a.step_stats[3 * t];
      bm = a.step_stats[3 * t + 1];
      bv = a.step_stats[3 * t + 2];
    } else {
      bn = (float)a.N;
      bm = wave_sum(s) / bn;
      float q = 0.f;
      for (int n = lane; n < a.N; n += 64) {
        const float d = a.rew_raw[(size_t)t * a.N + n] - bm;
        q += d * d;
      }
      bv = wave_sum(q) / bn;
    }
    const float delta = bm - mean, tot = cnt + bn;
    mean += delta * bn / tot;
    var = (var * cnt + bv * bn + delta * delta * cnt * bn / tot) / tot;
    cnt = tot;
  }
  if (lane == 0) {
    a.mean[0] = mean;
    a.var[0] = var;
    a.count[0] = cnt;
  }
}

// Reward of many transitions: one wave per row, rows strided over the grid; the MLP
// images are staged in LDS once per workgroup. Same fp32 arithmetic (and input layout)
// as the in-rollout reward, so the result is bit-identical to it.
__global__ __launch_bounds__(64) void reward_batch_kernel(RewardBatchArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_raw[];
  lf* p = (lf*)lds_raw;
  const int lane = threadIdx.x;
  LdsMLP rw, pt;
  p = load_mlp(a.rew, rw, p);
  if (a.shaped) p = load_mlp(a.pot, pt, p);
  wave_sync();
  const int D = a.D, A = a.A;
  for (int row = blockIdx.x; row < a.rows; row += gridDim.x) {
    const size_t r64 = (size_t)row;
    const float o = lane < D ? a.obs[r64 * D + lane] : 0.f;
    const float o_next = lane < D ? a.next_obs[r64 * D + lane] : 0.f;
    const float a_env = lane < A ? a.acts[r64 * A + lane] : 0.f;
    const bool done = a.dones[r64] > 0.5f;
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
    if (a.use_done) { if (lane == off) x = done ? 1.f : 0.f; off += 1; }
    const float logit = bcast(wave_mlp(rw, x), 0);
    float r = a.rew_transform == REW_SOFTPLUS ? (logit > 0.f ? logit + log1pf(expf(-logit)) : log1pf(expf(logit))) : logit;
    if (a.shaped) {
      const float phi_s = bcast(wave_mlp(pt, o), 0);
      const float phi_n = done ? 0.f : bcast(wave_mlp(pt, o_next), 0);
      r += a.shaping_gamma * phi_n - phi_s;
    }
    if (lane == 0) {
      if (a.rew_raw) a.rew_raw[r64] = r;
      a.rewards[r64] = r + a.boot[r64];
    }
  }
}

size_t rollout_lds_bytes(const RolloutArgs& a) {
  int f = mlp_lds_floats(a.pi) + mlp_lds_floats(a.vf) + (a.rew_enabled ? mlp_lds_floats(a.rew) : 0);
  if (a.rew_enabled && a.shaped) f += mlp_lds_floats(a.pot);
  if (a.pi.n_layers == a.vf.n_layers) f += pair_lds_floats(a.pi, a.vf);  // paired image
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

hipError_t reward_batch_launch(const RewardBatchArgs& a, hipStream_t s) {
  if (a.rows <= 0) return hipSuccess;
  if (a.D > kEngineMaxObs || a.A > kWaveMaxDim) return hipErrorInvalidValue;
  const size_t lds = (size_t)(mlp_lds_floats(a.rew) + (a.shaped ? mlp_lds_floats(a.pot) : 0)) * sizeof(float);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int rows_per_wg = 4;  // ~4 workgroups per CU, their waves interleave on the SIMDs
  const int grid = (a.rows + rows_per_wg - 1) / rows_per_wg;
  hipLaunchKernelGGL(reward_batch_kernel, dim3(grid), dim3(64), lds, s, a);
  return hipGetLastError();
}

hipError_t reward_outnorm_launch(const OutNormArgs& a, hipStream_t s) {
  if (a.T <= 0 || a.N <= 0) return hipSuccess;
  hipLaunchKernelGGL(reward_outnorm_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace ia

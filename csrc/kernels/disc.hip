// Fused discriminator update for the device adversarial engine.
//
// The reference's AdversarialTrainer.train_disc (src/imitation/algorithms/adversarial/
// common.py:353-420 + _make_disc_train_batches :583-653) issues, per update, a demo-
// loader batch, a replay-buffer sample, four torch.cat, a full policy evaluate_actions
// (whose only lasting effect for GAIL is the RunningNorm update of the policy's
// features extractor), preprocess, the reward-net forward (RunningNorm update + MLP),
// BCE, autograd backward, Adam and ~8 host syncs for statistics -- ~120 launches.
// Here one update is four launches with no host sync:
//
//   disc_gather      X = [expert rows ; generator rows] gathered by index into the
//                    reward-net input layout (obs | act or one-hot | next_obs | done),
//                    plus per-block shifted column sums (S1, S2) for the batch moments
//   disc_norm        fixed-order reduction of the block sums -> batch mean / var (fp64),
//                    Chan merge into the reward net's RunningNorm and (GAIL side effect
//                    of the log-prob pass) the policy's RunningNorm over the obs columns
//   tmlp_disc_fwd_bwd  (tmlp.hip) forward recompute + BCE gradient + backward + loss stats
//   disc_adam        fixed-order reduction of the per-block gradient slab and of the
//                    stats slab, then torch.optim.Adam's exact update on the flat params
//
// Every reduction is in a fixed order: replicas are bitwise reproducible.
#include <hip/hip_runtime.h>

#include "launchers.h"

namespace ia {
namespace {

constexpr int kGatherRows = 64;  // rows per gather block (>= 256 blocks for a 16k batch)

__device__ __forceinline__ float load_act(const DiscGatherArgs& a, bool expert, int64_t src, int j, int aw) {
  if (a.act_discrete) {
    const int64_t* acts = expert ? a.e_acts_i : a.g_acts_i;
    return (int)acts[src] == j ? 1.f : 0.f;
  }
  const float* acts = expert ? a.e_acts : a.g_acts;
  return acts[src * aw + j];
}

// Value of column c of the reward-net input for source row src of the expert/gen set.
__device__ __forceinline__ float gather_col(const DiscGatherArgs& a, bool expert, int64_t src, int c) {
  const int D = a.obs_dim, aw = a.act_width;
  if (a.use_state) {
    if (c < D) return (expert ? a.e_obs : a.g_obs)[src * D + c];
    c -= D;
  }
  if (a.use_action) {
    if (c < aw) return load_act(a, expert, src, c, aw);
    c -= aw;
  }
  if (a.use_next_state) {
    if (c < D) return (expert ? a.e_next_obs : a.g_next_obs)[src * D + c];
    c -= D;
  }
  return (expert ? a.e_dones : a.g_dones)[src] ? 1.f : 0.f;
}

// Block: 256 threads = 2 row phases x 128 columns; rows [blk*64, blk*64+64).
__global__ __launch_bounds__(256) void disc_gather_kernel(DiscGatherArgs a) {
  __shared__ float red[2][2][128];
  const int c = threadIdx.x & 127, ph = threadIdx.x >> 7;
  const int n = 2 * a.mb;
  const int r0 = blockIdx.x * kGatherRows;
  const bool col_ok = c < a.din;
  const float shift = col_ok && a.shift ? a.shift[c] : 0.f;
  float s1 = 0.f, s2 = 0.f;
  if (col_ok) {
    for (int rr = ph; rr < kGatherRows; rr += 2) {
      const int r = r0 + rr;
      if (r >= n) break;
      const bool expert = r < a.mb;
      const int64_t src = expert ? a.e_idx[r] : a.g_idx[r - a.mb];
      const float v = gather_col(a, expert, src, c);
      a.X[(size_t)r * a.din + c] = v;
      const float dv = v - shift;
      s1 += dv;
      s2 += dv * dv;
    }
  }
  red[ph][0][c] = s1;
  red[ph][1][c] = s2;
  __syncthreads();
  if (ph == 0 && col_ok) {
    float* out = a.partials + (size_t)blockIdx.x * 2 * a.din;
    out[c] = red[0][0][c] + red[1][0][c];
    out[a.din + c] = red[0][1][c] + red[1][1][c];
  }
}

__device__ __forceinline__ void chan_merge(float* rmean, float* rvar, int count, int c, float bmean, float bvar, int n) {
  // RunningNorm.update_stats (networks.py:94-111) in the same operation order (fp32)
  const float fc = (float)count, fn = (float)n, tot = (float)(count + n);
  const float delta = bmean - rmean[c];
  rmean[c] += delta * fn / tot;
  float v = rvar[c] * fc;
  v += bvar * fn;
  v += delta * delta * fc * fn / tot;
  rvar[c] = v / tot;
}

// 1024 threads = 8 block-phases x 128 columns: phase p sums partial blocks p, p+8, ... in
// order, then the 8 phase sums are added in phase order (fixed order: deterministic).
constexpr int kNormPhases = 8;

__global__ __launch_bounds__(128 * kNormPhases) void disc_norm_kernel(DiscNormArgs a) {
  __shared__ double red[kNormPhases][2][128];
  const int c = threadIdx.x & 127, ph = threadIdx.x >> 7;
  const int n = a.mode == 2 ? a.n_total : 2 * a.mb;
  const int rc = a.rew_count ? *a.rew_count : 0;
  const int pc = a.pol_count ? *a.pol_count : 0;
  if (a.mode != 2) {
    double s1 = 0.0, s2 = 0.0;
    if (c < a.din)
      for (int b = ph; b < a.nblk; b += kNormPhases) {
        const float* p = a.partials + (size_t)b * 2 * a.din;
        s1 += (double)p[c];
        s2 += (double)p[a.din + c];
      }
    red[ph][0][c] = s1;
    red[ph][1][c] = s2;
    __syncthreads();
  }
  if (ph == 0 && c < a.din) {
    double S1 = 0.0, S2 = 0.0;
    if (a.mode == 2) {
      S1 = a.sums[c];
      S2 = a.sums[a.din + c];
    } else {
      for (int q = 0; q < kNormPhases; ++q) {
        S1 += red[q][0][c];
        S2 += red[q][1][c];
      }
    }
    if (a.mode == 1) {
      a.sums[c] = S1;
      a.sums[a.din + c] = S2;
    } else {
      const double shift = a.shift ? (double)a.shift[c] : 0.0;
      const double m = S1 / n;
      double var = S2 / n - m * m;
      if (var < 0.0) var = 0.0;
      const float bmean = (float)(shift + m), bvar = (float)var;
      if (a.rew_mean) chan_merge(a.rew_mean, a.rew_var, rc, c, bmean, bvar, n);
      if (a.pol_defer && c < a.pol_cols) {
        a.pol_defer[c] = bmean;
        a.pol_defer[a.pol_cols + c] = bvar;
        if (c == 0) a.pol_defer[2 * a.pol_cols] = (float)n;
      } else if (a.pol_mean && c < a.pol_cols) {
        chan_merge(a.pol_mean, a.pol_var, pc, c, bmean, bvar, n);
      }
    }
  }
  if (a.mode == 1) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.rew_count) *a.rew_count = rc + n;
    if (a.pol_count && !a.pol_defer) *a.pol_count = pc + n;
  }
}

// One thread per column; slots merged in order (the policy RunningNorm side effect of
// the discriminator batches, deferred so that those updates can run concurrently with
// the PPO update that also merges into this norm).
__global__ __launch_bounds__(128) void pol_norm_merge_kernel(float* mean, float* var, int* count, const float* defer,
                                                             int n_slots, int cols) {
  const int c = threadIdx.x;
  int cnt = *count;
  for (int k = 0; k < n_slots; ++k) {
    const float* d = defer + (size_t)k * (2 * cols + 1);
    const int n = (int)d[2 * cols];
    if (c < cols) chan_merge(mean, var, cnt, c, d[c], d[cols + c], n);
    cnt += n;
  }
  __syncthreads();
  if (c == 0) *count = cnt;
}

// grid: ceil(n_params / 64) blocks of 1024 = 16 block-phases x 64 params (fixed-order
// reduction of the gradient slab: phase q sums slab blocks q, q+16, ...; phases in order).
constexpr int kAdamPhases = 16;

__global__ __launch_bounds__(64 * kAdamPhases) void disc_adam_kernel(DiscAdamArgs a) {
  __shared__ float red[kAdamPhases][64];
  __shared__ float sred[kAdamPhases][kDiscStats];
  const int pl = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + pl;
  float s = 0.f;
  if (a.reduce && e < a.n_params)
    for (int b = ph; b < a.nblk; b += kAdamPhases) s += a.slab[(size_t)b * a.n_params + e];
  red[ph][pl] = s;
  // loss statistics of this (last) minibatch: block 0, lanes 0..kDiscStats-1 of every phase
  const bool do_stats = a.reduce && blockIdx.x == 0 && a.stats_out;
  if (do_stats && pl < kDiscStats) {
    float t = 0.f;
    for (int b = ph; b < a.stats_nblk; b += kAdamPhases) t += a.stats_slab[(size_t)b * kDiscStats + pl];
    sred[ph][pl] = t;
  }
  __syncthreads();
  if (do_stats && threadIdx.x < kDiscStats) {
    float t = 0.f;
    for (int q = 0; q < kAdamPhases; ++q) t += sred[q][threadIdx.x];
    a.stats_out[threadIdx.x] = (a.stats_scale != 0.f ? a.stats_scale : 1.f) * t;
  }
  if (ph == 0 && e < a.n_params) {
    float acc = 0.f;
    for (int q = 0; q < kAdamPhases; ++q) acc += red[q][pl];
    red[0][pl] = acc;
  }
  if (ph != 0 || e >= a.n_params) return;
  float g;
  if (a.reduce) {
    g = red[0][pl];
    if (!a.adam) {
      a.grads[e] = g;
      return;
    }
  } else {
    g = a.grads[e];
  }
  float p = a.params[e];
  float step_size = a.step_size, bc2_sqrt = a.bc2_sqrt;
  if (a.step) {  // bias corrections from the device step counter (torch: lr / bc1, sqrt(bc2))
    const float t = *a.step;
    step_size = a.lr / (1.f - powf(a.beta1, t));
    bc2_sqrt = sqrtf(1.f - powf(a.beta2, t));
  }
  if (a.weight_decay != 0.f) {
    if (a.decoupled) p *= 1.f - a.lr * a.weight_decay;  // AdamW
    else g += a.weight_decay * p;
  }
  // torch.optim.Adam (_single_tensor/_multi_tensor, non-capturable): lerp, addcmul,
  // denom = sqrt(v) / sqrt(bc2) + eps, p -= lr / bc1 * m / denom
  float m = a.exp_avg[e];
  m += (1.f - a.beta1) * (g - m);
  float v = a.exp_avg_sq[e] * a.beta2 + (1.f - a.beta2) * g * g;
  a.exp_avg[e] = m;
  a.exp_avg_sq[e] = v;
  const float denom = sqrtf(v) / bc2_sqrt + a.eps;
  a.params[e] = p - step_size * (m / denom);
}

}  // namespace

int disc_gather_blocks(int mb) { return (2 * mb + kGatherRows - 1) / kGatherRows; }

hipError_t disc_gather(const DiscGatherArgs& a, hipStream_t s) {
  if (a.din > 128 || a.din <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(disc_gather_kernel, dim3(disc_gather_blocks(a.mb)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t disc_norm(const DiscNormArgs& a, hipStream_t s) {
  if (a.din > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(disc_norm_kernel, dim3(1), dim3(128 * kNormPhases), 0, s, a);
  return hipGetLastError();
}

hipError_t pol_norm_merge(float* mean, float* var, int* count, const float* defer, int n_slots, int cols,
                          hipStream_t s) {
  if (n_slots <= 0) return hipSuccess;
  if (cols > 128 || cols <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pol_norm_merge_kernel, dim3(1), dim3(128), 0, s, mean, var, count, defer, n_slots, cols);
  return hipGetLastError();
}

hipError_t disc_adam(const DiscAdamArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(disc_adam_kernel, dim3((a.n_params + 63) / 64), dim3(64 * kAdamPhases), 0, s, a);
  return hipGetLastError();
}

}  // namespace ia

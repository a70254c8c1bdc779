// RunningNorm / EMANorm (reference util/networks.py:80-201) update + normalise in
// ONE launch (EMANorm: same batch moments, exponential-moving-average merge).
//
// In training mode every RunningNorm forward merges the batch moments into the running
// statistics (Chan et al.) and then normalises: in torch that is mean, var, ~12 elementwise
// updates of the [D] statistics and the count, then (x - mean) / sqrt(var + eps) -- ~20
// launches of a few microseconds per norm layer, 3-4 layers per AIRL discriminator step.
// Here one workgroup: the batch mean and centred variance reduced in a fixed order through
// LDS (deterministic), the running mean / var updated with the same formulas as the module,
// the count advanced once, and the batch normalised with the updated statistics. Sized for the small-MLP batches of
// this framework (B * D <= 2^20); larger or data-parallel batches keep the torch path.
#include <hip/hip_runtime.h>
#include <math.h>

#include "launchers.h"

namespace ia {
namespace {

// EMANorm state (networks.py EMANorm.update_stats): the learning rate of this update is
// 1 / (inv_lr + decay^num_batches); null -> RunningNorm's Chan merge.
struct EmaState {
  float* inv_lr;
  int* num_batches;
  float decay;
};

__device__ __forceinline__ float ema_lr(const EmaState& e) {
  return 1.f / (e.inv_lr[0] + powf(e.decay, (float)e.num_batches[0]));
}

// merge one feature's batch moments (mean bm, biased var bv over bc rows) into the running
// statistics: Chan (RunningNorm) or the exponential moving average (EMANorm)
__device__ __forceinline__ void merge_stats(float* mean, float* var, int ff, float bm, float bv, float bc, float n_old,
                                            bool ema, float lr) {
  const float rm = mean[ff], rv = var[ff];
  const float delta = bm - rm;
  if (ema) {
    mean[ff] = rm + lr * delta;
    var[ff] = rv + lr * (bv + (1.f - lr) * delta * delta - rv);
  } else {
    const float tot = n_old + bc;
    mean[ff] = rm + delta * bc / tot;
    var[ff] = (rv * n_old + bv * bc + delta * delta * n_old * bc / tot) / tot;
  }
}

// count (+ the EMA's inverse learning rate and batch counter) after every lane merged
__device__ __forceinline__ void advance_counts(int* count, int B, const EmaState& e, bool ema) {
  count[0] = count[0] + B;
  if (ema) {
    e.inv_lr[0] = e.inv_lr[0] + powf(e.decay, (float)e.num_batches[0]);
    e.num_batches[0] = e.num_batches[0] + 1;
  }
}

// One workgroup. Features are processed 64 (or fewer: Dp = next power of two >= D) at a time
// with 256 / Dp row groups per feature, so a narrow batch (the reward output norm: D = 1,
// thousands of rows) still uses all 256 lanes. Two passes over the rows (sum -> mean, then
// the centred sum of squares), partials reduced across the groups in a fixed order.
__global__ __launch_bounds__(256) void running_norm_kernel(const float* __restrict__ x, int B, int D,
                                                           float* __restrict__ mean, float* __restrict__ var,
                                                           int* __restrict__ count, float eps, int update,
                                                           float* __restrict__ y, EmaState ema_st) {
  __shared__ float red[256];
  __shared__ float s_mean[256], s_rstd[256];
  const int tid = threadIdx.x;
  const bool ema = ema_st.inv_lr != nullptr;
  const float lr = (update && ema) ? ema_lr(ema_st) : 0.f;
  int Dp = 1;
  while (Dp < D && Dp < 64) Dp <<= 1;
  const int G = 256 / Dp, f = tid % Dp, g = tid / Dp;
  const float n_old = update ? (float)count[0] : 0.f;
  for (int f0 = 0; f0 < D; f0 += Dp) {
    const int ff = f0 + f;
    if (update) {
      float sum = 0.f;
      if (ff < D) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int r = g;
        for (; r + 7 * G < B; r += 8 * G) {  // 8 independent loads in flight
#pragma unroll
          for (int u = 0; u < 8; ++u) acc[u] += x[(size_t)(r + u * G) * D + ff];
        }
        for (; r < B; r += G) acc[0] += x[(size_t)r * D + ff];
        sum = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
      }
      red[tid] = sum;
      __syncthreads();
      if (g == 0) {
        float t = 0.f;
        for (int q = 0; q < G; ++q) t += red[q * Dp + f];
        s_mean[f] = t / (float)B;  // batch mean (scratch until the merge below)
      }
      __syncthreads();
      const float bm = s_mean[f];
      float sq = 0.f;
      if (ff < D) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int r = g;
        for (; r + 7 * G < B; r += 8 * G) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float d = x[(size_t)(r + u * G) * D + ff] - bm;
            acc[u] += d * d;
          }
        }
        for (; r < B; r += G) {
          const float d = x[(size_t)r * D + ff] - bm;
          acc[0] += d * d;
        }
        sq = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
      }
      __syncthreads();
      red[tid] = sq;
      __syncthreads();
      if (g == 0 && ff < D) {
        float t = 0.f;
        for (int q = 0; q < G; ++q) t += red[q * Dp + f];
        merge_stats(mean, var, ff, bm, t / (float)B, (float)B, n_old, ema, lr);
      }
      __syncthreads();
    }
  }
  __syncthreads();
  for (int ff = tid; ff < D; ff += 256) {
    s_mean[ff] = mean[ff];
    s_rstd[ff] = 1.f / sqrtf(var[ff] + eps);
  }
  __syncthreads();
  if (update && tid == 0) advance_counts(count, B, ema_st, ema);
  if (!y) return;
  const int total = B * D;
  for (int i = tid; i < total; i += 256) {
    const int ff = i % D;
    y[i] = (x[i] - s_mean[ff]) * s_rstd[ff];
  }
}

// ---- multi-workgroup path (large batches): the single-workgroup kernel walks B rows with
// 256 lanes (27 us for AIRL's 4096 x 14 discriminator batch, 4 per update); here
//   A: nb workgroups, each the exact two-pass (mean, centred M2) of its own row slice,
//   B: one workgroup Chan-merges the nb partials in block order (deterministic) and applies
//      the module's running-statistics merge + count update,
//   C: (training forward) nb workgroups normalise their slices with the updated statistics.
constexpr int kNormRowsPerBlock = 256;
constexpr int kNormMaxBlocks = 128;

__global__ __launch_bounds__(256) void running_norm_partial_kernel(const float* __restrict__ x, int B, int D, int rpb,
                                                                   float* __restrict__ part) {
  __shared__ float red[256];
  __shared__ float s_m[64];
  const int tid = threadIdx.x, b = blockIdx.x;
  const int r0 = b * rpb, r1 = min(B, r0 + rpb), nr = r1 - r0;
  int Dp = 1;
  while (Dp < D && Dp < 64) Dp <<= 1;
  const int G = 256 / Dp, f = tid % Dp, g = tid / Dp;
  for (int f0 = 0; f0 < D; f0 += Dp) {
    const int ff = f0 + f;
    float acc = 0.f;
    if (ff < D) {
#pragma unroll 4
      for (int r = r0 + g; r < r1; r += G) acc += x[(size_t)r * D + ff];
    }
    red[tid] = acc;
    __syncthreads();
    if (g == 0) {
      float t = 0.f;
      for (int q = 0; q < G; ++q) t += red[q * Dp + f];
      s_m[f] = t / (float)nr;
    }
    __syncthreads();
    const float bm = s_m[f];
    float sq = 0.f;
    if (ff < D) {
#pragma unroll 4
      for (int r = r0 + g; r < r1; r += G) {
        const float d = x[(size_t)r * D + ff] - bm;
        sq += d * d;
      }
    }
    __syncthreads();
    red[tid] = sq;
    __syncthreads();
    if (g == 0 && ff < D) {
      float t = 0.f;
      for (int q = 0; q < G; ++q) t += red[q * Dp + f];
      part[(size_t)b * 2 * D + ff] = bm;
      part[(size_t)b * 2 * D + D + ff] = t;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void running_norm_merge_kernel(const float* __restrict__ part, int nb, int rpb, int B,
                                                                 int D, float* __restrict__ mean, float* __restrict__ var,
                                                                 int* __restrict__ count, EmaState ema_st) {
  // the partials of a feature chunk are staged in LDS by all lanes at once (the serial merge
  // chain then reads LDS, not dependent global loads)
  __shared__ float sp[8192];
  const float n_old = (float)count[0];
  const bool ema = ema_st.inv_lr != nullptr;
  const float lr = ema ? ema_lr(ema_st) : 0.f;
  const int fc = min(D, (int)(8192 / (2 * nb)));
  for (int f0 = 0; f0 < D; f0 += fc) {
    const int nf = min(fc, D - f0);
    __syncthreads();
    for (int i = threadIdx.x; i < nb * 2 * nf; i += 256) {
      const int b = i / (2 * nf), j = i % (2 * nf);
      const int col = j < nf ? f0 + j : D + f0 + (j - nf);
      sp[i] = part[(size_t)b * 2 * D + col];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nf; k += 256) {
      float n = 0.f, m = 0.f, m2 = 0.f;
      for (int b = 0; b < nb; ++b) {  // Chan merge in block order
        const float nbf = (float)min(rpb, B - b * rpb);
        const float mb = sp[b * 2 * nf + k], m2b = sp[b * 2 * nf + nf + k];
        const float delta = mb - m, nn = n + nbf;
        m += delta * nbf / nn;
        m2 += m2b + delta * delta * n * nbf / nn;
        n = nn;
      }
      merge_stats(mean, var, f0 + k, m, m2 / (float)B, (float)B, n_old, ema, lr);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) advance_counts(count, B, ema_st, ema);
}

__global__ __launch_bounds__(256) void running_norm_apply_kernel(const float* __restrict__ x, int B, int D, int rpb,
                                                                 const float* __restrict__ mean,
                                                                 const float* __restrict__ var, float eps,
                                                                 float* __restrict__ y) {
  const size_t i0 = (size_t)blockIdx.x * rpb * D, i1 = min((size_t)B * D, i0 + (size_t)rpb * D);
  for (size_t i = i0 + threadIdx.x; i < i1; i += 256) {
    const int ff = (int)(i % D);
    y[i] = (x[i] - mean[ff]) * (1.f / sqrtf(var[ff] + eps));
  }
}

}  // namespace

bool running_norm_ok(int B, int D) { return B > 0 && D > 0 && D <= 256 && (long)B * D <= (1l << 20); }

int running_norm_blocks(int B) {
  if (B < 4 * kNormRowsPerBlock) return 1;  // small batches: the single-workgroup kernel
  int rpb = kNormRowsPerBlock;
  while ((B + rpb - 1) / rpb > kNormMaxBlocks) rpb *= 2;
  return (B + rpb - 1) / rpb;
}

size_t running_norm_ws_floats(int B, int D) {
  const int nb = running_norm_blocks(B);
  return nb > 1 ? (size_t)nb * 2 * D : 0;
}

hipError_t running_norm(const float* x, int B, int D, float* mean, float* var, int* count, float eps, int update, float* y,
                        float* ws, hipStream_t s, float* ema_inv_lr, int* ema_num_batches, float ema_decay) {
  if (!running_norm_ok(B, D)) return hipErrorInvalidValue;
  if ((ema_inv_lr == nullptr) != (ema_num_batches == nullptr)) return hipErrorInvalidValue;
  const EmaState ema{ema_inv_lr, ema_num_batches, ema_decay};
  const int nb = running_norm_blocks(B);
  if (nb <= 1 || !update || !ws) {
    hipLaunchKernelGGL(running_norm_kernel, dim3(1), dim3(256), 0, s, x, B, D, mean, var, count, eps, update, y, ema);
    return hipGetLastError();
  }
  const int rpb = (B + nb - 1) / nb;
  hipLaunchKernelGGL(running_norm_partial_kernel, dim3(nb), dim3(256), 0, s, x, B, D, rpb, ws);
  hipLaunchKernelGGL(running_norm_merge_kernel, dim3(1), dim3(256), 0, s, ws, nb, rpb, B, D, mean, var, count, ema);
  if (y) hipLaunchKernelGGL(running_norm_apply_kernel, dim3(nb), dim3(256), 0, s, x, B, D, rpb, mean, var, eps, y);
  return hipGetLastError();
}

}  // namespace ia

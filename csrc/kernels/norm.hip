// RunningNorm (reference util/networks.py:80-134) update + normalise in ONE launch.
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

// One workgroup. Features are processed 64 (or fewer: Dp = next power of two >= D) at a time
// with 256 / Dp row groups per feature, so a narrow batch (the reward output norm: D = 1,
// thousands of rows) still uses all 256 lanes. Two passes over the rows (sum -> mean, then
// the centred sum of squares), partials reduced across the groups in a fixed order.
__global__ __launch_bounds__(256) void running_norm_kernel(const float* __restrict__ x, int B, int D,
                                                           float* __restrict__ mean, float* __restrict__ var,
                                                           int* __restrict__ count, float eps, int update,
                                                           float* __restrict__ y) {
  __shared__ float red[256];
  __shared__ float s_mean[256], s_rstd[256];
  const int tid = threadIdx.x;
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
        const float bv = t / (float)B, bc = (float)B;
        const float rm = mean[ff], rv = var[ff];
        const float delta = bm - rm, tot = n_old + bc;
        mean[ff] = rm + delta * bc / tot;
        var[ff] = (rv * n_old + bv * bc + delta * delta * n_old * bc / tot) / tot;
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
  if (update && tid == 0) count[0] = count[0] + B;
  if (!y) return;
  const int total = B * D;
  for (int i = tid; i < total; i += 256) {
    const int ff = i % D;
    y[i] = (x[i] - s_mean[ff]) * s_rstd[ff];
  }
}

}  // namespace

bool running_norm_ok(int B, int D) { return B > 0 && D > 0 && D <= 256 && (long)B * D <= (1l << 20); }

hipError_t running_norm(const float* x, int B, int D, float* mean, float* var, int* count, float eps, int update, float* y,
                        hipStream_t s) {
  if (!running_norm_ok(B, D)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(running_norm_kernel, dim3(1), dim3(256), 0, s, x, B, D, mean, var, count, eps, update, y);
  return hipGetLastError();
}

}  // namespace ia

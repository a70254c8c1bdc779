// Bradley-Terry preference loss over fragment pairs (reference
// PreferenceModel.probability + CrossEntropyRewardLoss,
// src/imitation/algorithms/preference_comparisons.py:487-530, 1070-1090).
//
// The reference loops over pairs in Python: per pair, two reward-net calls and a
// handful of scalar torch ops. Here the reward net runs ONCE over all 2*P*L
// fragment transitions and this kernel does the rest for all pairs in one launch:
//   diff_i = sum_t g^t (r2[i,t] - r1[i,t])   (one wave per pair, wave-shuffle sum)
//   p_i    = noise/2 + (1-noise) / (1 + exp(clip(diff_i, +-thr)))
//   loss_i = BCE(p_i, y_i)  (log clamped at -100 like torch)
//   c_i    = dloss_i/ddiff_i  (saved for the backward kernel)
// Backward: dr2[i,t] = gout * c_i * g^t / P, dr1 = -dr2 (elementwise, one thread per entry).
#include <hip/hip_runtime.h>

#include "launchers.h"

namespace ia {
namespace {

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(256) void pref_fwd_kernel(const float* __restrict__ r1, const float* __restrict__ r2,
                                                       const float* __restrict__ prefs, int P, int L, float discount,
                                                       float threshold, float noise, float* __restrict__ probs,
                                                       float* __restrict__ losses, float* __restrict__ coef) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (i >= P) return;  // whole wave exits together
  const float* a = r1 + (size_t)i * L;
  const float* b = r2 + (size_t)i * L;
  float s = 0.f;
  if (discount == 1.f) {
    for (int t = lane; t < L; t += 64) s += b[t] - a[t];
  } else {
    const float lg = __log2f(discount);
    for (int t = lane; t < L; t += 64) s += exp2f(lg * (float)t) * (b[t] - a[t]);
  }
  const float diff = wave_sum(s);
  if (lane == 0) {
    const bool inside = diff >= -threshold && diff <= threshold;
    const float d = fminf(fmaxf(diff, -threshold), threshold);
    const float ed = expf(d);
    const float pm = 1.f / (1.f + ed);
    const float p = noise * 0.5f + (1.f - noise) * pm;
    const float y = prefs[i];
    const float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(logf(1.f - p), -100.f);
    losses[i] = -(y * lp + (1.f - y) * l1p);
    probs[i] = p;
    // noise == 0: dloss/ddiff = y - pm exactly. torch's BCE backward, (p - y) / max(p (1 - p), 1e-12)
    // times dp/ddiff, agrees with this while p stays away from 0/1 and is noise once it
    // saturates (1 - p rounds to 0 in fp32 past |diff| ~ 17; the 1e-12 clamp past ~ 27).
    // noise > 0 keeps p inside [noise/2, 1 - noise/2], where the chain rule is well conditioned;
    // dpm/ddiff = -pm^2 e^d avoids the cancellation in pm (1 - pm).
    float c;
    if (noise == 0.f) {
      c = y - pm;
    } else {
      const float dl_dp = (p - y) / fmaxf(p * (1.f - p), 1e-12f);
      c = dl_dp * ((1.f - noise) * -(pm * pm) * ed);
    }
    coef[i] = inside ? c : 0.f;
  }
}

__global__ __launch_bounds__(256) void pref_bwd_kernel(const float* __restrict__ coef, const float* __restrict__ gout,
                                                       int P, int L, float discount, float* __restrict__ d1,
                                                       float* __restrict__ d2) {
  const size_t n = (size_t)P * L;
  const float g = gout[0] / (float)P;
  const float lg = discount == 1.f ? 0.f : __log2f(discount);
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / L), t = (int)(e - (size_t)i * L);
    const float w = discount == 1.f ? 1.f : exp2f(lg * (float)t);
    const float v = g * coef[i] * w;
    d2[e] = v;
    d1[e] = -v;
  }
}

}  // namespace

hipError_t pref_loss_fwd(const float* r1, const float* r2, const float* prefs, int P, int L, float discount,
                         float threshold, float noise, float* probs, float* losses, float* coef, hipStream_t s) {
  if (P <= 0) return hipSuccess;
  const int waves_per_block = 4;
  hipLaunchKernelGGL(pref_fwd_kernel, dim3((P + waves_per_block - 1) / waves_per_block), dim3(64 * waves_per_block), 0, s,
                     r1, r2, prefs, P, L, discount, threshold, noise, probs, losses, coef);
  return hipGetLastError();
}

hipError_t pref_loss_bwd(const float* coef, const float* gout, int P, int L, float discount, float* d1, float* d2,
                         hipStream_t s) {
  const size_t n = (size_t)P * L;
  if (n == 0) return hipSuccess;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(pref_bwd_kernel, dim3(blocks), dim3(256), 0, s, coef, gout, P, L, discount, d1, d2);
  return hipGetLastError();
}

}  // namespace ia

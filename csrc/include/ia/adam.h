// One Adam / AdamW element update, shared by every kernel that applies the optimizer step:
// the flat-bucket launch (optim.hip adam_flat) and the BC step's fused epilogues (cnn_fc.hip
// fc_wgrad + Adam, conv.hip conv_reduce_adam). One definition = the same float operations in
// the same order everywhere, so a fused step is bitwise the separate adam_flat launch.
#pragma once
#include <hip/hip_runtime.h>

#include "ia/common.h"

namespace ia {

// bias corrections of step t (1-based): step_size = lr / (1 - b1^t), bc2_sqrt = sqrt(1 - b2^t)
__device__ __forceinline__ void adam_scalars(float t, float lr, float beta1, float beta2, float& step_size, float& bc2_sqrt) {
  const float bc1 = 1.f - powf(beta1, t);
  bc2_sqrt = sqrtf(1.f - powf(beta2, t));
  step_size = lr / bc1;
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, float lr, float beta1, float beta2, float eps,
                                          float weight_decay, int decoupled, int maximize, float step_size, float bc2_sqrt) {
  float gr = maximize ? -g : g;
  if (weight_decay != 0.f) {
    if (decoupled) p *= 1.f - lr * weight_decay;
    else gr += weight_decay * p;
  }
  m += (1.f - beta1) * (gr - m);
  v = v * beta2 + (1.f - beta2) * gr * gr;
  const float denom = sqrtf(v) / bc2_sqrt + eps;
  p -= step_size * (m / denom);
}

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamHyper& h, float step_size,
                                          float bc2_sqrt) {
  adam_elem(p, g, m, v, h.lr, h.beta1, h.beta2, h.eps, h.weight_decay, h.decoupled, h.maximize, step_size, bc2_sqrt);
}

}  // namespace ia

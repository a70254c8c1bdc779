// The fixed-order sum of a conv layer's weight-gradient block partials (slab column i), as device
// functions shared by conv_reduce(_multi) (conv.hip) and the Adam launch that folds the BC step's
// reductions into its own blocks (optim.hip): the same sums, so the two paths are bitwise equal.
#pragma once
#include <hip/hip_runtime.h>

#include "launchers.h"

namespace ia {

// The 4 fixed-order accumulators of a slab column (accumulator j: blocks b = j mod 4 in order,
// the tail blocks into s0). 16 loads are issued before their adds: the slabs of a BC step have
// ~50 blocks, and 4 loads per round trip made the sum a chain of ~13 L2 round trips.
__device__ __forceinline__ void slab_sum4(const float* __restrict__ slab, int nblk, int len, int i, float& s0, float& s1,
                                          float& s2, float& s3) {
  s0 = s1 = s2 = s3 = 0.f;
  int b = 0;
  for (; b + 15 < nblk; b += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = slab[(size_t)(b + u) * len + i];
#pragma unroll
    for (int u = 0; u < 16; u += 4) {
      s0 += v[u];
      s1 += v[u + 1];
      s2 += v[u + 2];
      s3 += v[u + 3];
    }
  }
  for (; b + 3 < nblk; b += 4) {
    s0 += slab[(size_t)b * len + i];
    s1 += slab[(size_t)(b + 1) * len + i];
    s2 += slab[(size_t)(b + 2) * len + i];
    s3 += slab[(size_t)(b + 3) * len + i];
  }
  for (; b < nblk; ++b) s0 += slab[(size_t)b * len + i];
}

// Slab column i of layer geometry g (i < N * Kp + N): its fixed-order sum, and where it lands --
// *w_idx the torch [N][C][KH][KW] index of a weight column (-1: a zero-padding column of Kp, or a
// bias column), *b_idx the bias index (-1: a weight / padding column).
__device__ __forceinline__ float slab_column(const float* __restrict__ slab, int nblk, const ConvGeo& g, int i, int* w_idx,
                                             int* b_idx) {
  const int len = g.N * g.Kp + g.N;
  float s0, s1, s2, s3;
  slab_sum4(slab, nblk, len, i, s0, s1, s2, s3);
  *w_idx = -1;
  *b_idx = -1;
  const int nk = g.N * g.Kp;
  if (i < nk) {
    const int n = i / g.Kp, k = i - n * g.Kp;
    const int taps = g.KH * g.KW;
    if (k < taps * g.C) {
      const int tap = k / g.C, c = k - tap * g.C;
      *w_idx = (n * g.C + c) * taps + tap;
    }
  } else {
    *b_idx = i - nk;
  }
  return (s0 + s1) + (s2 + s3);
}

}  // namespace ia

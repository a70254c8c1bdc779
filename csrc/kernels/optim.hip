// Fused Adam / AdamW over one flat fp32 parameter buffer (imitation_amd/ops/optim.py).
//
// torch.optim.Adam(capturable, foreach) spends ~8 multi-tensor launches per step on a
// model's parameter list (BC on NatureCNN: ~110 us of a ~1 ms graphed minibatch); the
// reference optimisers are th.optim.Adam (bc.py:284, common.py:123) and AdamW
// (preference_comparisons.py:1192). Here every parameter of a group lives in one
// contiguous buffer, so a step is ONE elementwise launch: 4 floats per thread, the
// bias corrections from the device step counter (graph-capturable), and the gradient
// slot cleared in the same pass (the next backward accumulates into a zeroed bucket).
#include <hip/hip_runtime.h>

#include "launchers.h"
#include "wgrad_reduce.h"

namespace ia {
namespace {

// FMA contraction off, the fused multiply-adds spelled out: the float4 path, the scalar tail and the
// folded-reduction blocks (one element per thread) then compute bitwise the same update (with
// contraction left to the compiler, the packed float4 code formed other FMAs than the scalar code).
__device__ __forceinline__ void adam_one(float& p, float& g, float& m, float& v, const AdamArgs& a, float step_size,
                                         float bc2_sqrt) {
#pragma clang fp contract(off)
  float gr = a.maximize ? -g : g;
  if (a.weight_decay != 0.f) {
    if (a.decoupled) p *= 1.f - a.lr * a.weight_decay;
    else gr = __builtin_fmaf(a.weight_decay, p, gr);
  }
  m = __builtin_fmaf(1.f - a.beta1, gr - m, m);
  v = __builtin_fmaf(v, a.beta2, ((1.f - a.beta2) * gr) * gr);
  const float denom = sqrtf(v) / bc2_sqrt + a.eps;
  p = __builtin_fmaf(-step_size, m / denom, p);
  if (a.zero_grad) g = 0.f;
}

// The folded reductions: per layer its weight and bias slot ranges in the flat buffer, and the
// block range that sums its slab columns.
struct AdamRed {
  ConvReduceMulti r;
  int64_t w_off[kMaxPack], b_off[kMaxPack];  // flat offsets of the dW / db slots
  int64_t lo[2 * kMaxPack], hi[2 * kMaxPack];  // the slot ranges (multiples of 4): the quads the
  int nr;                                      // elementwise blocks skip
  int ncol;                                    // blocks [0, ncol) the layers' column blocks
  int boff[kMaxPack + 1];                      // ([boff[l], boff[l + 1]) of layer l), then the
                                               // elementwise blocks: their chains of slab loads
                                               // start first and overlap the elementwise part
};

template <bool RED>
__global__ __launch_bounds__(256) void adam_flat_kernel(AdamArgs a, AdamRed rd) {
  // the bias corrections once per block (two powf per thread were ~100 VALU each); same values
  __shared__ float bcs[3];
  if (threadIdx.x == 0) {
    const float t0 = *a.step + (a.cnt ? 1.f : 0.f);
    bcs[0] = t0;
    bcs[1] = sqrtf(1.f - powf(a.beta2, t0));
    bcs[2] = a.lr / (1.f - powf(a.beta1, t0));
  }
  __syncthreads();
  const float t = bcs[0], bc2_sqrt = bcs[1], step_size = bcs[2];
  if (!RED || (int)blockIdx.x >= rd.ncol) {
    const int64_t i4 = ((int64_t)((int)blockIdx.x - (RED ? rd.ncol : 0)) * 256 + threadIdx.x) * 4;
    bool skip = false;  // a quad of a folded layer: its column block updates it
    if constexpr (RED) {
      for (int j = 0; j < rd.nr; ++j) skip |= i4 >= rd.lo[j] && i4 < rd.hi[j];
    }
    if (skip) {
    } else if (i4 + 3 < a.n) {
      float4 p = *reinterpret_cast<float4*>(a.params + i4);
      float4 g = *reinterpret_cast<float4*>(a.grads + i4);
      float4 m = *reinterpret_cast<float4*>(a.exp_avg + i4);
      float4 v = *reinterpret_cast<float4*>(a.exp_avg_sq + i4);
      adam_one(p.x, g.x, m.x, v.x, a, step_size, bc2_sqrt);
      adam_one(p.y, g.y, m.y, v.y, a, step_size, bc2_sqrt);
      adam_one(p.z, g.z, m.z, v.z, a, step_size, bc2_sqrt);
      adam_one(p.w, g.w, m.w, v.w, a, step_size, bc2_sqrt);
      *reinterpret_cast<float4*>(a.params + i4) = p;
      if (a.zero_grad) *reinterpret_cast<float4*>(a.grads + i4) = g;
      *reinterpret_cast<float4*>(a.exp_avg + i4) = m;
      *reinterpret_cast<float4*>(a.exp_avg_sq + i4) = v;
    } else {
      for (int64_t i = i4; i < a.n; ++i) adam_one(a.params[i], a.grads[i], a.exp_avg[i], a.exp_avg_sq[i], a, step_size, bc2_sqrt);
    }
  } else if constexpr (RED) {
    // slab column i of layer l: conv_reduce_multi's fixed-order sum, stored to its gradient slot
    // (or 0 with zero_grad) and that element's Adam update
    const int rb = (int)blockIdx.x;
    int l = 0;
    while (l + 1 < rd.r.n && rb >= rd.boff[l + 1]) ++l;  // (uniform)
    const ConvGeo& g = rd.r.g[l];
    const int i = (rb - rd.boff[l]) * 256 + threadIdx.x;
    if (i < g.N * g.Kp + g.N) {
      int wi, bi;
      float gs = slab_column(rd.r.slab[l], rd.r.nblk[l], g, i, &wi, &bi);
      const int64_t o = wi >= 0 ? rd.w_off[l] + wi : (bi >= 0 && rd.b_off[l] >= 0 ? rd.b_off[l] + bi : -1);
      if (o >= 0) {
        adam_one(a.params[o], gs, a.exp_avg[o], a.exp_avg_sq[o], a, step_size, bc2_sqrt);
        a.grads[o] = gs;
      }
    }
  }
  if (a.app_cursor && blockIdx.x == 0) {
    __shared__ int cur;
    if (threadIdx.x == 0) cur = *a.app_cursor;
    __syncthreads();
    for (int i = threadIdx.x; i < a.app_n; i += blockDim.x) a.app_all[(size_t)cur * a.app_n + i] = a.app_src[i];
    if (threadIdx.x == 0) *a.app_cursor = cur + 1;
  }
  if (a.cnt) {
    // the step counter advances once every block has read it: the last block to arrive stores
    // it (vector atomics, agent scope) -- no separate `step += 1` launch per optimizer step
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(a.cnt, 1u) == gridDim.x - 1;
    __syncthreads();
    if (last && threadIdx.x == 0) {
      __hip_atomic_store(a.step, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

hipError_t adam_flat(const AdamArgs& a, hipStream_t s, const ConvReduceMulti* red) {
  if (a.n <= 0) return hipSuccess;
  if (((uintptr_t)a.params | (uintptr_t)a.grads | (uintptr_t)a.exp_avg | (uintptr_t)a.exp_avg_sq) & 15)
    return hipErrorInvalidValue;  // float4 access needs 16-B aligned buffers
  const int64_t threads = (a.n + 3) / 4;
  const int nadam = (int)((threads + 255) / 256);
  AdamRed rd{};
  if (red == nullptr || red->n <= 0) {
    hipLaunchKernelGGL(adam_flat_kernel<false>, dim3((unsigned)nadam), dim3(256), 0, s, a, rd);
    return hipGetLastError();
  }
  if (red->n > kMaxPack) return hipErrorInvalidValue;
  rd.r = *red;
  int total = 0;
  for (int l = 0; l < red->n; ++l) {
    const ConvGeo& g = red->g[l];
    int mpb = 0;
    conv_wgrad_blocks(g, &rd.r.nblk[l], &mpb);
    const int64_t nw = (int64_t)g.N * g.C * g.KH * g.KW;
    rd.w_off[l] = red->dW[l] - a.grads;
    rd.b_off[l] = red->db[l] ? red->db[l] - a.grads : -1;
    // the slots must be whole quads of the flat buffer (the elementwise blocks skip them)
    if (rd.w_off[l] < 0 || rd.w_off[l] + nw > a.n || rd.w_off[l] % 4 || nw % 4) return hipErrorInvalidValue;
    rd.lo[rd.nr] = rd.w_off[l];
    rd.hi[rd.nr++] = rd.w_off[l] + nw;
    if (red->db[l]) {
      if (rd.b_off[l] < 0 || rd.b_off[l] + g.N > a.n || rd.b_off[l] % 4 || g.N % 4) return hipErrorInvalidValue;
      rd.lo[rd.nr] = rd.b_off[l];
      rd.hi[rd.nr++] = rd.b_off[l] + g.N;
    }
    rd.boff[l] = total;
    total += (g.N * g.Kp + g.N + 255) / 256;
  }
  rd.boff[red->n] = total;
  rd.ncol = total;
  hipLaunchKernelGGL(adam_flat_kernel<true>, dim3((unsigned)(nadam + total)), dim3(256), 0, s, a, rd);
  return hipGetLastError();
}

}  // namespace ia

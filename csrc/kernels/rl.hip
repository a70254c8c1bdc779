// RL update kernels: GAE as a parallel affine scan, and keyed pseudo-random
// permutations for the PPO minibatch order.
//
// GAE(gamma, lambda) over [T, N] rollouts (SB3 RolloutBuffer semantics; the
// reference reaches it through SB3 PPO). The backward
// recurrence  a_t = delta_t + c_t * a_{t+1},  c_t = gamma * lambda * (1 - start_{t+1}),
// is a composition of affine maps, so instead of one lane walking all T steps of an
// env (T dependent FMAs: 87 us for the 512-step GAIL round) each env gets one wave:
// lane l owns the contiguous steps [l*L, (l+1)*L), folds them into one map (C, D)
// with zero carry-in, a 6-step suffix scan across the 64 lanes composes the maps of
// all later chunks, and each lane replays its chunk with the exact carry-in. Fixed
// association order: deterministic, and within a few ulp of the serial loop.
//
// Minibatch permutations: SB3 draws np.random.permutation per epoch; the engine used
// torch.randperm (a device radix sort, ~40 us per epoch on the round's critical
// path). Here every index is mapped through a 4-round keyed Feistel network on the
// next even bit width >= log2(n) with cycle walking back into [0, n) -- a bijection,
// so each epoch's row order is a permutation, computed in one pass with no sort and
// no scratch. Keys come from mix64(seed, epoch), so DP replicas given the same
// seed produce the same order.
#include <hip/hip_runtime.h>

#include "ia/wave.h"
#include "launchers.h"

namespace ia {
namespace {

constexpr int kGaeWaves = 4;

// Per-env sums (sum R, sum R^2, sum A, sum A^2) of the returns R and advantages A = R - V:
// the moments of SB3's train/explained_variance = 1 - Var(R - V) / Var(R), combined on the
// host from the [N][4] partials (no extra pass over the rollout, no atomics).
__device__ __forceinline__ void store_moments(float* mom, int n, int lane, float m0, float m1, float m2, float m3) {
  m0 = wave_sum(m0);
  m1 = wave_sum(m1);
  m2 = wave_sum(m2);
  m3 = wave_sum(m3);
  if (lane == 0) {
    mom[4 * n + 0] = m0;
    mom[4 * n + 1] = m1;
    mom[4 * n + 2] = m2;
    mom[4 * n + 3] = m3;
  }
}
constexpr int kGaeRegSteps = 16;  // register fast path: T <= 64 * 16

__global__ __launch_bounds__(64 * kGaeWaves) void gae_scan_kernel(const float* __restrict__ rew,
                                                                  const float* __restrict__ val,
                                                                  const float* __restrict__ starts,
                                                                  const float* __restrict__ last_val,
                                                                  const float* __restrict__ dones, int T, int N,
                                                                  float gamma, float lam, float* __restrict__ adv,
                                                                  float* __restrict__ ret, float* __restrict__ mom) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * kGaeWaves + (threadIdx.x >> 6);
  if (n >= N) return;  // whole wave exits together
  const int L = (T + 63) >> 6;
  const int t0 = lane * L;
  const int t1 = t0 + L < T ? t0 + L : T;
  const float gl = gamma * lam;
  if (L <= kGaeRegSteps) {
    // chunks of <= 16 steps (T <= 1024): every load of the chunk is issued up front into
    // registers (one memory latency instead of one per step and pass); steps past the chunk
    // are identity maps (delta 0, c 1), so the fold and the replay are bitwise the loop's
    float dl[kGaeRegSteps], cl[kGaeRegSteps], vl[kGaeRegSteps];
#pragma unroll
    for (int i = 0; i < kGaeRegSteps; ++i) {
      const int t = t0 + i;
      dl[i] = 0.f;
      cl[i] = 1.f;
      vl[i] = 0.f;
      if (t < t1) {
        const size_t o = (size_t)t * N + n;
        float nv, nnt;
        if (t + 1 < T) {
          nv = val[o + N];
          nnt = 1.f - starts[o + N];
        } else {
          nv = last_val[n];
          nnt = 1.f - dones[n];
        }
        vl[i] = val[o];
        dl[i] = rew[o] + gamma * nv * nnt - vl[i];
        cl[i] = gl * nnt;
      }
    }
    float C = 1.f, D = 0.f;
#pragma unroll
    for (int i = kGaeRegSteps - 1; i >= 0; --i) {
      D = dl[i] + cl[i] * D;
      C = cl[i] * C;
    }
    float SC = C, SD = D;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      const float oc = __shfl_down(SC, k, 64);
      const float od = __shfl_down(SD, k, 64);
      if (lane + k < 64) {
        SD = SD + SC * od;
        SC = SC * oc;
      }
    }
    float a = __shfl_down(SD, 1, 64);
    if (lane == 63) a = 0.f;
    float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
#pragma unroll
    for (int i = kGaeRegSteps - 1; i >= 0; --i) {
      const int t = t0 + i;
      a = dl[i] + cl[i] * a;
      if (t < t1) {
        const size_t o = (size_t)t * N + n;
        const float r = a + vl[i];
        adv[o] = a;
        ret[o] = r;
        m0 += r;
        m1 += r * r;
        m2 += a;
        m3 += a * a;
      }
    }
    if (mom) store_moments(mom, n, lane, m0, m1, m2, m3);
    return;
  }
  // fold this lane's chunk: a(t0) = D + C * a(t1)
  float C = 1.f, D = 0.f;
  for (int t = t1 - 1; t >= t0; --t) {
    const size_t o = (size_t)t * N + n;
    float nv, nnt;
    if (t + 1 < T) {
      nv = val[o + N];
      nnt = 1.f - starts[o + N];
    } else {
      nv = last_val[n];
      nnt = 1.f - dones[n];
    }
    const float delta = rew[o] + gamma * nv * nnt - val[o];
    const float c = gl * nnt;
    D = delta + c * D;
    C = c * C;
  }
  // inclusive suffix scan of the maps over lanes l..63: (C, D)_l o (C, D)_{l+k}
  float SC = C, SD = D;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const float oc = __shfl_down(SC, k, 64);
    const float od = __shfl_down(SD, k, 64);
    if (lane + k < 64) {
      SD = SD + SC * od;
      SC = SC * oc;
    }
  }
  // carry into this chunk = a(t1) = suffix value of lane + 1 (zero past the end)
  float a = __shfl_down(SD, 1, 64);
  if (lane == 63) a = 0.f;
  float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
  for (int t = t1 - 1; t >= t0; --t) {
    const size_t o = (size_t)t * N + n;
    float nv, nnt;
    if (t + 1 < T) {
      nv = val[o + N];
      nnt = 1.f - starts[o + N];
    } else {
      nv = last_val[n];
      nnt = 1.f - dones[n];
    }
    const float v = val[o];
    const float delta = rew[o] + gamma * nv * nnt - v;
    a = delta + gl * nnt * a;
    adv[o] = a;
    ret[o] = a + v;
    m0 += a + v;
    m1 += (a + v) * (a + v);
    m2 += a;
    m3 += a * a;
  }
  if (mom) store_moments(mom, n, lane, m0, m1, m2, m3);
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// grid (ceil(n / 256), E); one thread per (epoch, index)
__global__ __launch_bounds__(256) void perm_feistel_kernel(int n, int half_bits, uint64_t seed, int* __restrict__ out) {
  const int e = blockIdx.y;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t k01 = mix64(seed ^ (0xA24BAED4963EE407ull * (uint64_t)(e + 1)));
  const uint64_t k23 = mix64(k01);
  const uint32_t key[4] = {(uint32_t)k01, (uint32_t)(k01 >> 32), (uint32_t)k23, (uint32_t)(k23 >> 32)};
  const uint32_t mask = (1u << half_bits) - 1u;
  uint32_t x = (uint32_t)i;
  do {  // cycle walking: the domain is < 4n, so this ends after < 4 rounds on average
    uint32_t Lh = x >> half_bits, Rh = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t f = mix32(Rh ^ key[r]) & mask;
      const uint32_t nl = Rh;
      Rh = Lh ^ f;
      Lh = nl;
    }
    x = (Lh << half_bits) | Rh;
  } while (x >= (uint32_t)n);
  out[(size_t)e * n + i] = (int)x;
}

}  // namespace

hipError_t gae_launch(const float* rew, const float* val, const float* starts, const float* last_val, const float* dones,
                      int T, int N, float gamma, float lam, float* adv, float* ret, hipStream_t s, float* mom) {
  if (T <= 0 || N <= 0) return hipSuccess;
  const int nblk = (N + kGaeWaves - 1) / kGaeWaves;
  hipLaunchKernelGGL(gae_scan_kernel, dim3(nblk), dim3(64 * kGaeWaves), 0, s, rew, val, starts, last_val, dones, T, N,
                     gamma, lam, adv, ret, mom);
  return hipGetLastError();
}

hipError_t perm_feistel(int E, int n, uint64_t seed, int* out, hipStream_t s) {
  if (E <= 0 || n <= 0) return hipSuccess;
  if (n > (1 << 30)) return hipErrorInvalidValue;
  int bits = 2;
  while ((1ll << bits) < (long long)n) bits += 2;
  hipLaunchKernelGGL(perm_feistel_kernel, dim3((n + 255) / 256, E), dim3(256), 0, s, n, bits / 2, seed, out);
  return hipGetLastError();
}


// ---------------------------------------------------------------- categorical evaluate_actions
// log pi(a|s) and the entropy of a categorical head from its raw logits [B][A] in one pass
// (logsumexp, gather, softmax, entropy: ~10 torch kernels), and the matching logit gradient
// dz_k = g_lp (1[k == a] - p_k) - g_ent p_k (log p_k + H). One thread per row (A <= 64).
namespace {
__global__ __launch_bounds__(256) void cat_eval_fwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ act,
                                                           int B, int A, float* __restrict__ logp, float* __restrict__ ent) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= B) return;
  const float* zr = z + (size_t)r * A;
  float mx = -INFINITY;
  for (int k = 0; k < A; ++k) mx = fmaxf(mx, zr[k]);
  float se = 0.f;
  for (int k = 0; k < A; ++k) se += expf(zr[k] - mx);
  const float lse = mx + logf(se);
  float h = 0.f;
  for (int k = 0; k < A; ++k) {
    const float lp = zr[k] - lse;
    h -= expf(lp) * lp;
  }
  const int a = (int)act[r];
  logp[r] = (a >= 0 && a < A) ? zr[a] - lse : -INFINITY;
  ent[r] = h;
}

__global__ __launch_bounds__(256) void cat_eval_bwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ act,
                                                           int B, int A, const float* __restrict__ g_lp,
                                                           const float* __restrict__ g_ent, float* __restrict__ dz) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= B) return;
  const float* zr = z + (size_t)r * A;
  float mx = -INFINITY;
  for (int k = 0; k < A; ++k) mx = fmaxf(mx, zr[k]);
  float se = 0.f;
  for (int k = 0; k < A; ++k) se += expf(zr[k] - mx);
  const float lse = mx + logf(se);
  float h = 0.f;
  for (int k = 0; k < A; ++k) {
    const float lp = zr[k] - lse;
    h -= expf(lp) * lp;
  }
  const float gl = g_lp ? g_lp[r] : 0.f, ge = g_ent ? g_ent[r] : 0.f;
  const int a = (int)act[r];
  for (int k = 0; k < A; ++k) {
    const float lp = zr[k] - lse, p = expf(lp);
    dz[(size_t)r * A + k] = gl * ((k == a ? 1.f : 0.f) - p) - ge * p * (lp + h);
  }
}
}  // namespace

hipError_t cat_eval_fwd(const float* z, const int64_t* act, int B, int A, float* logp, float* ent, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(cat_eval_fwd_kernel, dim3((B + 255) / 256), dim3(256), 0, s, z, act, B, A, logp, ent);
  return hipGetLastError();
}

hipError_t cat_eval_bwd(const float* z, const int64_t* act, int B, int A, const float* g_lp, const float* g_ent, float* dz,
                        hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(cat_eval_bwd_kernel, dim3((B + 255) / 256), dim3(256), 0, s, z, act, B, A, g_lp, g_ent, dz);
  return hipGetLastError();
}

// ---------------------------------------------------------------- BC categorical loss
// BehaviorCloningLossCalculator on a categorical head (reference algorithms/bc.py:100-130)
// as 2 forward launches + 1 backward launch instead of ~25 elementwise / reduce kernels:
//   sumsq_partials: fixed-order per-block partial sums of ||theta||^2 over the flat
//                   parameter buffer (FusedAdam's bucket);
//   bc_cat_loss_fwd: one block; per-row log pi(a), entropy, pi(a) reduced in a fixed
//                   order, the partials summed, and the metric vector written:
//                   [neglogp, entropy, ent_loss, prob_true_act, l2_norm, l2_loss, loss].
//   bc_cat_loss_bwd: logit gradient for an upstream gradient g[7] of the metric vector (and /
//                   or g_loss of the separately returned loss, added to g[6]):
//                   per row g_lp = (-g0 - g6)/B + g3 pi(a)/B, g_ent = (g1 - w g2 - w g6)/B,
//                   dz_k = g_lp (1[k == a] - p_k) - g_ent p_k (log p_k + H).
namespace {
constexpr int kLossThreads = 256;

__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(kLossThreads) void sumsq_partials_kernel(const float* __restrict__ x, long n,
                                                                      float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  const long n4 = n >> 2;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  for (long i = (long)blockIdx.x * kLossThreads + threadIdx.x; i < n4; i += (long)gridDim.x * kLossThreads) {
    const float4 v = x4[i];
    s += (v.x * v.x + v.y * v.y) + (v.z * v.z + v.w * v.w);
  }
  if (blockIdx.x == 0)
    for (long i = (n4 << 2) + threadIdx.x; i < n; i += kLossThreads) s += x[i] * x[i];
  s = block_sum256(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__device__ __forceinline__ void cat_row(const float* zr, int A, float& lse, float& h) {
  float mx = -INFINITY;
  for (int k = 0; k < A; ++k) mx = fmaxf(mx, zr[k]);
  float se = 0.f;
  for (int k = 0; k < A; ++k) se += expf(zr[k] - mx);
  lse = mx + logf(se);
  h = 0.f;
  for (int k = 0; k < A; ++k) {
    const float lp = zr[k] - lse;
    h -= expf(lp) * lp;
  }
}

__global__ __launch_bounds__(kLossThreads) void bc_cat_loss_fwd_kernel(const float* __restrict__ z,
                                                                       const int64_t* __restrict__ act, int B, int A,
                                                                       const float* __restrict__ part, int nparts,
                                                                       float ent_w, float l2_w, float* __restrict__ out,
                                                                       float* __restrict__ loss_out) {
  __shared__ float red[4];
  float slp = 0.f, sent = 0.f, sp = 0.f;
  for (int r = threadIdx.x; r < B; r += kLossThreads) {
    const float* zr = z + (size_t)r * A;
    float lse, h;
    cat_row(zr, A, lse, h);
    const int a = (int)act[r];
    const float lp = (a >= 0 && a < A) ? zr[a] - lse : -INFINITY;
    slp += lp;
    sent += h;
    sp += expf(lp);
  }
  float sq = 0.f;
  for (int i = threadIdx.x; i < nparts; i += kLossThreads) sq += part[i];
  slp = block_sum256(slp, red);
  sent = block_sum256(sent, red);
  sp = block_sum256(sp, red);
  sq = block_sum256(sq, red);
  if (threadIdx.x == 0) {
    const float inv = 1.f / (float)B;
    const float neglogp = -slp * inv, ent = sent * inv, ent_loss = -ent_w * ent;
    const float l2 = 0.5f * sq, l2_loss = l2_w * l2;
    out[0] = neglogp;
    out[1] = ent;
    out[2] = ent_loss;
    out[3] = sp * inv;
    out[4] = l2;
    out[5] = l2_loss;
    out[6] = neglogp + ent_loss + l2_loss;
    if (loss_out) loss_out[0] = out[6];
  }
}

__global__ __launch_bounds__(kLossThreads) void bc_cat_loss_bwd_kernel(const float* __restrict__ z,
                                                                       const int64_t* __restrict__ act, int B, int A,
                                                                       const float* __restrict__ g,
                                                                       const float* __restrict__ g_loss, float ent_w,
                                                                       float* __restrict__ dz) {
  const int r = blockIdx.x * kLossThreads + threadIdx.x;
  if (r >= B) return;
  const float* zr = z + (size_t)r * A;
  float lse, h;
  cat_row(zr, A, lse, h);
  const int a = (int)act[r];
  const float inv = 1.f / (float)B;
  const float pa = (a >= 0 && a < A) ? expf(zr[a] - lse) : 0.f;
  // upstream: the metric vector's gradient g[7] and / or the separate loss output's g_loss
  const float g6 = (g ? g[6] : 0.f) + (g_loss ? g_loss[0] : 0.f);
  const float g0 = g ? g[0] : 0.f, g1 = g ? g[1] : 0.f, g2 = g ? g[2] : 0.f, g3 = g ? g[3] : 0.f;
  const float gl = (-g0 - g6) * inv + g3 * pa * inv;
  const float ge = (g1 - ent_w * g2 - ent_w * g6) * inv;
  for (int k = 0; k < A; ++k) {
    const float lp = zr[k] - lse, p = expf(lp);
    dz[(size_t)r * A + k] = gl * ((k == a ? 1.f : 0.f) - p) - ge * p * (lp + h);
  }
}
}  // namespace

int sumsq_nparts(long n) {
  const long blocks = (n / 4 + kLossThreads * 8 - 1) / (kLossThreads * 8);
  return (int)(blocks < 1 ? 1 : (blocks > 256 ? 256 : blocks));
}

hipError_t bc_cat_loss_fwd(const float* z, const int64_t* act, int B, int A, const float* flat, long n, float* part,
                           float ent_w, float l2_w, float* out, float* loss_out, hipStream_t s) {
  int np = 0;
  if (flat && n > 0) {
    np = sumsq_nparts(n);
    hipLaunchKernelGGL(sumsq_partials_kernel, dim3(np), dim3(kLossThreads), 0, s, flat, n, part);
  }
  hipLaunchKernelGGL(bc_cat_loss_fwd_kernel, dim3(1), dim3(kLossThreads), 0, s, z, act, B, A, part, np, ent_w, l2_w, out,
                     loss_out);
  return hipGetLastError();
}

hipError_t bc_cat_loss_bwd(const float* z, const int64_t* act, int B, int A, const float* g, const float* g_loss,
                           float ent_w, float* dz, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(bc_cat_loss_bwd_kernel, dim3((B + kLossThreads - 1) / kLossThreads), dim3(kLossThreads), 0, s, z,
                     act, B, A, g, g_loss, ent_w, dz);
  return hipGetLastError();
}

}  // namespace ia

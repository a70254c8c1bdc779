// Inference tail of a NatureCNN actor for the device DAgger collector (engine/dagger.py).
//
// After the three conv_fwd launches (conv.hip) the policy still needs
// Linear(3136 -> 512) + ReLU, the action head Linear(512 -> A) and the action choice.
// Through torch that is ~25 launches per forward (flatten permute, hipBLASLt GEMM,
// bias/ReLU, logsumexp, argmax / Gumbel sampling, the β-mix), ~250 us for two policies at
// batch 8 -- more than the three convolutions. Here it is two launches (the FC of the
// expert and the learner share one, cnn_fc_pair, like their convs share conv_fwd_pair):
//
//   cnn_fc    h[B][H] = relu(X[B][K] . W1[H][K]^T + b1): v_mfma_f32_16x16x32_bf16 tiles of
//             16 rows x 16 hidden units, K split over the 4 waves of a block and summed in
//             LDS in wave order (deterministic); X is the conv3 output in its NHWC order and
//             W1's columns are permuted once per refresh to (h, w, c) to match.
//   cnn_head  one workgroup: logits[b][a] = W2[a] . h[b] + b2[a] (wave-reduced dots), then
//             argmax (deterministic) or Gumbel-max sampling from a counter-based hash keyed
//             by (seed, device call counter, b, a) -- a new draw every replay of a captured
//             graph -- and, optionally, the β-mix: executed = u > β ? own : expert.
#include <hip/hip_runtime.h>

#include "ia/mfma.h"
#include "launchers.h"

namespace ia {
namespace {

constexpr int kFcWaves = 8;

__device__ __forceinline__ void cnn_fc_tile(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                            const float* __restrict__ bias, float* __restrict__ H, int B, int K, int NH,
                                            int bx, int by) {
  __shared__ f32x4 red[kFcWaves][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n0 = bx * 16, m0 = by * 16;
  const int r = l & 15, kq = (l >> 4) * 8;
  const int ksteps = K / 32;
  const int per = (ksteps + kFcWaves - 1) / kFcWaves;
  const int s0 = w * per, s1 = s0 + per < ksteps ? s0 + per : ksteps;
  const int m = m0 + r;
  const bf16* xr = X + (size_t)(m < B ? m : 0) * K + kq;
  const bf16* wr = W + (size_t)(n0 + r) * K + kq;
  f32x4 acc = zero4();
#pragma unroll 4
  for (int s = s0; s < s1; ++s) {
    bf16x8 a = *reinterpret_cast<const bf16x8*>(xr + s * 32);
    if (m >= B) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = (bf16)0.f;
    }
    const bf16x8 b = *reinterpret_cast<const bf16x8*>(wr + s * 32);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
  red[w][l] = acc;
  __syncthreads();
  if (w != 0) return;
  f32x4 t = red[0][l];
#pragma unroll
  for (int q = 1; q < kFcWaves; ++q) {
    const f32x4 u = red[q][l];
    t[0] += u[0]; t[1] += u[1]; t[2] += u[2]; t[3] += u[3];
  }
  const int n = n0 + (l & 15);
  const float bb = bias[n];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + 4 * (l >> 4) + i;
    if (row < B) H[(size_t)row * NH + n] = fmaxf(t[i] + bb, 0.f);
  }
}

__global__ __launch_bounds__(64 * kFcWaves) void cnn_fc_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                              const float* __restrict__ bias, float* __restrict__ H, int B,
                                                              int K, int NH) {
  cnn_fc_tile(X, W, bias, H, B, K, NH, blockIdx.x, blockIdx.y);
}

// expert + learner FC layers in one launch (blockIdx.z = which), as conv_fwd_pair
__global__ __launch_bounds__(64 * kFcWaves) void cnn_fc_pair_kernel(CnnFcPair p, int B, int K, int NH) {
  const int z = blockIdx.z;
  cnn_fc_tile(static_cast<const bf16*>(p.X[z]), static_cast<const bf16*>(p.W[z]), p.bias[z], p.H[z], B, K, NH,
              blockIdx.x, blockIdx.y);
}

__device__ __forceinline__ uint64_t hmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// uniform in (0, 1)
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t ctr, int b, int a) {
  const uint64_t h = hmix(seed ^ hmix(ctr * 0x100000001B3ull + (uint64_t)b * 131ull + (uint64_t)a));
  return ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
}

constexpr int kMaxHeadActions = 64;

// One wave per batch row: every lane owns NH/64 hidden units and accumulates all A logits,
// then A wave reductions. For NH <= 64 * kHeadJ (NatureCNN: 512) every load of the row -- the
// lane's hidden values and the A x NH/64 weights -- is issued before the first FMA (one memory
// latency per row instead of one per 64 hidden units); the FMAs keep the j-ascending order of
// the general loop, so both paths give the same bits.
constexpr int kHeadRegA = 8;
constexpr int kHeadJ = 8;

__device__ __forceinline__ void head_logits(const CnnHeadArgs& a, const float* hb, int a0, int l, float (&acc)[kHeadRegA]) {
#pragma unroll
  for (int q = 0; q < kHeadRegA; ++q) acc[q] = 0.f;
  if (a.NH <= 64 * kHeadJ) {
    float hv[kHeadJ], wv[kHeadRegA][kHeadJ];
#pragma unroll
    for (int jj = 0; jj < kHeadJ; ++jj) {
      const int j = l + 64 * jj;
      hv[jj] = j < a.NH ? hb[j] : 0.f;
#pragma unroll
      for (int q = 0; q < kHeadRegA; ++q) wv[q][jj] = (j < a.NH && a0 + q < a.A) ? a.W2[(size_t)(a0 + q) * a.NH + j] : 0.f;
    }
#pragma unroll
    for (int jj = 0; jj < kHeadJ; ++jj) {
      if (l + 64 * jj >= a.NH) break;
#pragma unroll
      for (int q = 0; q < kHeadRegA; ++q)
        if (a0 + q < a.A) acc[q] += hv[jj] * wv[q][jj];
    }
    return;
  }
  for (int j = l; j < a.NH; j += 64) {
    const float hv = hb[j];
#pragma unroll
    for (int q = 0; q < kHeadRegA; ++q)
      if (a0 + q < a.A) acc[q] += hv * a.W2[(size_t)(a0 + q) * a.NH + j];
  }
}

// Row b's choice under head a (argmax, or Gumbel-max with the launch counter ctr).
__device__ __forceinline__ int head_row(const CnnHeadArgs& a, int b, uint64_t ctr, int l) {
  const float* hb = a.h + (size_t)b * a.NH;
  int best = 0;
  float best_v = -INFINITY;
  for (int a0 = 0; a0 < a.A; a0 += kHeadRegA) {
    float acc[kHeadRegA];
    head_logits(a, hb, a0, l, acc);
#pragma unroll
    for (int q = 0; q < kHeadRegA; ++q) {
      if (a0 + q >= a.A) break;
      float p = acc[q];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) p += __shfl_xor(p, o, 64);
      float v = p + a.b2[a0 + q];
      if (a.mode == 1) v += -logf(-logf(hash_uniform(a.seed, ctr, b, a0 + q)));
      if (v > best_v) {  // first maximum, like torch.argmax
        best_v = v;
        best = a0 + q;
      }
    }
  }
  return best;
}

// DAgger's per-step pair in ONE launch: the expert's argmax (e: its action and record slot) and
// the learner's sample (r), mixed as the learner's exec_out does with the expert's action of
// the same row. The two heads' rows run on different waves (2 B row tasks), their choices meet
// in LDS (B <= kHeadPairMaxB; larger batches loop both heads per wave).
constexpr int kHeadPairMaxB = 256;

__global__ __launch_bounds__(1024) void cnn_head_pair_kernel(CnnHeadArgs e, CnnHeadArgs r) {
  __shared__ int choice[2][kHeadPairMaxB];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t ctr_e = e.counter ? *e.counter : 0ull;
  const uint64_t ctr_r = r.counter ? *r.counter : 0ull;
  if (e.B <= kHeadPairMaxB) {
    for (int t = w; t < 2 * e.B; t += nw) {
      const int h = t & 1, b = t >> 1;
      const int c = h == 0 ? head_row(e, b, ctr_e, l) : head_row(r, b, ctr_r, l);
      if (l == 0) choice[h][b] = c;
    }
    __syncthreads();
    for (int b = threadIdx.x; b < e.B; b += blockDim.x) {
      const int be = choice[0][b], br = choice[1][b];
      e.out[b] = be;
      if (e.rec_out) e.rec_out[b] = be;
      r.out[b] = br;
      if (r.rec_out) r.rec_out[b] = br;
      if (r.exec_out) {
        const float u = hash_uniform(r.seed ^ 0x5DEECE66Dull, ctr_r, b, kMaxHeadActions);
        r.exec_out[b] = (u > *r.beta) ? (int64_t)br : (int64_t)be;
      }
    }
  } else {
    for (int b = w; b < e.B; b += nw) {
      const int be = head_row(e, b, ctr_e, l);
      const int br = head_row(r, b, ctr_r, l);
      if (l == 0) {
        e.out[b] = be;
        if (e.rec_out) e.rec_out[b] = be;
        r.out[b] = br;
        if (r.rec_out) r.rec_out[b] = br;
        if (r.exec_out) {
          const float u = hash_uniform(r.seed ^ 0x5DEECE66Dull, ctr_r, b, kMaxHeadActions);
          r.exec_out[b] = (u > *r.beta) ? (int64_t)br : (int64_t)be;
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (e.counter) *e.counter = ctr_e + 1;
    if (r.counter) *r.counter = ctr_r + 1;
  }
}

__global__ __launch_bounds__(1024) void cnn_head_kernel(CnnHeadArgs a) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t ctr = a.counter ? *a.counter : 0ull;
  for (int b = w; b < a.B; b += nw) {
    const int best = head_row(a, b, ctr, l);
    if (l == 0) {
      a.out[b] = best;
      if (a.rec_out) a.rec_out[b] = best;
      if (a.exec_out) {
        const float u = hash_uniform(a.seed ^ 0x5DEECE66Dull, ctr, b, kMaxHeadActions);
        a.exec_out[b] = (u > *a.beta) ? (int64_t)best : a.mix_expert[b];
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && a.counter) *a.counter = ctr + 1;
}

}  // namespace

hipError_t cnn_fc(const void* X, const void* W, const float* bias, float* H, int B, int K, int NH, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (K % 32 != 0 || NH % 16 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnn_fc_kernel, dim3(NH / 16, (B + 15) / 16), dim3(64 * kFcWaves), 0, s, static_cast<const bf16*>(X),
                     static_cast<const bf16*>(W), bias, H, B, K, NH);
  return hipGetLastError();
}

hipError_t cnn_fc_pair(const CnnFcPair& p, int B, int K, int NH, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (K % 32 != 0 || NH % 16 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cnn_fc_pair_kernel, dim3(NH / 16, (B + 15) / 16, 2), dim3(64 * kFcWaves), 0, s, p, B, K, NH);
  return hipGetLastError();
}

hipError_t cnn_head_pair(const CnnHeadArgs& e, const CnnHeadArgs& r, hipStream_t s) {
  if (e.B <= 0) return hipSuccess;
  if (e.B != r.B || e.NH != r.NH || e.A <= 0 || e.A > kMaxHeadActions || r.A <= 0 || r.A > kMaxHeadActions)
    return hipErrorInvalidValue;
  if (r.exec_out && !r.beta) return hipErrorInvalidValue;
  const int waves = 2 * e.B < 16 ? 2 * e.B : 16;
  hipLaunchKernelGGL(cnn_head_pair_kernel, dim3(1), dim3(64 * waves), 0, s, e, r);
  return hipGetLastError();
}

hipError_t cnn_head(const CnnHeadArgs& a, hipStream_t s) {
  if (a.B <= 0) return hipSuccess;
  if (a.A <= 0 || a.A > kMaxHeadActions) return hipErrorInvalidValue;
  const int waves = a.B < 16 ? a.B : 16;
  hipLaunchKernelGGL(cnn_head_kernel, dim3(1), dim3(64 * waves), 0, s, a);
  return hipGetLastError();
}

}  // namespace ia

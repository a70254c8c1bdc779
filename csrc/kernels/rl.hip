// RL update kernels: GAE scan.
//
// GAE(gamma, lambda) over [T, N] rollouts (SB3 RolloutBuffer semantics; the
// reference reaches it through SB3 PPO).  Each block
// owns 64 envs; its 256 threads stage a 64-step time chunk of rewards / values /
// episode_starts into LDS with coalesced loads (row t of the chunk is 64
// consecutive envs), then one wave scans the chunk backwards with the carry in a
// register, and the chunk's advantages/returns are written back coalesced.
#include <hip/hip_runtime.h>

#include "launchers.h"

namespace ia {
namespace {

constexpr int kEnvs = 64;
constexpr int kChunk = 64;

__global__ __launch_bounds__(256) void gae_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                  const float* __restrict__ starts, const float* __restrict__ last_val,
                                                  const float* __restrict__ dones, int T, int N, float gamma, float lam,
                                                  float* __restrict__ adv, float* __restrict__ ret) {
  __shared__ float sr[kChunk][kEnvs + 1];
  __shared__ float sv[kChunk + 1][kEnvs + 1];  // row kChunk = values of the step after the chunk
  __shared__ float ss[kChunk + 1][kEnvs + 1];
  __shared__ float sa[kChunk][kEnvs + 1];
  const int env0 = blockIdx.x * kEnvs;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int env = env0 + lane;
  float carry = 0.f;
  for (int t1 = T; t1 > 0; t1 -= kChunk) {
    const int t0 = t1 - kChunk > 0 ? t1 - kChunk : 0;
    const int len = t1 - t0;
    __syncthreads();
    for (int e = tid; e < (len + 1) * kEnvs; e += blockDim.x) {
      const int r = e / kEnvs, c = e - r * kEnvs;
      const int t = t0 + r, n = env0 + c;
      const bool ok = n < N;
      if (r < len) {
        sr[r][c] = ok ? rew[(size_t)t * N + n] : 0.f;
        sv[r][c] = ok ? val[(size_t)t * N + n] : 0.f;
        ss[r][c] = ok ? starts[(size_t)t * N + n] : 0.f;
      } else {  // boundary row: next step's value / start flag, or the bootstrap
        if (t < T) {
          sv[r][c] = ok ? val[(size_t)t * N + n] : 0.f;
          ss[r][c] = ok ? starts[(size_t)t * N + n] : 0.f;
        } else {
          sv[r][c] = ok ? last_val[n] : 0.f;
          ss[r][c] = ok ? dones[n] : 0.f;  // "next non-terminal" = 1 - dones at the end
        }
      }
    }
    __syncthreads();
    if (tid < 64) {
      for (int r = len - 1; r >= 0; --r) {
        const float nnt = 1.f - ss[r + 1][lane];
        const float delta = sr[r][lane] + gamma * sv[r + 1][lane] * nnt - sv[r][lane];
        carry = delta + gamma * lam * nnt * carry;
        sa[r][lane] = carry;
      }
    }
    __syncthreads();
    for (int e = tid; e < len * kEnvs; e += blockDim.x) {
      const int r = e / kEnvs, c = e - r * kEnvs;
      const int n = env0 + c;
      if (n < N) {
        const size_t o = (size_t)(t0 + r) * N + n;
        adv[o] = sa[r][c];
        ret[o] = sa[r][c] + sv[r][c];
      }
    }
  }
  (void)env;
}

}  // namespace

hipError_t gae_launch(const float* rew, const float* val, const float* starts, const float* last_val, const float* dones,
                      int T, int N, float gamma, float lam, float* adv, float* ret, hipStream_t s) {
  if (T <= 0 || N <= 0) return hipSuccess;
  const int nblk = (N + kEnvs - 1) / kEnvs;
  hipLaunchKernelGGL(gae_kernel, dim3(nblk), dim3(256), 0, s, rew, val, starts, last_val, dones, T, N, gamma, lam, adv,
                     ret);
  return hipGetLastError();
}

}  // namespace ia

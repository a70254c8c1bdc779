// Fused BC training head of a categorical CNN policy (DAgger-Pong's NatureCNN learner).
//
// The reference's BC minibatch (src/imitation/algorithms/bc.py:443-510: evaluate_actions,
// -log_prob.mean(), entropy bonus, ||theta||^2 / 2 metric, loss.backward()) spends, after the
// conv trunk and the 512-unit feature layer, ~10 small launches on the action head: the head
// GEMM, the loss forward / backward, the parameter-norm reduction, three GEMM / reduce
// launches for dW / db / dh and the gradient copies. Here ONE launch does all of it:
//
//   head blocks   : NH / 64, block c owns feature columns [64 c, 64 c + 64): W^T staged in
//                   LDS, the logits of every row (recomputed per block: no grid-wide step
//                   between the softmax and the gradients), per row the log-softmax, entropy
//                   and dL/dlogits; its columns of dW = dlog^T h (straight into the optimizer's
//                   gradient bucket) and dh = dlog W (the feature layer's upstream gradient,
//                   ReLU mask left to fc_backward); block 0 also db and the loss metrics;
//   sumsq blocks  : sum of squares of the flat parameter bucket (the logged l2_norm);
//   last block    : (agent-scope counter) reduces the nS partials in block order and finishes
//                   l2_norm / l2_loss / loss; resets the counter (graph replays).
//
// Every reduction has a fixed order, so the step is bitwise reproducible.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ia/wave.h"
#include "launchers.h"

namespace ia {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxB = 64;
constexpr int kMaxNH = 512;
constexpr int kMaxA = 8;  // minimal Atari action sets (Pong: 6); wider heads keep the autograd step

__device__ __forceinline__ void st_sc1(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// (wave sums: ia::wave_sum, DPP row sums + permlane swaps -- a __shfl_xor butterfly is six
// ds_bpermute round trips per call, ~18 of them on block 0's metrics path)
__device__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// Head blocks: NH / 64 of them, block c owning feature columns [64 c, 64 c + 64). Each
// recomputes the (tiny) logits of all B rows -- 4 waves x 8 rows, a lane 8 contiguous
// features, partials reduced through LDS in a fixed order -- so no grid-wide dependency
// separates the softmax from the gradients; then its columns of dW and dh.
constexpr int kAPad = 8;  // logits row stride (A <= kMaxA = 8)

template <int KPL>  // features per lane (NH / 64), compile-time: the logit loops carry no predicates
__global__ __launch_bounds__(kThreads) void bc_head_train_kernel(BcHeadArgs a, int n_head) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ float red[4];
  __shared__ int is_last;
  const int tid = threadIdx.x;
  const int ap = kAPad;
  if (a.prof && blockIdx.x == 0 && tid == 0) a.prof[0] = clock64();
  if ((int)blockIdx.x < n_head) {
    // LDS images laid out so that the 64 lanes of a wave touch 64 different banks:
    // W as given ([A][NH], lanes on consecutive features), logit partials [lane][pair] with a
    // 257-float row stride (pair = row-in-pass x action)
    constexpr int kPS = 257;
    float* wt = sm;                   // [ap][NH]
    float* part = wt + ap * a.NH;     // [64 lanes][kPS]
    float* lg = part + 64 * kPS;      // [B][ap] logits, then dL/dlogits
    float* pw = lg + kMaxB * ap;      // [4 row groups][ap][64] dW partials
    float* rowm = pw + 4 * ap * 64;   // [B][3]
    const int w = tid >> 6, lane = tid & 63;
    const int nh4 = a.NH >> 2;
    for (int r0 = 0; r0 < a.B; r0 += 32) {  // 32 rows per pass (B <= 64)
      // every h value of this wave's 8 rows in flight at once (one memory round trip), issued
      // before the W staging so both overlap
      float hv[8][KPL];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int r = r0 + w + 4 * q;
        const float* hr = a.h + (size_t)(r < a.B ? r : 0) * a.NH + lane;
#pragma unroll
        for (int i = 0; i < KPL; ++i) hv[q][i] = r < a.B ? hr[64 * i] : 0.f;
      }
      if (r0 == 0) {  // W rows A .. kMaxA - 1 are zero: every logit loop runs all kMaxA actions
        for (int i = tid; i < kMaxA * nh4; i += kThreads)
          reinterpret_cast<float4*>(wt)[i] =
              i < a.A * nh4 ? reinterpret_cast<const float4*>(a.W)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        __syncthreads();
        if (a.prof && blockIdx.x == 0 && tid == 0) a.prof[1] = clock64();
      }
      // ---- logit partials: wave w rows r0 + w + 4 q (q < 8). This lane's W columns go to
      // registers once: read inside the row loop they were re-read from LDS for every row (the
      // partial stores below may alias them as far as the compiler knows): 8x the LDS reads
      float wr[KPL][kMaxA];
#pragma unroll
      for (int i = 0; i < KPL; ++i)
#pragma unroll
        for (int j = 0; j < kMaxA; ++j) wr[i][j] = wt[j * KPL * 64 + 64 * i + lane];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float acc[kMaxA];
#pragma unroll
        for (int j = 0; j < kMaxA; ++j) acc[j] = 0.f;
#pragma unroll
        for (int i = 0; i < KPL; ++i) {
#pragma unroll
          for (int j = 0; j < kMaxA; ++j) acc[j] = fmaf(hv[q][i], wr[i][j], acc[j]);
        }
#pragma unroll
        for (int j = 0; j < kMaxA; ++j) part[lane * kPS + (w + 4 * q) * ap + j] = acc[j];
      }
      __syncthreads();
      if (a.prof && blockIdx.x == 0 && tid == 0) a.prof[2] = clock64();
      // ---- reduce: thread -> (row, action) pair, the 64 lane partials in lane order
      for (int pr = tid; pr < 32 * ap; pr += kThreads) {
        const int rl = pr / ap, j = pr - rl * ap;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll 4
        for (int v = 0; v < 64; v += 4) {
          s0 += part[(v + 0) * kPS + pr];
          s1 += part[(v + 1) * kPS + pr];
          s2 += part[(v + 2) * kPS + pr];
          s3 += part[(v + 3) * kPS + pr];
        }
        const int r = r0 + rl;
        if (r < a.B && j < a.A) lg[r * ap + j] = ((s0 + s1) + (s2 + s3)) + a.b[j];
      }
      __syncthreads();
      if (a.prof && blockIdx.x == 0 && tid == 0) a.prof[3] = clock64();
    }
    // ---- per row: log-softmax, entropy, dL/dlogits (loss = -mean log p(a) - ent_w mean H)
    const float inv = 1.f / (float)a.B;
    if (tid < a.B) {
      // one exp per action: p_j = e_j / sum e, log p_j = z_j - lse
      float* z = lg + tid * ap;
      float zz[kMaxA], e[kMaxA];
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < kMaxA; ++j) {
        zz[j] = z[j];
        if (j < a.A) mx = fmaxf(mx, zz[j]);
      }
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < kMaxA; ++j) {
        e[j] = j < a.A ? expf(zz[j] - mx) : 0.f;
        se += e[j];
      }
      const float lse = mx + logf(se), rse = 1.f / se;
      float h = 0.f;
#pragma unroll
      for (int j = 0; j < kMaxA; ++j)
        if (j < a.A) h -= (e[j] * rse) * (zz[j] - lse);
      const int act = (int)a.acts[tid];
      const bool ok = act >= 0 && act < a.A;
      float lpa = -INFINITY, pa = 0.f;
#pragma unroll
      for (int j = 0; j < kMaxA; ++j)
        if (j == act) {
          lpa = zz[j] - lse;
          pa = e[j] * rse;
        }
      rowm[tid * 3 + 0] = ok ? lpa : -INFINITY;
      rowm[tid * 3 + 1] = h;
      rowm[tid * 3 + 2] = ok ? pa : 0.f;
#pragma unroll
      for (int j = 0; j < kMaxA; ++j) {
        float g = 0.f;
        if (j < a.A) {
          const float lp = zz[j] - lse, p = e[j] * rse;
          g = inv * (p - (j == act ? 1.f : 0.f)) + a.ent_w * inv * p * (lp + h);
        }
        z[j] = g;
      }
    }
    __syncthreads();
    if (a.prof && blockIdx.x == 0 && tid == 0) a.prof[4] = clock64();
    // ---- this block's 64 columns: dh = dlog W (thread: column c, row group rg), dW partials
    {
      const int c = tid & 63, rg = tid >> 6;
      const int k = blockIdx.x * 64 + c;
      float pdw[kMaxA];
#pragma unroll
      for (int j = 0; j < kMaxA; ++j) pdw[j] = 0.f;
      float wk[kMaxA];
#pragma unroll
      for (int j = 0; j < kMaxA; ++j) wk[j] = wt[j * KPL * 64 + k];
      // rows rg, rg + 4, ... (<= 16 per group): all h loads in flight first
      constexpr int kRpg = kMaxB / 4;
      float hv[kRpg];
#pragma unroll
      for (int u = 0; u < kRpg; ++u) {
        const int r = rg + 4 * u;
        hv[u] = r < a.B ? a.h[(size_t)r * a.NH + k] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kRpg; ++u) {
        const int r = rg + 4 * u;
        if (r < a.B) {
          const float* g = lg + r * ap;
          float d = 0.f;
#pragma unroll
          for (int j = 0; j < kMaxA; ++j) {
            d = fmaf(g[j], wk[j], d);
            pdw[j] = fmaf(g[j], hv[u], pdw[j]);
          }
          a.dh[(size_t)r * a.NH + k] = d;
        }
      }
#pragma unroll
      for (int j = 0; j < kMaxA; ++j)
        if (j < ap) pw[(rg * ap + j) * 64 + c] = pdw[j];
      __syncthreads();
      if (a.prof && blockIdx.x == 0 && tid == 0) a.prof[5] = clock64();
      if (rg == 0)
        for (int j = 0; j < a.A; ++j)
          a.dW[(size_t)j * a.NH + k] = (pw[(0 * ap + j) * 64 + c] + pw[(1 * ap + j) * 64 + c]) +
                                       (pw[(2 * ap + j) * 64 + c] + pw[(3 * ap + j) * 64 + c]);
    }
    if (blockIdx.x == 0) {
      if (tid < a.A) {
        float s = 0.f;
        for (int r = 0; r < a.B; ++r) s += lg[r * ap + tid];
        a.db[tid] = s;
      }
      // ---- metrics (l2 terms finished by the last block)
      float slp = 0.f, sent = 0.f, sp = 0.f;
      if (tid < a.B) {
        slp = rowm[tid * 3 + 0];
        sent = rowm[tid * 3 + 1];
        sp = rowm[tid * 3 + 2];
      }
      slp = block_sum(slp, red);
      sent = block_sum(sent, red);
      sp = block_sum(sp, red);
      if (tid == 0) {
        const float neglogp = -slp * inv, ent = sent * inv, ent_loss = -a.ent_w * ent;
        st_sc1(a.metrics + 0, neglogp);
        st_sc1(a.metrics + 1, ent);
        st_sc1(a.metrics + 2, ent_loss);
        st_sc1(a.metrics + 3, sp * inv);
      }
    }
  } else {
    // ---- ||theta||^2 partial of this block's fixed float4 slice
    const int nb = gridDim.x - n_head, b = blockIdx.x - n_head;
    const long n4 = a.n_params >> 2;
    const long per = (n4 + nb - 1) / nb, i0 = (long)b * per, i1 = min(n4, i0 + per);
    const float4* x4 = reinterpret_cast<const float4*>(a.params);
    float s = 0.f;
    // 8 independent float4 loads in flight per lane per pass
    for (long i = i0 + tid; i < i1; i += 8 * kThreads) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = i + u * kThreads < i1 ? x4[i + u * kThreads] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (v[u].x * v[u].x + v[u].y * v[u].y) + (v[u].z * v[u].z + v[u].w * v[u].w);
    }
    if (b == nb - 1)
      for (long i = (n4 << 2) + tid; i < a.n_params; i += kThreads) s += a.params[i] * a.params[i];
    s = block_sum(s, red);
    if (tid == 0) st_sc1(a.partials + b, s);
  }
  // ---- hand-off: the last block to finish finishes the l2 terms and the loss
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) is_last = atomicAdd(a.cnt, 1u) == gridDim.x - 1;
  __syncthreads();
  if (a.prof && blockIdx.x == 0 && tid == 0) a.prof[6] = clock64();
  if (!is_last) return;
  // every partial and the two head metrics in flight at once (ONE memory round trip), then a
  // fixed-order block sum
  const int nb = gridDim.x - n_head;
  float s = 0.f, neglogp = 0.f, ent_loss = 0.f;
  if (tid < nb) asm volatile("global_load_dword %0, %1, off sc1" : "=v"(s) : "v"(a.partials + tid) : "memory");
  if (tid == 0) {
    asm volatile("global_load_dword %0, %1, off sc1" : "=v"(neglogp) : "v"(a.metrics + 0) : "memory");
    asm volatile("global_load_dword %0, %1, off sc1" : "=v"(ent_loss) : "v"(a.metrics + 2) : "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(s), "+v"(neglogp), "+v"(ent_loss) : : "memory");
  for (int b = tid + kThreads; b < nb; b += kThreads) s += ld_sc1(a.partials + b);
  s = block_sum(s, red);
  if (tid == 0) {
    const float l2 = 0.5f * s, l2_loss = a.l2_w * l2;
    a.metrics[4] = l2;
    a.metrics[5] = l2_loss;
    a.metrics[6] = neglogp + ent_loss + l2_loss;
    __hip_atomic_store(a.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

int bc_head_sumsq_blocks(long n_params) {
  const long blocks = (n_params / 4 + kThreads * 16 - 1) / (kThreads * 16);
  return (int)(blocks < 1 ? 1 : (blocks > 255 ? 255 : blocks));
}

size_t bc_head_lds_bytes(int B, int NH, int A) {
  const int ap = kAPad;
  (void)B;
  (void)A;
  return (size_t)(NH * ap + 64 * 257 + kMaxB * ap + 4 * ap * 64 + 3 * kMaxB) * sizeof(float);
}

bool bc_head_ok(int B, int NH, int A) {
  return B > 0 && B <= kMaxB && (NH == 512 || NH == 256) && A > 0 && A <= kMaxA &&
         bc_head_lds_bytes(B, NH, A) <= 160 * 1024;
}

hipError_t bc_head_train(const BcHeadArgs& a, hipStream_t s) {
  if (!bc_head_ok(a.B, a.NH, a.A)) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(a.h) | reinterpret_cast<uintptr_t>(a.W) | reinterpret_cast<uintptr_t>(a.params)) & 15)
    return hipErrorInvalidValue;
  const int nb = bc_head_sumsq_blocks(a.n_params), n_head = a.NH / 64;
  const dim3 grid(n_head + nb), block(kThreads);
  const size_t lds = bc_head_lds_bytes(a.B, a.NH, a.A);
  if (a.NH == 512)
    hipLaunchKernelGGL(bc_head_train_kernel<8>, grid, block, lds, s, a, n_head);
  else
    hipLaunchKernelGGL(bc_head_train_kernel<4>, grid, block, lds, s, a, n_head);
  return hipGetLastError();
}

}  // namespace ia

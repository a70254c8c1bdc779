// Wide MLP layers (widths 129..1024) on MFMA: bf16 operands, fp32 accumulation.
//
// The tiny-MLP kernels (tmlp.hip) keep a whole <= 128-wide network in one block's LDS; the
// fork's multi-agent policies do not fit: HomogenousFeedForward32Policy is [256, 256, 128]
// with the agents folded into the batch (src/imitation/policies/base.py:222-234,
// algorithms/bc.py:758-759) and SAC1024Policy is [1024, 1024] (policies/base.py:237-250).
// Those layers run here, one launch per layer and pass, with bias / activation /
// activation-derivative fused into the epilogues (no separate elementwise launches):
//
//   wlin_fwd    Y = act(X W^T + b)                        [M x N], reduce over K
//   wlin_dx     G = (dZ W) * act'(H)                      [M x K], reduce over N
//   wlin_dw     dW = dZ^T X (+ db = sum_m dZ)             [N x K], reduce over M
//
// Every block computes one 32 x 32 output tile with v_mfma_f32_32x32x16_bf16. Its four waves
// split the reduction dimension (each a contiguous quarter) and the four partial tiles are
// summed through LDS in wave order (fixed order: deterministic). The operands are loaded from
// global memory straight into the MFMA lane layout -- lane l holds row/column (l & 31) and
// 8 consecutive reduction indices starting at 8 (l >> 5) -- so there is no LDS staging;
// operand re-reads across blocks are L2 hits (a 1024 x 1024 fp32 weight is 4 MB).
#include <hip/hip_runtime.h>

#include "ia/common.h"
#include "launchers.h"

namespace ia {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 32;
constexpr int kWaves = 4;

__device__ __forceinline__ float act_f(int act, float x) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_TANH: return tanhf(x);
    case ACT_LEAKY_RELU: return x > 0.f ? x : 0.01f * x;
    case ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    default: return x;
  }
}
// derivative through the activation OUTPUT h
__device__ __forceinline__ float act_g(int act, float h) {
  switch (act) {
    case ACT_RELU: return h > 0.f ? 1.f : 0.f;
    case ACT_TANH: return 1.f - h * h;
    case ACT_LEAKY_RELU: return h > 0.f ? 1.f : 0.01f;
    case ACT_SIGMOID: return h * (1.f - h);
    default: return 1.f;
  }
}

// 8 consecutive floats p[0..7] of a row (valid for index < lim), as bf16; VEC: 16-B aligned.
template <bool VEC>
__device__ __forceinline__ bf16x8 load_row8(const float* __restrict__ p, int valid) {
  bf16x8 v;
  if (VEC && valid >= 8) {
    const f4 a = *reinterpret_cast<const f4*>(p);
    const f4 b = *reinterpret_cast<const f4*>(p + 4);
    v[0] = (__bf16)a.x, v[1] = (__bf16)a.y, v[2] = (__bf16)a.z, v[3] = (__bf16)a.w;
    v[4] = (__bf16)b.x, v[5] = (__bf16)b.y, v[6] = (__bf16)b.z, v[7] = (__bf16)b.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)(j < valid ? p[j] : 0.f);
  }
  return v;
}
// 8 floats with stride ld (p[j * ld]) for j < valid, as bf16 (coalesced across lanes)
__device__ __forceinline__ bf16x8 load_col8(const float* __restrict__ p, size_t ld, int valid) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)(j < valid ? p[j * ld] : 0.f);
  return v;
}

// sum of the four waves' partial tiles (fixed wave order); lane layout of the 32x32 C tile:
// element r of lane l is C[row (r & 3) + 8 (r >> 2) + 4 (l >> 5)][col l & 31]
__device__ __forceinline__ void reduce_tile(f32x16 acc, float (*red)[kTile][kTile + 1]) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int col = l & 31, h = l >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) red[w][(r & 3) + 8 * (r >> 2) + 4 * h][col] = acc[r];
  __syncthreads();
}

// K range of wave w: quarters rounded to the MFMA's 16
__device__ __forceinline__ void wave_range(int K, int w, int& k0, int& k1) {
  const int q = ((K + 4 * 16 - 1) / (4 * 16)) * 16;
  k0 = min(K, w * q);
  k1 = min(K, k0 + q);
}

template <bool VEC>
__global__ __launch_bounds__(64 * kWaves) void wlin_fwd_kernel(WideLinArgs a) {
  __shared__ float red[kWaves][kTile][kTile + 1];
  const int n0 = blockIdx.x * kTile, m0 = blockIdx.y * kTile;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 31, h = l >> 5;
  int k0, k1;
  wave_range(a.K, w, k0, k1);
  const int m = m0 + r, n = n0 + r;
  const float* xr = a.X + (size_t)min(m, a.M - 1) * a.K;
  const float* wr = a.W + (size_t)min(n, a.N - 1) * a.K;
  f32x16 acc = {};
#pragma unroll 4
  for (int k = k0; k < k1; k += 16) {
    const int kk = k + 8 * h;
    const int va = m < a.M ? min(8, max(0, k1 - kk)) : 0;
    const int vb = n < a.N ? min(8, max(0, k1 - kk)) : 0;
    const bf16x8 A = load_row8<VEC>(xr + kk, va);
    const bf16x8 B = load_row8<VEC>(wr + kk, vb);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, acc, 0, 0, 0);
  }
  reduce_tile(acc, red);
  for (int e = threadIdx.x; e < kTile * kTile; e += 64 * kWaves) {
    const int i = e / kTile, j = e - i * kTile;
    const int mm = m0 + i, nn = n0 + j;
    if (mm >= a.M || nn >= a.N) continue;
    float v = red[0][i][j] + red[1][i][j] + red[2][i][j] + red[3][i][j];
    if (a.b) v += a.b[nn];
    a.Y[(size_t)mm * a.N + nn] = act_f(a.act, v);
  }
}

// 4 floats base[row][col .. col+3] (zero outside rows x cols); VEC: cols % 4 == 0 and base
// 16-B aligned, so a quad is either wholly inside or wholly outside
template <bool VEC>
__device__ __forceinline__ f4 load4(const float* __restrict__ base, int row, int col, int rows, int cols) {
  f4 v = {0.f, 0.f, 0.f, 0.f};
  if (row < rows) {
    const float* p = base + (size_t)row * cols + col;
    if (VEC) {
      if (col < cols) v = *reinterpret_cast<const f4*>(p);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (col + j < cols) v[j] = p[j];
    }
  }
  return v;
}

// sc1 (L1-bypassing, agent-coherent) 16-B accesses for the dW split hand-off; inline asm so a
// lane issues its partial loads back to back, tied to the vmcnt(0) wait by "+v" operands
__device__ __forceinline__ void st_sc1_x4(float* p, f4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ f4 ld_sc1_x4(const float* p) {
  f4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void wait_vm8(f4 (&v)[8]) {
  asm volatile("s_waitcnt vmcnt(0)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])::"memory");
}

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {
  return (unsigned)__builtin_bit_cast(unsigned short, (__bf16)lo) |
         ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)hi) << 16);
}

// Transposed bf16 staging: rows (2p, 2p+1) x columns 4q..4q+3 of a row-major fp32 tile go to
// T[4q + j][2p .. 2p+1] as one 32-bit LDS store per column (pitch in bf16 elements).
__device__ __forceinline__ void stage_pair_t(__bf16* T, int pitch, int q, int p2, f4 lo, f4 hi) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    *reinterpret_cast<unsigned*>(T + (4 * q + j) * pitch + p2) = pack_bf16x2(lo[j], hi[j]);
}

// G[M x K] = (dZ[M x N] . W[N x K]) * act'(H[M x K]); reduction over N.
// Reading W down its columns is strided, so the block first stages its strip W[:, c0:c0+32]
// transposed into LDS (bf16, row pitch N + 8: 16-B aligned rows, conflict-free b128 reads);
// dZ rows are read straight into the MFMA lane layout. The block covers 64 rows: wave w
// takes rows 32 (w & 1) .. +32 and half (w >> 1) of N; the two halves meet in LDS.
template <bool VEC>
__global__ __launch_bounds__(64 * kWaves) void wlin_dx_kernel(WideLinArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char dx_smem[];
  float(*red)[kTile][kTile + 1] = reinterpret_cast<float(*)[kTile][kTile + 1]>(dx_smem);
  __bf16* wt = reinterpret_cast<__bf16*>(dx_smem + sizeof(float) * kWaves * kTile * (kTile + 1));
  const int npad = (a.N + 63) / 64 * 64, pitch = npad + 8;
  const int c0 = blockIdx.x * kTile, m0 = blockIdx.y * 2 * kTile;
  const int t = threadIdx.x, q = t & 7, p = t >> 3;
  for (int nb = 0; nb < npad; nb += 64) {  // 64 rows of W per pass: pairs (2p, 2p+1)
    const f4 lo = load4<VEC>(a.W, nb + 2 * p, c0 + 4 * q, a.N, a.K);
    const f4 hi = load4<VEC>(a.W, nb + 2 * p + 1, c0 + 4 * q, a.N, a.K);
    stage_pair_t(wt, pitch, q, nb + 2 * p, lo, hi);
  }
  __syncthreads();
  const int w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
  const int half = (npad / 2 + 15) / 16 * 16;
  const int n0 = (w >> 1) * half, n1 = min(npad, n0 + half);
  const int m = m0 + 32 * (w & 1) + r;
  const float* zr = a.dZ + (size_t)min(m, a.M - 1) * a.N;
  const __bf16* wr = wt + r * pitch;
  f32x16 acc = {};
#pragma unroll 4
  for (int n = n0; n < n1; n += 16) {
    const int nn = n + 8 * h;
    const int va = m < a.M ? min(8, max(0, a.N - nn)) : 0;
    const bf16x8 A = load_row8<VEC>(zr + nn, va);
    const bf16x8 B = *reinterpret_cast<const bf16x8*>(wr + nn);  // zero rows past N
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, acc, 0, 0, 0);
  }
  reduce_tile(acc, red);
  for (int e = t; e < 2 * kTile * kTile; e += 64 * kWaves) {
    const int sub = e / (kTile * kTile), i = (e / kTile) % kTile, j = e % kTile;
    const int mm = m0 + 32 * sub + i, cc = c0 + j;
    if (mm >= a.M || cc >= a.K) continue;
    float v = red[sub][i][j] + red[sub + 2][i][j];
    if (a.H) v *= act_g(a.act, a.H[(size_t)mm * a.K + cc]);
    if (a.scale) v *= a.scale[cc];  // input normaliser (x - mean) * rstd: dx = g * rstd
    a.G[(size_t)mm * a.K + cc] = v;
  }
}

// dW[N x K] = dZ^T X, reduction over M (+ db = sum_m dZ in the blocks of the first K tile).
// Both operands are read down their columns, so the block stages chunks of 128 rows of
// dZ[:, n0:n0+32] and X[:, c0:c0+32] transposed into LDS (coalesced 128-B row segments in,
// packed bf16 pairs out); wave w reduces rows 32w .. 32w+32 of every chunk. The M axis is
// also split over gridDim.z blocks (a 256 x 256 layer has only 64 output tiles): each split
// writes its partial tile to the workspace and the last split to finish -- counted with one
// global atomic per tile -- sums the partials in split order (deterministic) and resets the
// counter for the next launch.
constexpr int kChunk = 128;
constexpr int kChunkPitch = kChunk + 8;
constexpr int kTilePartial = kTile * kTile + kTile;  // dW tile + db slice

template <bool VEC>
__global__ __launch_bounds__(64 * kWaves) void wlin_dw_kernel(WideLinArgs a) {
  __shared__ __attribute__((aligned(16))) __bf16 zt[kTile * kChunkPitch];
  __shared__ __attribute__((aligned(16))) __bf16 xt[kTile * kChunkPitch];
  __shared__ float red[kWaves][kTile][kTile + 1];
  __shared__ float dbr[kTile][kTile + 1];
  __shared__ int is_last;
  const int c0 = blockIdx.x * kTile, n0 = blockIdx.y * kTile, split = blockIdx.z, S = gridDim.z;
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
  const int t = threadIdx.x, q = t & 7, p = t >> 3;
  const int w = t >> 6, l = t & 63, r = l & 31, h = l >> 5;
  const bool do_db = a.db != nullptr && blockIdx.x == 0;
  const int nchunks = (a.M + kChunk - 1) / kChunk;
  f4 dbs = {0.f, 0.f, 0.f, 0.f};
  f32x16 acc = {};
  for (int ch = split; ch < nchunks; ch += S) {
    const int mb = ch * kChunk;
    f4 z[4], x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // rows mb + 2p + (i & 1) + 64 (i >> 1)
      const int row = mb + 2 * p + (i & 1) + 64 * (i >> 1);
      z[i] = load4<VEC>(a.dZ, row, n0 + 4 * q, a.M, a.N);
      x[i] = load4<VEC>(a.X, row, c0 + 4 * q, a.M, a.K);
    }
    if (do_db) dbs += (z[0] + z[1]) + (z[2] + z[3]);  // fp32 (not the bf16 operand)
    __syncthreads();  // the previous chunk's operand reads are done
    stage_pair_t(zt, kChunkPitch, q, 2 * p, z[0], z[1]);
    stage_pair_t(zt, kChunkPitch, q, 64 + 2 * p, z[2], z[3]);
    stage_pair_t(xt, kChunkPitch, q, 2 * p, x[0], x[1]);
    stage_pair_t(xt, kChunkPitch, q, 64 + 2 * p, x[2], x[3]);
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int mo = 32 * w + 16 * ks + 8 * h;
      const bf16x8 A = *reinterpret_cast<const bf16x8*>(zt + r * kChunkPitch + mo);
      const bf16x8 B = *reinterpret_cast<const bf16x8*>(xt + r * kChunkPitch + mo);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A, B, acc, 0, 0, 0);
    }
  }
  if (do_db) {
#pragma unroll
    for (int j = 0; j < 4; ++j) dbr[p][4 * q + j] = dbs[j];
  }
  reduce_tile(acc, red);  // (includes the barrier that publishes dbr)
  float v[4];
  const int i = (4 * t) / kTile, j0 = (4 * t) % kTile;  // 4 consecutive columns per thread
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = (red[0][i][j0 + u] + red[1][i][j0 + u]) + (red[2][i][j0 + u] + red[3][i][j0 + u]);
  float db = 0.f;
  if (do_db && t < kTile) {
    for (int pp = 0; pp < kTile; ++pp) db += dbr[pp][t];
  }
  if (S > 1) {
    // hand-off without L2 write-back / invalidate fences (MI355X_MICROARCH inter-workgroup
    // visibility, table row 1): sc1 stores, every storing wave's vmcnt(0), a barrier, one
    // agent-scope add per workgroup; the workgroup whose add returns S - 1 reads every
    // partial with sc1 loads behind a barrier
    float* part = a.ws + ((size_t)split * gridDim.x * gridDim.y + tile) * kTilePartial;
    st_sc1_x4(part + 4 * t, f4{v[0], v[1], v[2], v[3]});
    if (do_db && t < kTile) __hip_atomic_store(part + kTile * kTile + t, db, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) is_last = atomicAdd(a.cnt + tile, 1) == S - 1;
    __syncthreads();
    if (!is_last) return;
    f4 acc4 = {0.f, 0.f, 0.f, 0.f};
    db = 0.f;
    const size_t stride = (size_t)gridDim.x * gridDim.y * kTilePartial;
    const float* p0 = a.ws + (size_t)tile * kTilePartial;
    for (int s0 = 0; s0 < S; s0 += 8) {  // 8 loads in flight, summed in split order
      f4 pv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) pv[u] = ld_sc1_x4(p0 + (size_t)min(s0 + u, S - 1) * stride + 4 * t);
      wait_vm8(pv);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (s0 + u < S) acc4 += pv[u];
      if (do_db && t < kTile)
        for (int u = s0; u < min(S, s0 + 8); ++u)
          db += __hip_atomic_load(p0 + (size_t)u * stride + kTile * kTile + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = acc4[u];
    if (t == 0) __hip_atomic_store(a.cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int nn = n0 + i;
  if (nn < a.N) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int cc = c0 + j0 + u;
      if (cc >= a.K) continue;
      float* dst = a.dW + (size_t)nn * a.K + cc;
      *dst = a.accumulate ? *dst + v[u] : v[u];
    }
  }
  if (do_db && t < kTile && n0 + t < a.N) {
    float* dst = a.db + n0 + t;
    *dst = a.accumulate ? *dst + db : db;
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

hipError_t wlin_forward(const WideLinArgs& a, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  const dim3 grid((a.N + kTile - 1) / kTile, (a.M + kTile - 1) / kTile), block(64 * kWaves);
  const bool vec = a.K % 8 == 0 && aligned16(a.X) && aligned16(a.W);
  if (vec) hipLaunchKernelGGL(wlin_fwd_kernel<true>, grid, block, 0, s, a);
  else hipLaunchKernelGGL(wlin_fwd_kernel<false>, grid, block, 0, s, a);
  return hipGetLastError();
}

size_t wlin_dx_lds_bytes(int N) {
  const int npad = (N + 63) / 64 * 64;
  return sizeof(float) * kWaves * kTile * (kTile + 1) + sizeof(__bf16) * kTile * (npad + 8);
}

hipError_t wlin_backward_x(const WideLinArgs& a, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  const dim3 grid((a.K + kTile - 1) / kTile, (a.M + 2 * kTile - 1) / (2 * kTile)), block(64 * kWaves);
  const size_t lds = wlin_dx_lds_bytes(a.N);
  static bool big_lds = [] {  // N up to 1024: the W strip exceeds the 64 KB default
    const int cap = 160 * 1024;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&wlin_dx_kernel<true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, cap) == hipSuccess &&
           hipFuncSetAttribute(reinterpret_cast<const void*>(&wlin_dx_kernel<false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, cap) == hipSuccess;
  }();
  if (!big_lds && lds > 64 * 1024) return hipErrorInvalidConfiguration;
  const bool vec = a.N % 8 == 0 && a.K % 4 == 0 && aligned16(a.dZ) && aligned16(a.W);
  if (vec) hipLaunchKernelGGL(wlin_dx_kernel<true>, grid, block, lds, s, a);
  else hipLaunchKernelGGL(wlin_dx_kernel<false>, grid, block, lds, s, a);
  return hipGetLastError();
}

int wlin_dw_tiles(int N, int K) { return ((K + kTile - 1) / kTile) * ((N + kTile - 1) / kTile); }

int wlin_dw_splits(int M, int N, int K) {
  const int tiles = wlin_dw_tiles(N, K), nchunks = (M + kChunk - 1) / kChunk;
  const int want = (512 + tiles - 1) / tiles;  // ~2 blocks per CU
  return max(1, min(min(nchunks, want), 64));
}

size_t wlin_dw_ws_floats(int M, int N, int K) {
  const int S = wlin_dw_splits(M, N, K);
  return S > 1 ? (size_t)S * wlin_dw_tiles(N, K) * kTilePartial : 0;
}

hipError_t wlin_backward_w(const WideLinArgs& a, hipStream_t s) {
  if (a.M <= 0) return hipSuccess;
  const int S = wlin_dw_splits(a.M, a.N, a.K);
  if (S > 1 && (a.ws == nullptr || a.cnt == nullptr)) return hipErrorInvalidValue;
  const dim3 grid((a.K + kTile - 1) / kTile, (a.N + kTile - 1) / kTile, S), block(64 * kWaves);
  const bool vec = a.N % 4 == 0 && a.K % 4 == 0 && aligned16(a.dZ) && aligned16(a.X);
  if (vec) hipLaunchKernelGGL(wlin_dw_kernel<true>, grid, block, 0, s, a);
  else hipLaunchKernelGGL(wlin_dw_kernel<false>, grid, block, 0, s, a);
  return hipGetLastError();
}

}  // namespace ia

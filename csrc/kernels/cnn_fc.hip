// Backward of the NatureCNN feature layer Linear(C*H*W -> NH) + ReLU on bf16 MFMA tiles, for
// training steps whose conv trunk runs on conv.hip (ops/conv.py conv_stack_fc; BC / DAgger
// minibatches, reference bc.py:100-130 through SB3's NatureCNN).
//
// The forward is cnn_fc (cnn_infer.hip) on the conv trunk's NHWC bf16 output and the weight
// packed to (h, w, c) column order, so there is no flatten permute in either direction. At the
// BC batch (32 rows) the torch form is three fp32 hipBLASLt GEMMs (~30 us, each reading or
// writing the 6.4 MB fp32 weight), a permute copy each way, ReLU / bias kernels. Here:
//   fc_wgrad  dW[n][col] = sum_m dZ[m][n] X[m][k(col)],  db[n] = sum_m dZ[m][n],
//             dZ = dH * [h > 0] formed on the fly. Block = 64 n x 64 torch columns (4 waves
//             x 4 16x16 tiles); per 32-row step dZ^T and X are staged transposed in LDS so both MFMA
//             operands read 8 consecutive rows; dW rows are stored contiguously.
//   fc_dgrad  dX[m][k] = sum_n dZ[m][n] Wt[k][n] (Wt: the weight packed [(h, w, c)][NH], dZ
//             in bf16 from fc_wgrad), bf16 out in NHWC order = the conv trunk's upstream
//             gradient. One wave per 16x16 tile, 8 loads in flight per k-batch.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "ia/mfma.h"
#include "launchers.h"

namespace ia {
namespace {

// db[col] = sum_m dH[m][col] * [Hout[m][col] > 0] in row order. The loads of 16 rows are issued
// before the first add: a one-load-per-iteration loop paid M dependent L2 round trips (~5 us at
// M = 32) in the bias lane's tail. Same additions in the same order (bitwise).
__device__ __forceinline__ float relu_bias_sum(const float* __restrict__ dH, const float* __restrict__ Hout, int M, int NH,
                                               int col) {
  float s = 0.f;
  for (int m0 = 0; m0 < M; m0 += 16) {
    float z[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int m = m0 + u;
      z[u] = 0.f;
      if (m < M) {
        const size_t o = (size_t)m * NH + col;
        z[u] = Hout[o] > 0.f ? dH[o] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 16; ++u)
      if (m0 + u < M) s += z[u];
  }
  return s;
}

// Block = 64 n x 64 torch columns (4 waves, wave w owns n rows 16w..16w+15 and four 16x16
// column tiles). The 64 columns are consecutive in torch's (c, h, w) order, so every dW row
// segment is one 256-B run; they are gathered from X through the column -> NHWC index map while
// staged, once per block for all 4 waves. 4 column tiles per block (was 1): the dZ staging --
// every block re-reads the 64 x M slab of dH / H -- drops 4x (~26 -> ~6 MB of L2 reads per
// step at NatureCNN / batch 32). The blocks of the first column tile also write dZ in bf16 (the
// data-gradient operand) and db. Same MFMA per dW element as before (bitwise).
constexpr int kFcCT = 4;  // 16-column tiles per block

__global__ __launch_bounds__(256) void fc_wgrad_kernel(const bf16* __restrict__ X, const float* __restrict__ dH,
                                                       const float* __restrict__ Hout, float* __restrict__ dW,
                                                       float* __restrict__ db, bf16* __restrict__ dZb, int M, int K, int NH,
                                                       int C, int HW) {
  __shared__ __attribute__((aligned(16))) bf16 zs[64][40];            // dZ^T chunk [n][m] (+8 pad)
  __shared__ __attribute__((aligned(16))) bf16 xs[16 * kFcCT][40];    // X^T chunk [col][m]
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int col0 = blockIdx.x * 16 * kFcCT, n0 = blockIdx.y * 64;
  const bool first = blockIdx.x == 0;
  // this thread's staged (column, row) elements of X: 64 columns x 4 rows per pass, 8 passes
  const int xc = tid & 63, xm = tid >> 6;
  const int xcol = col0 + xc, xch = xcol / HW;
  const int koff = (xcol - xch * HW) * C + xch;
  f32x4 acc[kFcCT];
#pragma unroll
  for (int t = 0; t < kFcCT; ++t) acc[t] = zero4();
  for (int m0 = 0; m0 < M; m0 += 32) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // dZ^T: 64 n x 32 m, coalesced along n
      const int i = tid + 256 * e, nn = i & 63, mm = i >> 6;
      const int m = m0 + mm;
      float z = 0.f;
      if (m < M) {
        const size_t o = (size_t)m * NH + n0 + nn;
        z = Hout[o] > 0.f ? dH[o] : 0.f;
        if (first && dZb) dZb[o] = (bf16)z;
      }
      zs[nn][mm] = (bf16)z;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {  // X^T: 64 columns x 32 m
      const int mm = xm + 4 * e, m = m0 + mm;
      xs[xc][mm] = m < M ? X[(size_t)m * K + koff] : (bf16)0.f;
    }
    __syncthreads();
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(&zs[w * 16 + (l & 15)][(l >> 4) * 8]);
#pragma unroll
    for (int t = 0; t < kFcCT; ++t) {
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(&xs[16 * t + (l & 15)][(l >> 4) * 8]);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[t], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < kFcCT; ++t) {
    const int col = col0 + 16 * t + (l & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) dW[(size_t)(n0 + w * 16 + 4 * (l >> 4) + i) * K + col] = acc[t][i];
  }
  if (first && tid < 64) db[n0 + tid] = relu_bias_sum(dH, Hout, M, NH, n0 + tid);  // fixed row order
}

// Channel-aligned variant: a block owns kChG whole channels, i.e. the contiguous torch columns
// [c0 * HW, (c0 + kChG) * HW), for 64 n rows. Its X operand is then kChG consecutive NHWC
// channels per (row, position): one 16-B load each. The 64-consecutive-column blocks above load
// X element by element, every element from a different 128-B line (NHWC stride C): at NatureCNN
// / batch 32 that is ~100 MB of L2 line traffic per step against ~13 MB here. 8 waves: wave w
// owns n rows 16 (w & 3) .. + 15 and the column tiles of parity w >> 2. Same MFMA per dW element
// (same operands, same 32-row m chunks), so dW is bitwise the other kernel's.
constexpr int kChG = 8;          // channels per block
constexpr int kChMaxCols = 416;  // kChG * HW bound: 26 tiles of 16 columns
constexpr int kChTilesW = 13;    // tiles per wave (parity split)
constexpr int kChXIt = 4;        // X loads per thread per 32-row chunk: ceil(32 * 52 / 512)
constexpr int kChHwSplit = 4;  // HW position groups per (channel group, n block): 256 blocks at NatureCNN (64 before; BC step -1 us, profiles/r6_bc_step.md)

// (bx, by, bz): channel group, n block, position group. (A one-launch FC backward -- these blocks
// plus the data gradient forming its dZ from dH / Hout -- measured slower: 25 us vs 12 + 6 for
// the two launches, call W, profiles/r6_bc_step.md.)
__device__ __forceinline__ void fc_wgrad_ch_body(const bf16* __restrict__ X, const float* __restrict__ dH,
                                                 const float* __restrict__ Hout, float* __restrict__ dW,
                                                 float* __restrict__ db, bf16* __restrict__ dZb, int M, int K, int NH,
                                                 int C, int HW, int hws, int bx, int by, int bz) {
  __shared__ __attribute__((aligned(16))) bf16 zs[64][40];          // dZ^T chunk [n][m] (+8 pad)
  __shared__ __attribute__((aligned(16))) bf16 xs[kChMaxCols][40];  // X^T chunk [column][m]
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int wn = w & 3, par = w >> 2;
  const int c0 = bx * kChG, n0 = by * 64;
  // bz: positions [hw0, hw0 + hwn) of the kChG channels (a block's columns: channel g, position
  // hw0 + j -> local column g * hwn + j)
  const int hw0 = bz * hws, hwn = HW - hw0 < hws ? HW - hw0 : hws;
  const int ncols = kChG * hwn, ntiles = (ncols + 15) / 16, nx = 32 * hwn;
  const bool first = bx == 0 && bz == 0;
  f32x4 acc[kChTilesW];
#pragma unroll
  for (int j = 0; j < kChTilesW; ++j) acc[j] = zero4();
  for (int m0 = 0; m0 < M; m0 += 32) {
    bf16x8 xv[kChXIt];
#pragma unroll
    for (int e = 0; e < kChXIt; ++e) {  // all of this thread's X loads in flight first
      const int i = tid + 512 * e, mm = i / hwn, hw = hw0 + i - mm * hwn, m = m0 + mm;
      xv[e] = (i < nx && m < M) ? *reinterpret_cast<const bf16x8*>(X + (size_t)m * K + (size_t)hw * C + c0) : bf16x8{};
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {  // dZ^T: 64 n x 32 m, coalesced along n
      const int i = tid + 512 * e, nn = i & 63, mm = i >> 6;
      const int m = m0 + mm;
      float z = 0.f;
      if (m < M) {
        const size_t o = (size_t)m * NH + n0 + nn;
        z = Hout[o] > 0.f ? dH[o] : 0.f;
        if (first) dZb[o] = (bf16)z;
      }
      zs[nn][mm] = (bf16)z;
    }
#pragma unroll
    for (int e = 0; e < kChXIt; ++e) {
      const int i = tid + 512 * e, mm = i / hwn, hl = i - mm * hwn;
      if (i < nx) {
#pragma unroll
        for (int g = 0; g < kChG; ++g) xs[g * hwn + hl][mm] = xv[e][g];
      }
    }
    __syncthreads();
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(&zs[wn * 16 + (l & 15)][(l >> 4) * 8]);
#pragma unroll
    for (int j = 0; j < kChTilesW; ++j) {
      const int t = par + 2 * j;
      if (t < ntiles) {  // (wave-uniform) the last tile's columns past ncols are computed, never stored
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(&xs[16 * t + (l & 15)][(l >> 4) * 8]);
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < kChTilesW; ++j) {
    const int lc = 16 * (par + 2 * j) + (l & 15);  // local column: channel lc / hwn, position hw0 + lc % hwn
    if (lc < ncols) {
      const int g = lc / hwn;
      const int col = (c0 + g) * HW + hw0 + (lc - g * hwn);
#pragma unroll
      for (int i = 0; i < 4; ++i) dW[(size_t)(n0 + wn * 16 + 4 * (l >> 4) + i) * K + col] = acc[j][i];
    }
  }
  if (first && tid < 64) db[n0 + tid] = relu_bias_sum(dH, Hout, M, NH, n0 + tid);  // fixed row order
}

__global__ __launch_bounds__(512) void fc_wgrad_ch_kernel(const bf16* __restrict__ X, const float* __restrict__ dH,
                                                          const float* __restrict__ Hout, float* __restrict__ dW,
                                                          float* __restrict__ db, bf16* __restrict__ dZb, int M, int K,
                                                          int NH, int C, int HW, int hws) {
  fc_wgrad_ch_body(X, dH, Hout, dW, db, dZb, M, K, NH, C, HW, hws, blockIdx.x, blockIdx.y, blockIdx.z);
}

// One wave = 16 rows x 16 NHWC columns; the n loop is issued 4 k-steps (8 loads) at a time
// so the L2 round trips overlap (the wave reads 16 KB of Wt).
__device__ __forceinline__ void fc_dgrad_body(const bf16* __restrict__ dZb, const bf16* __restrict__ Wt,
                                              bf16* __restrict__ dX, int M, int K, int NH, const bf16* __restrict__ Xm,
                                              int wave) {
  const int l = threadIdx.x & 63;
  const int ktiles = K / 16;
  const int mt = wave / ktiles, kt = wave - mt * ktiles;
  const int m0 = mt * 16, k0 = kt * 16;
  if (m0 >= M) return;
  const int m = m0 + (l & 15);
  const bool mv = m < M;
  const int nq = (l >> 4) * 8;
  const size_t ao = (size_t)(mv ? m : 0) * NH + nq;
  const bf16* ar = dZb + ao;
  const bf16* br = Wt + (size_t)(k0 + (l & 15)) * NH + nq;
  f32x4 acc = zero4();
  for (int n0 = 0; n0 < NH; n0 += 128) {
    bf16x8 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const bool ok = n0 + 32 * u < NH;
      a[u] = ok ? *reinterpret_cast<const bf16x8*>(ar + n0 + 32 * u) : bf16x8{};
      b[u] = ok ? *reinterpret_cast<const bf16x8*>(br + n0 + 32 * u) : bf16x8{};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!mv) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[u][j] = (bf16)0.f;
      }
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[u], acc, 0, 0, 0);
    }
  }
  const int k = k0 + (l & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + 4 * (l >> 4) + i;
    if (row < M) {
      float v = acc[i];
      if (Xm && !((float)Xm[(size_t)row * K + k] > 0.f)) v = 0.f;  // top-layer ReLU mask (same select as load_dz8)
      dX[(size_t)row * K + k] = (bf16)v;
    }
  }
}

__global__ __launch_bounds__(256) void fc_dgrad_kernel(const bf16* __restrict__ dZb, const bf16* __restrict__ Wt,
                                                       bf16* __restrict__ dX, int M, int K, int NH,
                                                       const bf16* __restrict__ Xm) {
  fc_dgrad_body(dZb, Wt, dX, M, K, NH, Xm, blockIdx.x * 4 + (threadIdx.x >> 6));
}

}  // namespace

bool fc_train_ok(int M, int K, int NH, int C, int HW) {
  return M > 0 && NH > 0 && NH % 64 == 0 && K % 64 == 0 && C > 0 && HW > 0 && K == C * HW;
}

hipError_t fc_backward(const void* X, const float* dH, const float* Hout, const void* Wt, float* dW, float* db, void* dX,
                       void* dZb, int M, int K, int NH, int C, int HW, hipStream_t s, bool mask_dx) {
  if (!fc_train_ok(M, K, NH, C, HW)) return hipErrorInvalidValue;
  // channel-aligned blocks (16-B NHWC loads) when X allows them, else the 64-column blocks
  const bool ch = C % kChG == 0 && kChG * HW <= kChMaxCols && reinterpret_cast<uintptr_t>(X) % 16 == 0;
  // each block's positions: a split of the HW positions over gridDim.z (more blocks than the
  // C / kChG x NH / 64 = 64 of NatureCNN, each with fewer column tiles)
  const int hws = (HW + kChHwSplit - 1) / kChHwSplit;
  const int gx = C / kChG, gy = NH / 64, gz = (HW + hws - 1) / hws;
  if (ch)
    hipLaunchKernelGGL(fc_wgrad_ch_kernel, dim3(gx, gy, gz), dim3(512), 0, s,
                       static_cast<const bf16*>(X), dH, Hout, dW, db, static_cast<bf16*>(dZb), M, K, NH, C, HW, hws);
  else
    hipLaunchKernelGGL(fc_wgrad_kernel, dim3(K / (16 * kFcCT), NH / 64), dim3(256), 0, s, static_cast<const bf16*>(X), dH, Hout,
                       dW, db, static_cast<bf16*>(dZb), M, K, NH, C, HW);
  if (dX) {
    const int waves = ((M + 15) / 16) * (K / 16);
    hipLaunchKernelGGL(fc_dgrad_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, static_cast<const bf16*>(dZb),
                       static_cast<const bf16*>(Wt), static_cast<bf16*>(dX), M, K, NH,
                       mask_dx ? static_cast<const bf16*>(X) : nullptr);
  }
  return hipGetLastError();
}

}  // namespace ia

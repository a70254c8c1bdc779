// CDNA4 (gfx950) MFMA tile primitives for the tiny-MLP kernels.
//
// Everything here is wave-level: one 64-lane wave computes one 16x16 fp32
// output tile with v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulate).
//
// Operand convention (see cdna_hip_programming.md §3, "A/B operand lane maps"):
//   lane l holds A[m = l&15][k = 8*(l>>4) + j] and B[k = 8*(l>>4) + j][n = l&15],
//   j = 0..7, so BOTH operands are read as 16 contiguous bytes from an LDS
//   image whose *contraction index is contiguous*:
//     A  is stored  [m][k]   (row-major, "a")
//     B  is stored  [n][k]   (i.e. B^T row-major, "bt")
//   Output C/D: lane l holds C[m = 4*(l>>4) + i][n = l&15], i = 0..3.
// Row strides are padded to (multiple of 32) + 8 bf16 so that the 16 lanes of
// a ds_read_b128 group land on distinct bank slots.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ia/common.h"

namespace ia {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// LDS-typed (address_space 3) views: images reached through these compile to ds_read /
// ds_write. A generic pointer into LDS compiles to FLAT accesses, which count in vmcnt as
// well as lgkmcnt (every LDS wait then also waits for outstanding global memory ops).
typedef __attribute__((address_space(3))) bf16 lbf;
typedef __attribute__((address_space(3))) bf16x8 lbf8;
typedef __attribute__((address_space(3))) bf16x4 lbf4;
typedef __attribute__((address_space(3))) float lfl;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }


__device__ __forceinline__ bf16 to_bf16(float x) { return (bf16)x; }
__device__ __forceinline__ float from_bf16(bf16 x) { return (float)x; }

// acc += A[16 x K] * B[K x 16]; a -> A row 0 (ld lda), bt -> B^T row 0 (ld ldb).
// K must be a multiple of 32 (pad regions of both images must hold zeros).
__device__ __forceinline__ f32x4 mma_16x16(const bf16* a, int lda, const bf16* bt, int ldb, int K, f32x4 acc) {
  const int l = lane_id();
  const int r = l & 15;
  const int kq = (l >> 4) * 8;
  const bf16* ap = a + r * lda + kq;
  const bf16* bp = bt + r * ldb + kq;
  for (int k = 0; k < K; k += 32) {
    bf16x8 av = *reinterpret_cast<const bf16x8*>(ap + k);
    bf16x8 bv = *reinterpret_cast<const bf16x8*>(bp + k);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
  return acc;
}

// the same on LDS-typed images (ds_read_b128 operands)
__device__ __forceinline__ f32x4 mma_16x16(const lbf* a, int lda, const lbf* bt, int ldb, int K, f32x4 acc) {
  const int l = lane_id();
  const int r = l & 15;
  const int kq = (l >> 4) * 8;
  const lbf* ap = a + r * lda + kq;
  const lbf* bp = bt + r * ldb + kq;
  for (int k = 0; k < K; k += 32) {
    bf16x8 av = *(const lbf8*)(ap + k);
    bf16x8 bv = *(const lbf8*)(bp + k);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
  }
  return acc;
}

__device__ __forceinline__ f32x4 zero4() {
  f32x4 z = {0.f, 0.f, 0.f, 0.f};
  return z;
}

// Output coordinates of accumulator element i for this lane.
__device__ __forceinline__ int acc_row(int i) { return 4 * (lane_id() >> 4) + i; }
__device__ __forceinline__ int acc_col() { return lane_id() & 15; }

__device__ __forceinline__ float apply_act(int act, float x) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_TANH: return tanhf(x);
    case ACT_LEAKY_RELU: return x > 0.f ? x : 0.01f * x;
    case ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    default: return x;
  }
}
// derivative expressed through the activation OUTPUT h (and pre-activation sign for relu-likes)
__device__ __forceinline__ float act_grad_from_out(int act, float h) {
  switch (act) {
    case ACT_RELU: return h > 0.f ? 1.f : 0.f;
    case ACT_TANH: return 1.f - h * h;
    case ACT_LEAKY_RELU: return h > 0.f ? 1.f : 0.01f;
    case ACT_SIGMOID: return h * (1.f - h);
    default: return 1.f;
  }
}

// Block-cooperative zero fill of an LDS region (bytes multiple of 16).
__device__ __forceinline__ void lds_zero(void* p, int bytes) {
  uint4* q = reinterpret_cast<uint4*>(p);
  const uint4 z = {0u, 0u, 0u, 0u};
  for (int i = threadIdx.x; i < bytes / 16; i += blockDim.x) q[i] = z;
}

}  // namespace ia

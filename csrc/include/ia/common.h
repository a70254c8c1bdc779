// Host/device-neutral helpers (safe to include from g++-compiled binding TUs).
#pragma once
#include <hip/hip_runtime.h>

namespace ia {

__host__ __device__ __forceinline__ int pad16(int x) { return (x + 15) & ~15; }
__host__ __device__ __forceinline__ int pad32(int x) { return (x + 31) & ~31; }
// LDS leading dimension (bf16 elements) for a K-contiguous MFMA operand image:
// K padded to the 32-wide k-step plus 8 elements (16 B) so the 16 lanes of a
// ds_read_b128 group start on different bank slots.
__host__ __device__ __forceinline__ int ld_for_k(int k) { return pad32(k) + 8; }

enum Act : int { ACT_IDENTITY = 0, ACT_RELU = 1, ACT_TANH = 2, ACT_LEAKY_RELU = 3, ACT_SIGMOID = 4 };

}  // namespace ia

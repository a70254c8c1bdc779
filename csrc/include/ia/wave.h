// Single-wave device helpers shared by the rollout-chain kernel (rollout.hip) and the
// per-row post-pass kernels (engine.hip): LDS-typed pointers, intra-wave ordering,
// lane broadcasts and reductions, fast activations, the counter-based key hash.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ia/common.h"
#include "ia/mfma.h"
#include "ia/rng.h"

namespace ia {

// LDS pointers typed address_space(3) (32-bit, ds_read/ds_write, counted in lgkmcnt --
// a generic/flat access would also wait on vmcnt, i.e. behind every global store).
typedef __attribute__((address_space(3))) float lf;
typedef float f32v4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f32v4 lf4;
typedef __attribute__((address_space(3))) int li;

// One wave per workgroup: a wave's LDS accesses complete in issue order, so a
// wavefront-scope fence (compiler ordering point) replaces __syncthreads(), whose
// workgroup-scope release would also wait for every outstanding global store.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float bcast(float v, int k) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}


// DPP lane moves (bound_ctrl: out-of-row sources read 0).
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}
// Sum over lanes 0..7 (the joint lanes; lanes 8.. must hold 0 in each 16-lane row's
// upper half for rows != 0 to not matter -- only lane 7 of row 0 is read): two
// quad_perm butterflies give quad sums, row_shr:4 adds quad 0 into quad 1.
__device__ __forceinline__ float sum_lanes8(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x114>(v);  // row_shr:4
  return bcast(v, 7);
}

// Sum over the 16 lanes of each DPP row, result in every lane of the row: pair and quad
// butterflies (quad_perm), then row_half_mirror (quad 0 <-> quad 1 of each 8-lane half)
// and row_mirror (half 0 <-> half 1). Four v_add_f32_dpp, no LDS traffic (a __shfl_xor
// butterfly is four ds_bpermute round trips).
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}
__device__ __forceinline__ float row_max16(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  v = fmaxf(v, dpp<0x140>(v));
  return v;
}

// Lane i <-> lane i ^ 16 (gfx950 v_permlane16_swap: odd rows of the first operand trade
// places with even rows of the second); returns own + partner / max(own, partner).
__device__ __forceinline__ float add_rows16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float max_rows16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max_halves(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Lane i <-> lane i ^ 32 (gfx950 v_permlane32_swap: lanes 32-63 of the first operand
// trade places with lanes 0-31 of the second); returns own + partner in every lane.
__device__ __forceinline__ float add_halves(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// Whole-wave sum / max in every lane: DPP row reduction, then the two cross-row swaps.
__device__ __forceinline__ float wave_sum(float v) { return add_halves(add_rows16(row_sum16(v))); }
__device__ __forceinline__ float wave_max(float v) { return max_halves(max_rows16(row_max16(v))); }

// tanh as 1 - 2 / (exp(2x) + 1) on v_exp_f32 / v_rcp_f32 (|err| ~2e-7 abs; the hardware
// reciprocal, not the ~11-instruction IEEE divide sequence)
__device__ __forceinline__ float act_fast(int act, float x) {
  if (act == ACT_TANH) {
    const float e = __expf(2.f * fminf(fmaxf(x, -15.f), 15.f));
    return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
  }
  return apply_act(act, x);
}

__device__ __forceinline__ uint64_t hash3(uint64_t a, uint64_t b, uint64_t c) {
  uint64_t s = a ^ (0x9E3779B97F4A7C15ull * (b + 1)) ^ (0xC2B2AE3D27D4EB4Full * (c + 1));
  splitmix64(s);
  return s;
}

// Per-step, per-lane noise streams of the rollout (action sampling / exploration).
// key = hash3(seed, env, global step); continuous dims and categorical slots xor in
// their lane, exploration draws use a separate tweak.
constexpr uint64_t kLaneTweak = 0xD6E8FEB86659FD93ull;
constexpr uint64_t kExploreTweak = 0x5851F42D4C957F2Dull;
constexpr uint64_t kExploreDiscreteTweak = 0x2545F4914F6CDD1Dull;

__device__ __forceinline__ float softplus_f(float x) { return x > 0.f ? x + log1pf(expf(-x)) : log1pf(expf(x)); }

}  // namespace ia

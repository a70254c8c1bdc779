// Counter-free per-stream RNG usable from host code and from HIP kernels.
//
// Every batched environment / sampler owns one 64-bit state per stream so that
// env i on rank r is reproducible regardless of how many envs or ranks exist
// (the reference derives per-env seeds in util/util.py:181-199 `make_seeds`).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define IA_HD __host__ __device__ __forceinline__

namespace ia {

IA_HD uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform in [0, 1)
IA_HD float uniform01(uint64_t& s) {
  return (float)(splitmix64(s) >> 40) * (1.0f / 16777216.0f);
}

IA_HD float uniform(uint64_t& s, float lo, float hi) { return lo + (hi - lo) * uniform01(s); }

// standard normal via Box-Muller (one sample, discards the pair)
IA_HD float normal01(uint64_t& s) {
  float u1 = uniform01(s);
  float u2 = uniform01(s);
  u1 = u1 < 1e-7f ? 1e-7f : u1;
  return sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
}

IA_HD uint64_t seed_stream(uint64_t seed, uint64_t stream) {
  uint64_t s = seed ^ (0xD1B54A32D192ED03ull * (stream + 1));
  splitmix64(s);
  return s;
}

}  // namespace ia

// Host launch entry points of every HIP kernel (raw pointers + stream only, so
// that the torch-facing binding TUs never include device code and the kernel
// TUs never include torch headers).  All launchers are graph-capture safe: no
// allocation, no synchronisation.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ia/engine.h"
#include "ia/tmlp.h"

namespace ia {

// ---- tmlp.hip: fused tiny-MLP
int tmlp_waves_for(const MLPDesc& d);
size_t tmlp_slab_floats(const MLPDesc& d, int B);
hipError_t tmlp_forward(const MLPDesc& d, const float* X, int B, float* Y, hipStream_t s);
hipError_t tmlp_backward(const MLPDesc& d, const float* X, const float* dY, int B, float* dX, const MLPGrads& g,
                         float* slab, hipStream_t s);

// ---- rl.hip: GAE scan over [T, N]
hipError_t gae_launch(const float* rew, const float* val, const float* starts, const float* last_val, const float* dones,
                      int T, int N, float gamma, float lam, float* adv, float* ret, hipStream_t s);

// ---- pref.hip: Bradley-Terry preference loss over fragment pairs
hipError_t pref_loss_fwd(const float* r1, const float* r2, const float* prefs, int P, int L, float discount,
                         float threshold, float noise, float* probs, float* losses, float* coef, hipStream_t s);
hipError_t pref_loss_bwd(const float* coef, const float* gout, int P, int L, float discount, float* d1, float* d2,
                         hipStream_t s);

// ---- engine.hip: device-resident rollout (policy + env + learned reward)
size_t rollout_lds_bytes(const RolloutArgs& a);
hipError_t rollout_launch(const RolloutArgs& a, hipStream_t s);

// ---- ppo.hip: persistent PPO update
size_t ppo_lds_bytes(const PPOArgs& a);
hipError_t ppo_launch(const PPOArgs& a, hipStream_t s);

}  // namespace ia

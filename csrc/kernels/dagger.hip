// Device env stepping for the DAgger collector (imitation_amd/engine/dagger.py).
//
// The reference collects DAgger rounds on the host: InteractiveTrajectoryCollector
// wraps a (Subproc)VecEnv, every step crosses a pipe per env, frames are copied to the
// device twice (expert and learner forward) and back (src/imitation/algorithms/
// dagger.py:151-287). Here the env lives in HBM: one workgroup per env applies the
// executed (β-mixed) action with the same IA_HD physics the host BatchedEnv runs
// (csrc/include/ia/envs.h), so for equal actions the device trajectory is the host's
// bit for bit; Pong frames are rendered straight into the observation tensor the two
// CNN policies read next.
//
// Frame stack: HWC uint8 with 4 channels = one 32-bit word per pixel, so the
// VecFrameStack shift (channels k <- k+1, newest frame into channel 3) is one
// (old >> 8) | (v << 24) per pixel and a reset stack is v * 0x01010101.
//
// Per step and env (mode 0): step -> TimeLimit -> render; on episode end the
// terminal observation is copied to its slot, the env is reset and re-rendered --
// exactly BatchedEnv::step (csrc/runtime/vec_env.cpp). Mode 1 resets every env.
#include <hip/hip_runtime.h>

#include "launchers.h"

namespace ia {
namespace {

constexpr int kThreads = 1024;  // 7056 pixels: ~7 per thread
constexpr int kPix = kPongH * kPongW;

// rec (optional): receives the stack as it was before this render
__device__ __forceinline__ void render(const float* s, uint32_t* frame, bool reset_stack, uint32_t* rec = nullptr) {
  for (int p = threadIdx.x; p < kPix; p += kThreads) {
    const uint32_t v = pong_pixel(s, p / kPongW, p % kPongW);
    const uint32_t old = frame[p];
    if (rec) rec[p] = old;
    frame[p] = reset_stack ? v * 0x01010101u : ((old >> 8) | (v << 24));
  }
}

__global__ __launch_bounds__(kThreads) void dagger_env_kernel(DaggerEnvArgs a) {
  __shared__ int s_done;
  __shared__ float s_state[kMaxState];
  const int n = blockIdx.x;
  const bool img = a.P.kind == ENV_PONG;
  float* st = a.state + (size_t)n * a.sdim;
  uint32_t* frame = img ? reinterpret_cast<uint32_t*>(a.obs_u8 + (size_t)n * kPix * kPongStack) : nullptr;
  if (a.mode == 1) {  // reset all
    if (threadIdx.x == 0) {
      uint64_t r = a.rng[n];
      env_reset(a.P, st, r);
      a.rng[n] = r;
      a.elapsed[n] = 0;
      a.ep_ret[n] = 0.f;
      for (int k = 0; k < a.sdim; ++k) s_state[k] = st[k];
      if (!img) env_obs(a.P, st, a.obs_f + (size_t)n * a.P.obs_dim);
    }
    __syncthreads();
    if (img) render(s_state, frame, true);
    return;
  }
  if (threadIdx.x == 0) {
    float act[kMaxJoints];
    if (a.act_i) {
      act[0] = (float)a.act_i[n];
    } else {
      for (int k = 0; k < a.P.act_dim; ++k) act[k] = a.act_f[(size_t)n * a.P.act_dim + k];
    }
    uint64_t r = a.rng[n];
    int term = 0;
    const float rew = env_step(a.P, st, act, &term, r);
    const int t = a.elapsed[n] + 1;
    const bool trunc = !term && a.max_steps > 0 && t >= a.max_steps;
    const float ret = a.ep_ret[n] + rew;
    a.rew[n] = rew;
    a.term[n] = (uint8_t)term;
    a.trunc[n] = (uint8_t)trunc;
    const bool done = term || trunc;
    a.ep_ret_out[n] = done ? ret : 0.f;
    a.ep_len_out[n] = done ? t : 0;
    for (int k = 0; k < a.sdim; ++k) s_state[k] = st[k];
    if (!img) {
      float* o = a.obs_f + (size_t)n * a.P.obs_dim;
      if (a.obs_rec)
        for (int k = 0; k < a.P.obs_dim; ++k) static_cast<float*>(a.obs_rec)[(size_t)n * a.P.obs_dim + k] = o[k];
      env_obs(a.P, st, o);
      if (done) {
        for (int k = 0; k < a.P.obs_dim; ++k) a.term_obs_f[(size_t)n * a.P.obs_dim + k] = o[k];
        env_reset(a.P, st, r);
        env_obs(a.P, st, o);
      }
    } else if (done) {
      env_reset(a.P, st, r);  // st now holds the new episode; s_state the terminal state
    }
    a.rng[n] = r;
    a.elapsed[n] = done ? 0 : t;
    a.ep_ret[n] = done ? 0.f : ret;
    s_done = done;
  }
  __syncthreads();
  if (!img) return;
  uint32_t* rec = a.obs_rec ? static_cast<uint32_t*>(a.obs_rec) + (size_t)n * kPix : nullptr;
  render(s_state, frame, false, rec);  // the post-step frame (pre-step stack -> rec)
  if (s_done) {
    __syncthreads();
    uint32_t* tobs = reinterpret_cast<uint32_t*>(a.term_obs_u8 + (size_t)n * kPix * kPongStack);
    for (int p = threadIdx.x; p < kPix; p += kThreads) tobs[p] = frame[p];
    __syncthreads();
    if (threadIdx.x == 0)
      for (int k = 0; k < a.sdim; ++k) s_state[k] = st[k];
    __syncthreads();
    render(s_state, frame, true);
  }
}

}  // namespace

hipError_t dagger_env_step(const DaggerEnvArgs& a, hipStream_t s) {
  if (a.N <= 0) return hipSuccess;
  if (a.sdim > kMaxState || (a.P.kind != ENV_PONG && a.P.obs_dim <= 0)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(dagger_env_kernel, dim3(a.N), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace ia

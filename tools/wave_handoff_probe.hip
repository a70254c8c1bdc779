// What does splitting one env's rollout step over two waves cost?
//
// The rollout chain's step is one dependent chain (actor -> action -> 5 physics substeps ->
// observation -> actor). A second wave can only take work off it if the hand-off of the values it
// needs -- LDS write, workgroup barrier, LDS read -- costs less than the work it takes off.
// This measures that hand-off on the card: per iteration a value goes wave 0 -> wave 1 -> wave 0
// (the shape of "actor on one wave, physics on the other"), against the same dependent arithmetic
// done by one wave alone. Core-clock cycles per iteration (s_memtime; reads only).
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/wave_handoff_probe tools/wave_handoff_probe.hip
//   /tmp/wave_handoff_probe
#include <hip/hip_runtime.h>

#include <cstdio>

namespace {

constexpr int kIters = 4096;
constexpr int kWork = 16;  // dependent FMAs per half step (a stand-in for either side's work)

__device__ __forceinline__ long long clk() {
  long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

__device__ __forceinline__ float work(float v) {
#pragma unroll
  for (int i = 0; i < kWork; ++i) v = fmaf(v, 0.999f, 0.001f);
  return v;
}

// mode 0: one wave does both halves' work; mode 1: wave 0 / wave 1 alternate through LDS + barrier;
// mode 2: the barriers alone (both waves, no data dependence through LDS)
__global__ __launch_bounds__(128) void handoff(int mode, long long* cycles, float* sink) {
  __shared__ float x[2];
  const int w = threadIdx.x >> 6;
  float v = 1.0f + threadIdx.x * 1e-3f;
  if (threadIdx.x == 0) x[0] = x[1] = 0.f;
  __syncthreads();
  const long long t0 = clk();
  if (mode == 0) {
    if (w == 0)
      for (int i = 0; i < kIters; ++i) v = work(work(v));
  } else if (mode == 1) {
    for (int i = 0; i < kIters; ++i) {
      if (w == 0) {
        v = work(v);
        x[0] = v;
      }
      __syncthreads();
      if (w == 1) {
        v = work(x[0]);
        x[1] = v;
      }
      __syncthreads();
      if (w == 0) v = x[1];
    }
  } else {
    for (int i = 0; i < kIters; ++i) {
      v = work(v);
      __syncthreads();
      __syncthreads();
    }
  }
  const long long t1 = clk();
  if ((threadIdx.x & 63) == 0) cycles[w] = t1 - t0;
  sink[threadIdx.x] = v;
}

}  // namespace

int main() {
  long long* cyc;
  float* sink;
  if (hipMalloc(&cyc, 2 * sizeof(long long)) != hipSuccess || hipMalloc(&sink, 128 * sizeof(float)) != hipSuccess) return 1;
  const char* names[3] = {"one wave, both halves", "two waves, LDS + barrier hand-off each way", "two waves, barriers only"};
  for (int mode = 0; mode < 3; ++mode) {
    long long best = -1;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(handoff, dim3(1), dim3(128), 0, 0, mode, cyc, sink);
      long long h[2];
      if (hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
      if (best < 0 || h[0] < best) best = h[0];
    }
    printf("{\"mode\": \"%s\", \"cycles_per_iteration\": %.1f, \"work_fmas_per_iteration\": %d}\n", names[mode],
           (double)best / kIters, 2 * kWork);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

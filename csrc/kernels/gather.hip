// Multi-array row gather for the device-resident replay / demonstration stores
// (data/buffer.py DeviceBuffer, rl/buffers.py ReplayBuffer, engine/dagger.py demo loader;
// SURVEY N8). A minibatch draw touches every field of the store (obs, next_obs, acts,
// rewards, dones, timeouts, ...): torch issues one advanced-indexing kernel per field (plus
// the index arithmetic), ~3 us each for a few KB. Here all fields move in ONE launch: a
// table of up to kGatherMax (src, dst, row bytes) entries, row r of the output taken from
// source row b[r] * n_envs + e[r] (e == nullptr: b[r]). Each workgroup copies whole rows
// with 16-B vector accesses when a field's row size and pointers allow it, 4-B otherwise,
// bytes as the last resort; grid.y walks the fields. Out-of-range source rows read as zeros.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gather_body.h"
#include "launchers.h"

namespace ia {
namespace {

__global__ __launch_bounds__(256) void gather_rows_kernel(GatherArgs a, const int64_t* __restrict__ b,
                                                          const int64_t* __restrict__ e, int n_envs, int n) {
  const GatherField& f = a.f[blockIdx.y];
  const int64_t rb = f.row_bytes;
  const char* __restrict__ src = static_cast<const char*>(f.src);
  char* __restrict__ dst = static_cast<char*>(f.dst);
  const int vec = ((rb & 15) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) ? 16
                  : ((rb & 3) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 3) == 0) ? 4 : 1;
  const int64_t units = rb / vec;
  const int64_t total = (int64_t)n * units;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / units, u = i - r * units;
    const int64_t srow = e ? b[r] * n_envs + e[r] : b[r];
    if (srow < 0 || srow >= f.rows) {
      if (vec == 16) reinterpret_cast<uint4*>(dst + r * rb)[u] = make_uint4(0, 0, 0, 0);
      else if (vec == 4) reinterpret_cast<uint32_t*>(dst + r * rb)[u] = 0;
      else dst[r * rb + u] = 0;
      continue;
    }
    if (vec == 16) {
      reinterpret_cast<uint4*>(dst + r * rb)[u] = reinterpret_cast<const uint4*>(src + srow * rb)[u];
    } else if (vec == 4) {
      reinterpret_cast<uint32_t*>(dst + r * rb)[u] = reinterpret_cast<const uint32_t*>(src + srow * rb)[u];
    } else {
      dst[r * rb + u] = src[srow * rb + u];
    }
  }
}

// Cursor-driven form for HIP-graph epochs (the BC epoch graph, algorithms/bc.py): row r of the
// output is source row perm[*cursor * n + r] (int32 permutation, one entry per source row), so
// a captured sequence of minibatch steps walks an epoch's order without host arguments.
__global__ __launch_bounds__(256) void gather_rows_cursor_kernel(GatherArgs a, const int* __restrict__ perm,
                                                                 const int* __restrict__ cursor, int n, float* inc) {
  gather_rows_cursor_block(a, perm, cursor, n, inc, blockIdx.x, blockIdx.y, gridDim.x);
}

// all[*cursor][0 .. n) = src[0 .. n), then ++*cursor (one block): per-step metrics of a graphed
// epoch land in their own row, the cursor names the next minibatch
__global__ void append_at_cursor_kernel(const float* __restrict__ src, float* __restrict__ all, int n, int* cursor) {
  const int cur = *cursor;
  __syncthreads();  // every thread has read the cursor before thread 0 moves it
  for (int i = threadIdx.x; i < n; i += blockDim.x) all[(size_t)cur * n + i] = src[i];
  if (threadIdx.x == 0) *cursor = cur + 1;
}

}  // namespace

hipError_t gather_rows_cursor(const GatherArgs& a, const int* perm, const int* cursor, int n, hipStream_t s, float* inc) {
  if (n <= 0 || a.k <= 0) return hipSuccess;
  if (a.k > kGatherMax) return hipErrorInvalidValue;
  const int bx = gather_cursor_blocks(a, n);
  hipLaunchKernelGGL(gather_rows_cursor_kernel, dim3((unsigned)bx, a.k), dim3(256), 0, s, a, perm, cursor, n, inc);
  return hipGetLastError();
}

hipError_t append_at_cursor(const float* src, float* all, int n, int* cursor, hipStream_t s) {
  hipLaunchKernelGGL(append_at_cursor_kernel, dim3(1), dim3(64), 0, s, src, all, n, cursor);
  return hipGetLastError();
}

hipError_t gather_rows(const GatherArgs& a, const int64_t* b, const int64_t* e, int n_envs, int n, hipStream_t s) {
  if (n <= 0 || a.k <= 0) return hipSuccess;
  if (a.k > kGatherMax) return hipErrorInvalidValue;
  int64_t most = 0;
  for (int i = 0; i < a.k; ++i) {
    const int64_t units = a.f[i].row_bytes / ((a.f[i].row_bytes & 15) == 0 ? 16 : 1);
    most = units * n > most ? units * n : most;
  }
  int64_t bx = (most + 255) / 256;
  bx = bx < 1 ? 1 : (bx > 1024 ? 1024 : bx);
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)bx, a.k), dim3(256), 0, s, a, b, e, n_envs, n);
  return hipGetLastError();
}

}  // namespace ia

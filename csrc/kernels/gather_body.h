// One block of the cursor-indexed row gather (gather.hip), as a device function so that another
// launch can run it in a block range of its own (conv.hip: the BC step's weight packing).
#pragma once
#include <hip/hip_runtime.h>

#include "launchers.h"

namespace ia {

// (bx, by) = (block of the field's rows, field); gx = blocks per field. Row r of every field's
// output is source row perm[*cursor * n + r]; inc (if set): ++*inc by one thread.
__device__ __forceinline__ void gather_rows_cursor_block(const GatherArgs& a, const int* __restrict__ perm,
                                                         const int* __restrict__ cursor, int n, float* inc, int bx,
                                                         int by, int gx) {
  if (inc && bx == 0 && by == 0 && threadIdx.x == 0) *inc += 1.f;  // (nothing else here reads it)
  const GatherField& f = a.f[by];
  const int64_t rb = f.row_bytes;
  const char* __restrict__ src = static_cast<const char*>(f.src);
  char* __restrict__ dst = static_cast<char*>(f.dst);
  const int* __restrict__ b = perm + (int64_t)(*cursor) * n;
  const int vec = ((rb & 15) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) ? 16
                  : ((rb & 3) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 3) == 0) ? 4 : 1;
  const int64_t units = rb / vec;
  const int64_t total = (int64_t)n * units;
  for (int64_t i = (int64_t)bx * blockDim.x + threadIdx.x; i < total; i += (int64_t)gx * blockDim.x) {
    const int64_t r = i / units, u = i - r * units;
    const int64_t srow = b[r];
    const bool ok = srow >= 0 && srow < f.rows;
    if (vec == 16) {
      reinterpret_cast<uint4*>(dst + r * rb)[u] = ok ? reinterpret_cast<const uint4*>(src + srow * rb)[u] : make_uint4(0, 0, 0, 0);
    } else if (vec == 4) {
      reinterpret_cast<uint32_t*>(dst + r * rb)[u] = ok ? reinterpret_cast<const uint32_t*>(src + srow * rb)[u] : 0u;
    } else {
      dst[r * rb + u] = ok ? src[srow * rb + u] : (char)0;
    }
  }
}

// blocks per field of a 256-thread gather launch
inline int gather_cursor_blocks(const GatherArgs& a, int n) {
  int64_t most = 0;
  for (int i = 0; i < a.k; ++i) {
    const int64_t units = a.f[i].row_bytes / ((a.f[i].row_bytes & 15) == 0 ? 16 : 1);
    most = units * n > most ? units * n : most;
  }
  int64_t bx = (most + 255) / 256;
  return (int)(bx < 1 ? 1 : (bx > 1024 ? 1024 : bx));
}

}  // namespace ia

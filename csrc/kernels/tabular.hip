// Tabular / non-parametric estimators of the MCE-IRL and density baselines, fp64.
//
// MCE-IRL (reference algorithms/mce_irl.py:38-144). Both recursions are
// H-step loops of a tiny mat-vec: per step the torch form is ~6 launches (matmul, add,
// logsumexp's 3, the copy into Q[t]) of a few microseconds each, so a 100-step horizon is
// ~600 launches of nothing. Here each recursion is ONE workgroup that keeps the running
// vector (V_{t+1} or D_t) and the step's intermediate (Q_t or D_t * pi_t) in LDS and loops
// over the horizon with workgroup barriers; T [S][A][S'] streams from L2 (it is re-read
// every step and stays resident: S=400, A=4 is 5 MB).
//   soft value iteration:  Q_t[s,a] = R[s] + gamma * sum_p T[s,a,p] V_{t+1}[p],
//                          V_t = logsumexp_a Q_t,  pi_t = exp(Q_t - V_t)
//     one wave per (s,a) row group, lanes stride over p (coalesced), shuffle reduction;
//   occupancy:             D_{t+1}[p] = sum_{s,a} D_t[s] pi_t[s,a] T[s,a,p]
//     one thread per p (coalesced over p for a fixed (s,a)).
//
// KDE scoring (reference algorithms/density.py via sklearn KernelDensity):
// log p(q) = logsumexp_j log k(|q - x_j| / h) - log N + log-normaliser. Exact squared
// distances (sum of (q - x)^2, not the |q|^2 + |x|^2 - 2 q.x expansion) with an online
// logsumexp per query: 256 queries per block (one per thread), the data points staged
// through LDS 64 at a time, and the data split over grid.y so that a few thousand queries
// still fill the chip; a second launch merges the (max, sum) partials in a fixed order.
#include <hip/hip_runtime.h>
#include <math.h>

#include "launchers.h"

namespace ia {
namespace {

constexpr int kVIThreads = 1024;

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kVIThreads) void soft_vi_kernel(const double* __restrict__ T, const double* __restrict__ R,
                                                             int S, int A, int H, double gamma, double* __restrict__ V,
                                                             double* __restrict__ Q, double* __restrict__ P) {
  extern __shared__ double lds[];
  double* vnext = lds;      // [S]
  double* qt = lds + S;     // [S*A]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = kVIThreads / 64;
  const int SA = S * A;
  for (int t = H - 1; t >= 0; --t) {
    if (t == H - 1) {
      for (int i = tid; i < SA; i += kVIThreads) qt[i] = R[i / A];
    } else {
      for (int row = wave; row < SA; row += nw) {
        const double* tr = T + (size_t)row * S;
        double acc = 0.0;
        for (int p = lane; p < S; p += 64) acc += tr[p] * vnext[p];
        acc = wave_sum_f64(acc);
        if (lane == 0) qt[row] = R[row / A] + gamma * acc;
      }
    }
    __syncthreads();
    for (int s = tid; s < S; s += kVIThreads) {
      const double* qs = qt + (size_t)s * A;
      double mx = -INFINITY;
      for (int a = 0; a < A; ++a) mx = fmax(mx, qs[a]);
      double se = 0.0;
      for (int a = 0; a < A; ++a) se += exp(qs[a] - mx);
      const double v = mx + log(se);
      vnext[s] = v;
      V[(size_t)t * S + s] = v;
      for (int a = 0; a < A; ++a) {
        Q[((size_t)t * S + s) * A + a] = qs[a];
        P[((size_t)t * S + s) * A + a] = exp(qs[a] - v);
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kVIThreads) void occupancy_kernel(const double* __restrict__ T, const double* __restrict__ P,
                                                               const double* __restrict__ D0, int S, int A, int H,
                                                               double* __restrict__ D) {
  extern __shared__ double lds[];
  double* dcur = lds;   // [S]
  double* w = lds + S;  // [S*A]
  const int tid = threadIdx.x, SA = S * A;
  for (int s = tid; s < S; s += kVIThreads) {
    dcur[s] = D0[s];
    D[s] = D0[s];
  }
  __syncthreads();
  for (int t = 0; t < H; ++t) {
    const double* pt = P + (size_t)t * SA;
    for (int i = tid; i < SA; i += kVIThreads) w[i] = dcur[i / A] * pt[i];
    __syncthreads();
    for (int p = tid; p < S; p += kVIThreads) {
      double acc = 0.0;
      for (int r = 0; r < SA; ++r) acc += w[r] * T[(size_t)r * S + p];
      D[(size_t)(t + 1) * S + p] = acc;
      dcur[p] = acc;  // own column only; the next step's w reads it after the barrier
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ KDE
constexpr int kKdeQ = 256;   // queries per block
constexpr int kKdeTile = 64;  // data points per LDS tile

__device__ __forceinline__ double kde_logk(double d2, double inv_h, int kind) {
  if (kind == 0) return -0.5 * d2 * inv_h * inv_h;       // gaussian
  const double r = sqrt(d2) * inv_h;
  if (kind == 1) return -r;                              // exponential
  if (kind == 2) return r < 1.0 ? 0.0 : -INFINITY;       // tophat
  if (kind == 3) return r < 1.0 ? log(1.0 - r * r) : -INFINITY;  // epanechnikov
  if (kind == 4) return r < 1.0 ? log(1.0 - r) : -INFINITY;      // linear
  return r < 1.0 ? log(cos(0.5 * M_PI * r)) : -INFINITY;         // cosine
}

__global__ __launch_bounds__(kKdeQ) void kde_partial_kernel(const double* __restrict__ q, const double* __restrict__ x,
                                                            int NQ, int N, int d, int per_split, double inv_h, int kind,
                                                            double* __restrict__ pmax, double* __restrict__ psum) {
  extern __shared__ double tile[];  // [kKdeTile][d]
  const int qi = blockIdx.x * kKdeQ + threadIdx.x;
  const int j0 = blockIdx.y * per_split;
  const int j1 = min(N, j0 + per_split);
  double qr[kKdeMaxDim];
#pragma unroll
  for (int k = 0; k < kKdeMaxDim; ++k) qr[k] = (qi < NQ && k < d) ? q[(size_t)qi * d + k] : 0.0;
  double mx = -INFINITY, se = 0.0;
  for (int jt = j0; jt < j1; jt += kKdeTile) {
    const int nt = min(kKdeTile, j1 - jt);
    __syncthreads();
    for (int i = threadIdx.x; i < nt * d; i += kKdeQ) tile[i] = x[(size_t)jt * d + i];
    __syncthreads();
    for (int j = 0; j < nt; ++j) {
      const double* xr = tile + j * d;
      double d2 = 0.0;
#pragma unroll
      for (int k = 0; k < kKdeMaxDim; ++k)
        if (k < d) {
          const double df = qr[k] - xr[k];
          d2 += df * df;
        }
      const double lk = kde_logk(d2, inv_h, kind);
      if (lk > mx) {
        se = se * exp(mx - lk) + 1.0;  // exp(-inf) = 0 on the first finite term
        mx = lk;
      } else if (lk > -INFINITY) {
        se += exp(lk - mx);
      }
    }
  }
  if (qi < NQ) {
    pmax[(size_t)blockIdx.y * NQ + qi] = mx;
    psum[(size_t)blockIdx.y * NQ + qi] = se;
  }
}

__global__ __launch_bounds__(256) void kde_combine_kernel(const double* __restrict__ pmax, const double* __restrict__ psum,
                                                          int NQ, int nsplit, double offset, double* __restrict__ out) {
  const int qi = blockIdx.x * 256 + threadIdx.x;
  if (qi >= NQ) return;
  double mx = -INFINITY;
  for (int k = 0; k < nsplit; ++k) mx = fmax(mx, pmax[(size_t)k * NQ + qi]);
  if (mx == -INFINITY) {
    out[qi] = -INFINITY;
    return;
  }
  double se = 0.0;
  for (int k = 0; k < nsplit; ++k) {
    const double m = pmax[(size_t)k * NQ + qi];
    if (m > -INFINITY) se += psum[(size_t)k * NQ + qi] * exp(m - mx);
  }
  out[qi] = mx + log(se) + offset;
}

}  // namespace

bool soft_vi_fits(int S, int A) { return S > 0 && A > 0 && (size_t)S * (A + 1) * sizeof(double) <= 150 * 1024; }

hipError_t soft_value_iteration(const double* T, const double* R, int S, int A, int H, double gamma, double* V, double* Q,
                                double* P, hipStream_t s) {
  if (!soft_vi_fits(S, A) || H <= 0) return hipErrorInvalidValue;
  const size_t lds = (size_t)S * (A + 1) * sizeof(double);
  hipLaunchKernelGGL(soft_vi_kernel, dim3(1), dim3(kVIThreads), lds, s, T, R, S, A, H, gamma, V, Q, P);
  return hipGetLastError();
}

hipError_t occupancy_measures(const double* T, const double* P, const double* D0, int S, int A, int H, double* D,
                              hipStream_t s) {
  if (!soft_vi_fits(S, A) || H < 0) return hipErrorInvalidValue;
  const size_t lds = (size_t)S * (A + 1) * sizeof(double);
  hipLaunchKernelGGL(occupancy_kernel, dim3(1), dim3(kVIThreads), lds, s, T, P, D0, S, A, H, D);
  return hipGetLastError();
}

int kde_splits(int NQ, int N) {
  const int qb = (NQ + kKdeQ - 1) / kKdeQ;
  int want = (512 + qb - 1) / qb;                // ~2 blocks per CU in total
  const int most = (N + kKdeTile - 1) / kKdeTile;  // at least one tile per split
  want = want < 1 ? 1 : want;
  return want < most ? want : (most < 1 ? 1 : most);
}

hipError_t kde_score(const double* q, const double* x, int NQ, int N, int d, double inv_h, int kind, double offset,
                     double* pmax, double* psum, double* out, hipStream_t s) {
  if (NQ <= 0) return hipSuccess;
  if (d <= 0 || d > kKdeMaxDim || N <= 0 || kind < 0 || kind > 5) return hipErrorInvalidValue;
  const int ns = kde_splits(NQ, N);
  int per = (N + ns - 1) / ns;
  per = (per + kKdeTile - 1) / kKdeTile * kKdeTile;
  const size_t lds = (size_t)kKdeTile * d * sizeof(double);
  hipLaunchKernelGGL(kde_partial_kernel, dim3((NQ + kKdeQ - 1) / kKdeQ, ns), dim3(kKdeQ), lds, s, q, x, NQ, N, d, per,
                     inv_h, kind, pmax, psum);
  hipLaunchKernelGGL(kde_combine_kernel, dim3((NQ + 255) / 256), dim3(256), 0, s, pmax, psum, NQ, ns, offset, out);
  return hipGetLastError();
}

}  // namespace ia

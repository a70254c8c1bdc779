// Fused preference reward-model minibatch (DRLHP reward training).
//
// Reference semantics: one minibatch of BasicRewardTrainer._train
// (src/imitation/algorithms/preference_comparisons.py:1255-1282): the fragment pairs' transitions
// through the reward net (BasicRewardNet, input RunningNorm in train mode: networks.py:94-111),
// PreferenceModel.probability (Bradley-Terry over discounted fragment returns, clipped at
// +-threshold, label noise, :411-530), CrossEntropyRewardLoss (:1050-1090) scaled by
// n / batch_size, backward, AdamW (the trainer's optimizer, :1192). The autograd fast path runs
// that as ~50 launches per minibatch; here it is four:
//
//   pref_gather   rows of the minibatch's pairs (pair ids idx, 2L rows each: fragment 1 then
//                 fragment 2) gathered into the reward-net input X; per-block shifted column
//                 sums for the RunningNorm, reduced (fixed order, fp64) by the last block to
//                 finish; block 0 bumps the device Adam step and snapshots the running
//                 statistics
//   pref_fwd      every block Chan-merges the batch moments into the snapshot and normalises
//                 its 64 rows (block 0 publishes the merged statistics); reward-net forward ->
//                 r[row]
//   pref_bwd      per 64-row block: the Bradley-Terry terms of the pairs its rows belong to
//                 (from r: fragment returns, probability, loss, dloss/ddiff), the per-row
//                 reward gradient, the forward recomputed and the backward -> one slab row;
//                 per-pair loss / accuracy / ground-truth loss
//   disc_adam     (disc.hip) fixed-order slab reduction + AdamW on the flat parameters, with
//                 the bias corrections from the device step counter (graph-capturable), and
//                 the minibatch means of the pair statistics
//
// Matrix work is v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulation) through the
// block MLP helpers of ia/dmlp.h; every reduction has a fixed order (bitwise reproducible
// replicas under data parallelism).
#include <hip/hip_runtime.h>

#include "ia/dmlp.h"
#include "ia/mfma.h"
#include "launchers.h"

namespace ia {
namespace {

using namespace dmlp;

__device__ __forceinline__ float bt_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// column c of the reward-net input for dataset row src
__device__ __forceinline__ float pref_col(const PrefRmArgs& a, int64_t src, int c) {
  if (c < a.ds) return a.s_all[src * a.ds + c];
  c -= a.ds;
  if (c < a.da) return a.a_all[src * a.da + c];
  c -= a.da;
  if (c < a.dns) return a.ns_all[src * a.dns + c];
  return a.d_all[src];
}

// sc1 (L1-bypassing, agent-coherent) 4-B accesses for the last-block reduction of the
// gather's column sums; inline asm so a lane keeps 8 loads in flight before ONE wait
__device__ __forceinline__ void st_sc1(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// pair ids of this minibatch (epoch graphs: offset by the device epoch cursor)
__device__ __forceinline__ const int64_t* pair_ids(const PrefRmArgs& a) {
  return a.cursor ? a.idx + (int64_t)(*a.cursor) * a.idx_stride : a.idx;
}

// block b covers rows [64 b, 64 b + 64): the 64 x din tile element-parallel (consecutive
// threads read consecutive columns of a row, all loads independent), staged in LDS for the
// shifted column sums (4 row phases x 64 columns, fixed order). The block sums are handed to
// the LAST block to finish (MI355X_MICROARCH inter-workgroup visibility, row 1: sc1 stores,
// every storing wave's vmcnt(0), a barrier, one agent-scope add per block; the block whose add
// returns nblocks - 1 reads them with sc1 loads), which reduces them in block order (fp64) into
// sums -- so the forward's blocks read 2 din values instead of re-reducing every block's.
__global__ __launch_bounds__(256) void pref_gather_kernel(PrefRmArgs a) {
  __shared__ float tile[kRows][129];
  __shared__ float red[4][2][64];
  __shared__ double dred[4][128];
  __shared__ int is_last;
  const int rows = 2 * a.n * a.L, twoL = 2 * a.L, din = a.din;
  const int r0 = blockIdx.x * kRows;
  const int64_t* idx = pair_ids(a);
  for (int e = threadIdx.x; e < kRows * din; e += 256) {
    const int rr = e / din, c = e - rr * din;
    const int r = r0 + rr;
    float v = 0.f;
    if (r < rows) {
      const int i = r / twoL, t = r - i * twoL;
      v = pref_col(a, idx[i] * (int64_t)twoL + t, c);
      a.X[(size_t)r * din + c] = v;
    }
    tile[rr][c] = v;
  }
  if (a.rmean) {
    __syncthreads();
    const int nv = min(kRows, rows - r0);
    for (int c0 = 0; c0 < din; c0 += 64) {
      const int c = c0 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
      float s1 = 0.f, s2 = 0.f;
      if (c < din) {
        const float shift = a.rmean[c];
        for (int rr = ph; rr < nv; rr += 4) {
          const float dv = tile[rr][c] - shift;
          s1 += dv;
          s2 += dv * dv;
        }
      }
      red[ph][0][threadIdx.x & 63] = s1;
      red[ph][1][threadIdx.x & 63] = s2;
      __syncthreads();
      if (ph == 0 && c < din) {
        float* out = a.partials + (size_t)blockIdx.x * 2 * din;
        const int j = threadIdx.x & 63;
        st_sc1(out + c, (red[0][0][j] + red[1][0][j]) + (red[2][0][j] + red[3][0][j]));
        st_sc1(out + din + c, (red[0][1][j] + red[1][1][j]) + (red[2][1][j] + red[3][1][j]));
      }
      __syncthreads();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) is_last = atomicAdd(a.cnt, 1u) == gridDim.x - 1;
    __syncthreads();
    if (is_last) {
      // sums[j] = sum over blocks b (in order) of partials[b][j]: 64 sums x 4 block phases
      // per pass, 8 sc1 loads in flight per lane
      const int nb = gridDim.x, ns = 2 * din;
      for (int j0 = 0; j0 < ns; j0 += 64) {
        const int j = j0 + (threadIdx.x & 63), q = threadIdx.x >> 6;
        double acc = 0.0;
        if (j < ns)
          for (int b0 = q; b0 < nb; b0 += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = ld_sc1(a.partials + (size_t)min(b0 + 4 * u, nb - 1) * ns + j);
            asm volatile("s_waitcnt vmcnt(0)"
                         : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
                         :
                         : "memory");
#pragma unroll
            for (int u = 0; u < 8; ++u)
              if (b0 + 4 * u < nb) acc += (double)v[u];
          }
        dred[q][threadIdx.x & 63] = acc;
        __syncthreads();
        if (q == 0 && j < ns) a.sums[j] = (dred[0][threadIdx.x] + dred[1][threadIdx.x]) + (dred[2][threadIdx.x] + dred[3][threadIdx.x]);
        __syncthreads();
      }
      if (threadIdx.x == 0) __hip_atomic_store(a.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  const int c = threadIdx.x & 127;
  const bool col_ok = c < din;
  if (blockIdx.x == 0) {
    if (a.rmean && threadIdx.x < 128 && col_ok) {  // running statistics before this minibatch
      a.old_mv[c] = a.rmean[c];
      a.old_mv[128 + c] = a.rvar[c];
    }
    if (threadIdx.x == 0) {
      if (a.rcount) a.old_cnt[0] = *a.rcount;
      if (a.step) *a.step += 1.f;
    }
  }
}

// LDS layout of pref_fwd / pref_bwd (PrefPlan): weight images, row images, backward scratch.
// Image addresses are computed per use from the plan (a kernel argument, read with scalar
// loads): an array of LDS pointers indexed by the run-time layer would be kept in scratch.
struct WImg {  // forward ([o][i]) or transposed ([i][o]) weight image of layer l
  char* smem;
  const int* off;
  __device__ lbf* operator[](int l) const { return (lbf*)(smem + off[l]); }
};
struct HImg {  // row image of layer l's input (the output layer reuses the last slot)
  char* base;
  int bytes, last;
  __device__ lbf* operator[](int l) const { return (lbf*)(base + (size_t)min(l, last) * bytes); }
};
struct ZImg {  // double-buffered dZ / dZ^T images
  char* base;
  int stride;
  __device__ lbf* operator[](int z) const { return (lbf*)(base + (size_t)z * stride); }
};
struct Imgs {
  WImg Wf, Wt;
  HImg H;
  lbf* HT;
  ZImg dZ, dZT;
  lfl* dbs;
};

__device__ __forceinline__ Imgs carve(char* smem, const PrefPlan& p, int n_layers) {
  Imgs m;
  m.Wf = WImg{smem, p.wf_off};
  m.Wt = WImg{smem, p.wt_off};
  m.H = HImg{smem + p.rimg_off, p.rimg_bytes, n_layers - 1};
  char* sc = smem + p.scratch_off;
  m.HT = (lbf*)(sc);
  m.dZ = ZImg{sc + p.ht_bytes, p.rimg_bytes};
  m.dZT = ZImg{sc + p.ht_bytes + 2 * p.rimg_bytes, p.ht_bytes};
  m.dbs = (lfl*)(sc + 3 * p.ht_bytes + 2 * p.rimg_bytes);
  return m;
}

// moments from sums (the gather's; under data parallelism all-reduced over n_total rows)
__global__ __launch_bounds__(64 * kNW) void pref_fwd_kernel(PrefRmArgs a, PrefPlan p, int n_total) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float nrm[256];
  __shared__ float out[kRows];
  const int c = threadIdx.x & 127;
  const int rows = 2 * a.n * a.L;
  const int row0 = blockIdx.x * kRows;
  Imgs m = carve(smem, p, a.net.n_layers);
  lds_zero(smem, p.lds_bytes);
  // ---- RunningNorm: batch moments (fixed order), Chan merge into the pre-minibatch snapshot
  if (a.rmean) {
    if (threadIdx.x < 128) {
      float mean = 0.f, rstd = 1.f;
      if (c < a.din) {
        const double S1 = a.sums[c], S2 = a.sums[a.din + c];
        const int n = n_total > 0 ? n_total : rows;
        float rm = a.old_mv[c], rv = a.old_mv[128 + c];
        if (a.merge) {
          const double bm = S1 / n;
          double bv = S2 / n - bm * bm;
          if (bv < 0.0) bv = 0.0;
          chan_merge(&rm, &rv, a.old_cnt[0], 0, (float)((double)a.old_mv[c] + bm), (float)bv, n);
        }
        mean = rm;
        rstd = rsqrtf(rv + a.eps);
        if (blockIdx.x == 0) {
          if (a.merge) {
            a.rmean[c] = rm;
            a.rvar[c] = rv;
          }
          a.nrm[c] = mean;
          a.nrm[128 + c] = rstd;
        }
      }
      nrm[c] = mean;
      nrm[128 + c] = rstd;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.merge) *a.rcount = a.old_cnt[0] + (n_total > 0 ? n_total : rows);
  } else if (threadIdx.x < 128) {
    nrm[c] = 0.f;
    nrm[128 + c] = 1.f;
    if (blockIdx.x == 0) {
      a.nrm[c] = 0.f;
      a.nrm[128 + c] = 1.f;
    }
  }
  __syncthreads();
  for (int l = 0; l < a.net.n_layers; ++l) stage_weights(m.Wf[l], a.net.W[l], a.net.dims[l + 1], a.net.dims[l], false);
  stage_rows(m.H[0], p.ldr, a.X, a.din, rows, row0, nrm);
  __syncthreads();
  mlp_forward(a.net, m.H, p.ldr, m.Wf, (lfl*)out, 1);
  __syncthreads();
  if (threadIdx.x < kRows && row0 + (int)threadIdx.x < rows) a.r[row0 + threadIdx.x] = out[threadIdx.x];
}

__device__ __forceinline__ float bce_clamped(float p, float y) {
  const float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(logf(1.f - p), -100.f);
  return -(y * lp + (1.f - y) * l1p);
}

__global__ __launch_bounds__(64 * kNW) void pref_bwd_kernel(PrefRmArgs a, PrefPlan p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float dy[kRows];
  __shared__ float coef[kRows + 2];
  __shared__ float out[kRows];
  const int rows = 2 * a.n * a.L, twoL = 2 * a.L;
  const int row0 = blockIdx.x * kRows;
  const int w = wave_id(), lane = lane_id();
  Imgs m = carve(smem, p, a.net.n_layers);
  lds_zero(smem, p.lds_bytes);
  __syncthreads();
  const AirlNet& net = a.net;
  for (int l = 0; l < net.n_layers; ++l) {
    stage_weights(m.Wf[l], net.W[l], net.dims[l + 1], net.dims[l], false);
    if (l > 0) stage_weights(m.Wt[l], net.W[l], net.dims[l + 1], net.dims[l], true);
  }
  stage_rows(m.H[0], p.ldr, a.X, a.din, rows, row0, a.nrm);
  // ---- Bradley-Terry terms of the pairs this block's rows belong to (one wave per pair)
  const int last_row = min(rows, row0 + kRows) - 1;
  const int p_lo = row0 / twoL, p_hi = last_row / twoL;
  const float lg = a.discount == 1.f ? 0.f : __log2f(a.discount);
  for (int pi = p_lo + w; pi <= p_hi; pi += kNW) {
    const float* r1 = a.r + (size_t)pi * twoL;
    const float* r2 = r1 + a.L;
    float s = 0.f, sg = 0.f;
    const int64_t gi = pair_ids(a)[pi];
    for (int t = lane; t < a.L; t += 64) {
      const float wt = a.discount == 1.f ? 1.f : exp2f(lg * (float)t);
      s += wt * (r2[t] - r1[t]);
      if (a.gt_all) sg += wt * (a.gt_all[(gi * 2 + 1) * a.L + t] - a.gt_all[gi * 2 * a.L + t]);
    }
    const float diff = bt_wave_sum(s);
    const float gdiff = bt_wave_sum(sg);
    if (lane == 0) {
      const float y = a.prefs_all[gi];
      const bool inside = diff >= -a.threshold && diff <= a.threshold;
      const float d = fminf(fmaxf(diff, -a.threshold), a.threshold);
      const float ed = expf(d);
      const float pm = 1.f / (1.f + ed);
      const float pr = a.noise * 0.5f + (1.f - a.noise) * pm;
      float cf;
      if (a.noise == 0.f) {
        cf = y - pm;  // dloss/ddiff (pref.hip: the exact form for noise 0)
      } else {
        const float dl_dp = (pr - y) / fmaxf(pr * (1.f - pr), 1e-12f);
        cf = dl_dp * ((1.f - a.noise) * -(pm * pm) * ed);
      }
      coef[pi - p_lo] = inside ? cf : 0.f;
      if (pi * twoL >= row0) {  // this block owns the pair's statistics
        float* st = a.pstats + (size_t)pi * 8;
        st[0] = bce_clamped(pr, y);
        st[1] = ((pr > 0.5f) == (y > 0.5f)) ? 1.f : 0.f;
        float gl = 0.f;
        if (a.gt_all) {
          const float gd = fminf(fmaxf(gdiff, -a.threshold), a.threshold);
          gl = bce_clamped(a.noise * 0.5f + (1.f - a.noise) / (1.f + expf(gd)), y);
        }
        st[2] = gl;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x < kRows) {
    const int gr = row0 + threadIdx.x;
    float g = 0.f;
    if (gr < rows) {
      const int pi = gr / twoL, t = gr - pi * twoL;
      const int tt = t < a.L ? t : t - a.L;
      const float wt = a.discount == 1.f ? 1.f : exp2f(lg * (float)tt);
      // d loss_mean / d r: dr2 = coef w_t / n, dr1 = -dr2; times the trainer's n / batch_size
      g = a.gscale * coef[pi - p_lo] * wt * (t < a.L ? -1.f : 1.f);
    }
    dy[threadIdx.x] = g;
  }
  __syncthreads();
  mlp_forward(net, m.H, p.ldr, m.Wf, (lfl*)out, 1);  // hidden images for the backward
  float* slab_row = a.slab + (size_t)blockIdx.x * a.n_params;
  mlp_backward(net, m.H, p.ldr, m.Wt, (const lfl*)dy, m.HT, p.ld_ht, m.dZ, m.dZT, m.dbs, p.dmax_pad, slab_row, false);
}

__global__ void pref_epoch_end_kernel(const float* __restrict__ metrics, float* __restrict__ all, int n, int* cursor) {
  const int cur = *cursor;
  __syncthreads();  // every thread has read the cursor before thread 0 moves it
  for (int i = threadIdx.x; i < n; i += blockDim.x) all[(size_t)cur * n + i] = metrics[i];
  if (threadIdx.x == 0) *cursor = cur + 1;
}

}  // namespace

hipError_t pref_rm_epoch_end(const float* metrics, float* all, int n, int* cursor, hipStream_t s) {
  hipLaunchKernelGGL(pref_epoch_end_kernel, dim3(1), dim3(256), 0, s, metrics, all, n, cursor);
  return hipGetLastError();
}

int pref_rm_blocks(int n_pairs, int L) { return (2 * n_pairs * L + kRows - 1) / kRows; }

bool pref_rm_plan(const PrefRmArgs& a, PrefPlan& p) {
  p = PrefPlan{};
  const AirlNet& n = a.net;
  if (n.n_layers < 1 || n.n_layers > kAirlMaxLayers) return false;
  int rmax = 0;
  for (int l = 0; l <= n.n_layers; ++l) {
    if (n.dims[l] <= 0 || n.dims[l] > 64) return false;
    rmax = rmax > n.dims[l] ? rmax : n.dims[l];
  }
  if (n.dims[n.n_layers] != 1 || n.dims[0] != a.din || a.din > 128 || a.L < 1) return false;
  p.ldr = ld_for_k(rmax);
  p.ld_ht = ld_for_k(kRows);
  p.dmax_pad = pad32(rmax);
  p.rimg_bytes = kRows * p.ldr * 2;
  p.ht_bytes = pad32(rmax) * p.ld_ht * 2;
  if (p.ht_bytes < kRows * 32 * 2) p.ht_bytes = kRows * 32 * 2;
  int off = 0;
  for (int l = 0; l < kAirlMaxLayers; ++l) {
    p.wf_off[l] = p.wt_off[l] = 0;
    if (l >= n.n_layers) continue;
    const int din = n.dims[l], dout = n.dims[l + 1];
    p.wf_off[l] = off;
    off += (pad32(dout) * ld_for_k(din) * 2 + 15) & ~15;
    if (l > 0) {
      p.wt_off[l] = off;
      off += (pad32(din) * ld_for_k(dout) * 2 + 15) & ~15;
    }
  }
  p.rimg_off = off;
  off += n.n_layers * p.rimg_bytes;
  p.scratch_off = off;
  off += (3 * p.ht_bytes + 2 * p.rimg_bytes + (2 * kNW * p.dmax_pad + 16) * 4 + 15) & ~15;
  p.lds_bytes = off;
  return p.lds_bytes <= 128 * 1024;
}

hipError_t pref_rm_gather(const PrefRmArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(pref_gather_kernel, dim3(pref_rm_blocks(a.n, a.L)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t pref_rm_fwd(const PrefRmArgs& a, const PrefPlan& p, int n_total, hipStream_t s) {
  hipLaunchKernelGGL(pref_fwd_kernel, dim3(pref_rm_blocks(a.n, a.L)), dim3(64 * kNW), p.lds_bytes, s, a, p, n_total);
  return hipGetLastError();
}

hipError_t pref_rm_bwd(const PrefRmArgs& a, const PrefPlan& p, hipStream_t s) {
  hipLaunchKernelGGL(pref_bwd_kernel, dim3(pref_rm_blocks(a.n, a.L)), dim3(64 * kNW), p.lds_bytes, s, a, p);
  return hipGetLastError();
}

}  // namespace ia

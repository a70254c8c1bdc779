// Fused tiny-MLP forward / backward on CDNA4 MFMA (bf16 operands, fp32 accumulate).
//
// Replaces the chain of PyTorch Linear/ReLU/Tanh launches the reference issues
// for every reward-net / policy evaluation (reward_nets.py:441-457 BasicRewardNet,
// SB3 MlpExtractor + heads via policies/base.py:208-220) with ONE launch:
//   * forward: input (optionally RunningNorm-normalised, networks.py:79-91) ->
//     all layers -> output, activations never leave LDS;
//   * backward: recompute the forward tile in LDS (cheaper than storing it),
//     then dZ -> dW/db (MFMA over the row dimension) -> dX, per 16*NW-row block.
//     Per-block parameter gradients go to a slab that tmlp_grad_reduce sums
//     deterministically (bitwise-reproducible DP replicas).
//
// Block = NW waves; wave w owns rows [16w, 16w+16) of the block tile.
#include <hip/hip_runtime.h>

#include "ia/mfma.h"
#include "ia/tmlp.h"
#include "launchers.h"

namespace ia {
namespace {

// X[row0 .. row0+rows) x [0 .. din) -> bf16 image [rows][ld], normalised, zero padded.
__device__ void stage_input(bf16* H, int ld, const float* __restrict__ X, int B, int row0, int rows, const MLPDesc& d) {
  const int din = d.dims[0];
  const int kp = pad32(din);
  const int n = rows * kp;
  const long long go = (long long)blockIdx.y * d.gs_norm;
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int r = e / kp, c = e - r * kp;
    const int gr = row0 + r;
    float v = 0.f;
    if (gr < B && c < din) {
      v = X[(size_t)gr * din + c];
      if (d.norm_mean) {
        v = (v - d.norm_mean[go + c]) * rsqrtf(d.norm_var[go + c] + d.norm_eps);
        if (d.norm_clip > 0.f) v = fminf(fmaxf(v, -d.norm_clip), d.norm_clip);
      }
    }
    H[r * ld + c] = to_bf16(v);
  }
}

// Full padded weight image: rows [0, pad32(out)), cols [0, pad32(in)); zeros outside.
__device__ void stage_w(bf16* dst, const float* __restrict__ W, int dout, int din, bool transposed) {
  if (!transposed) {
    const int ld = ld_for_k(din), R = pad32(dout), C = pad32(din);
    for (int e = threadIdx.x; e < R * C; e += blockDim.x) {
      const int o = e / C, i = e - o * C;
      dst[o * ld + i] = to_bf16((o < dout && i < din) ? W[o * din + i] : 0.f);
    }
  } else {
    const int ld = ld_for_k(dout), R = pad32(din), C = pad32(dout);
    for (int e = threadIdx.x; e < R * C; e += blockDim.x) {
      const int i = e / C, o = e - i * C;
      dst[i * ld + o] = to_bf16((o < dout && i < din) ? W[o * din + i] : 0.f);
    }
  }
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void tmlp_fwd_kernel(MLPDesc d, TmlpPlan p, const float* __restrict__ X, int B,
                                                           float* __restrict__ Y) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16* Wb = reinterpret_cast<bf16*>(smem);
  bf16* H0 = reinterpret_cast<bf16*>(smem + p.w_bytes);
  bf16* H1 = reinterpret_cast<bf16*>(smem + p.w_bytes + p.h_bytes);
  const int row0 = blockIdx.x * p.rows;
  const int w = wave_id();
  const long long grp = blockIdx.y;
  X += grp * d.gs_x;
  Y += grp * d.gs_y;
  lds_zero(smem, p.fwd_lds);
  __syncthreads();
  stage_input(H0, p.ld_h, X, B, row0, p.rows, d);
  bf16* Hin = H0;
  bf16* Hout = H1;
  for (int l = 0; l < d.n_layers; ++l) {
    const int din = d.dims[l], dout = d.dims[l + 1];
    __syncthreads();
    stage_w(Wb, d.W[l] + grp * d.gs_w[l], dout, din, false);
    __syncthreads();
    const int K = pad32(din), ldw = ld_for_k(din);
    const bool last = l == d.n_layers - 1;
    const int act = layer_act(d, l);
    const int ntiles = last ? pad16(dout) / 16 : pad32(dout) / 16;
    const bf16* A = Hin + w * 16 * p.ld_h;
    const float* __restrict__ bias = d.b[l] + grp * d.gs_b[l];
    for (int nt = 0; nt < ntiles; ++nt) {
      f32x4 acc = mma_16x16(A, p.ld_h, Wb + nt * 16 * ldw, ldw, K, zero4());
      const int col = nt * 16 + acc_col();
      const float bv = col < dout ? bias[col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = w * 16 + acc_row(i);
        const float v = col < dout ? apply_act(act, acc[i] + bv) : 0.f;
        if (last) {
          const int gr = row0 + r;
          if (gr < B && col < dout) Y[(size_t)gr * dout + col] = v;
        } else {
          Hout[r * p.ld_h + col] = to_bf16(v);
        }
      }
    }
    bf16* t = Hin;
    Hin = Hout;
    Hout = t;
  }
}

// Sum of this lane's 4 accumulator rows over the wave's 16 rows, for column acc_col().
__device__ __forceinline__ float wave_colsum(float s) {
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
  return s;
}

__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// kDisc: dY is not read; it is formed from the logits and labels (see DiscLoss) and the
// block's loss statistics are written next to its gradient slab row.
template <int NW, bool kDisc>
__global__ __launch_bounds__(64 * NW) void tmlp_bwd_kernel(MLPDesc d, TmlpPlan p, const float* __restrict__ X,
                                                           const float* __restrict__ dY, int B, float* __restrict__ dX,
                                                           MLPGrads g, float* __restrict__ slab, DiscLoss dl) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float disc_st[NW][kDiscStats];
  float st[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int L = d.n_layers;
  char* q = smem;
  bf16* Wb = reinterpret_cast<bf16*>(q);
  q += p.w_bytes;
  bf16* Hs[kMaxLayers];
  for (int l = 0; l < L; ++l) {
    Hs[l] = reinterpret_cast<bf16*>(q);
    q += p.h_bytes;
  }
  bf16* HT = reinterpret_cast<bf16*>(q);
  q += p.ht_bytes;
  bf16* dZ[2];
  bf16* dZT[2];
  for (int z = 0; z < 2; ++z) {
    dZ[z] = reinterpret_cast<bf16*>(q);
    q += p.h_bytes;
    dZT[z] = reinterpret_cast<bf16*>(q);
    q += p.ht_bytes;
  }
  float* dbs = reinterpret_cast<float*>(q);  // [2][NW][dmax_pad]

  const int row0 = blockIdx.x * p.rows;
  const int w = wave_id();
  const int ROWS = p.rows;
  const bool direct = !kDisc && gridDim.x == 1;
  const long long grp = blockIdx.y;  // grouped launch: this group's inputs / params / grads
  X += grp * d.gs_x;
  if (dY) dY += grp * d.gs_y;
  if (dX) dX += grp * d.gs_x;
  float* slab_row = direct ? nullptr : slab + ((size_t)grp * gridDim.x + blockIdx.x) * p.n_params;

  lds_zero(smem, p.bwd_lds);
  __syncthreads();
  stage_input(Hs[0], p.ld_h, X, B, row0, ROWS, d);

  // ---------------- forward recompute (keeps every layer input in LDS) + last-layer dZ
  for (int l = 0; l < L; ++l) {
    const int din = d.dims[l], dout = d.dims[l + 1];
    __syncthreads();
    stage_w(Wb, d.W[l] + grp * d.gs_w[l], dout, din, false);
    __syncthreads();
    const int K = pad32(din), ldw = ld_for_k(din);
    const int act = layer_act(d, l);
    const bool last = l == L - 1;
    const int ntiles = pad32(dout) / 16;
    const bf16* A = Hs[l] + w * 16 * p.ld_h;
    for (int nt = 0; nt < ntiles; ++nt) {
      f32x4 acc = mma_16x16(A, p.ld_h, Wb + nt * 16 * ldw, ldw, K, zero4());
      const int col = nt * 16 + acc_col();
      const float bv = col < dout ? d.b[l][grp * d.gs_b[l] + col] : 0.f;
      float colsum = 0.f;
      float dzv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = w * 16 + acc_row(i);
        const float h = col < dout ? apply_act(act, acc[i] + bv) : 0.f;
        if (!last) {
          Hs[l + 1][r * p.ld_h + col] = to_bf16(h);
        } else {
          const int gr = row0 + r;
          float dy;
          if constexpr (kDisc) {
            dy = 0.f;
            if (gr < B && col == 0) {
              const float y = gr < dl.n_expert ? 1.f : 0.f;
              const float sg = 1.f / (1.f + expf(-h));
              const float sp = fmaxf(h, 0.f) + log1pf(expf(-fabsf(h)));  // softplus(z)
              dy = (sg - y) * dl.scale;
              const bool gen_pred = h < 0.f, gen_true = y == 0.f, correct = gen_pred == gen_true;
              st[0] += sp - h * y;  // BCE-with-logits
              st[1] += correct ? 1.f : 0.f;
              st[2] += gen_pred ? 1.f : 0.f;
              st[3] += (!gen_true && correct) ? 1.f : 0.f;
              st[4] += (gen_true && correct) ? 1.f : 0.f;
              st[5] += sp - h * sg;  // entropy of Bernoulli(sigmoid(z))
            }
          } else {
            dy = (gr < B && col < dout) ? dY[(size_t)gr * dout + col] : 0.f;
          }
          float dz = dy * act_grad_from_out(act, h);
          dzv[i] = dz;
          colsum += dz;
          dZ[0][r * p.ld_h + col] = to_bf16(dz);
        }
      }
      if (last) {
        // dZ^T image: [col][rows], this lane's 4 consecutive rows are contiguous
        const int r0 = w * 16 + acc_row(0);
        bf16x4 v4 = {to_bf16(dzv[0]), to_bf16(dzv[1]), to_bf16(dzv[2]), to_bf16(dzv[3])};
        *reinterpret_cast<bf16x4*>(&dZT[0][col * p.ld_ht + r0]) = v4;
        colsum = wave_colsum(colsum);
        if (lane_id() < 16) dbs[(0 * NW + w) * p.dmax_pad + col] = colsum;
      }
    }
  }

  if constexpr (kDisc) {
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const float v = wave_sum64(st[k]);
      if (lane_id() == 0) disc_st[w][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < kDiscStats) {
      float v = 0.f;
      if (threadIdx.x < 6)
        for (int ww = 0; ww < NW; ++ww) v += disc_st[ww][threadIdx.x];
      dl.stats_slab[(size_t)blockIdx.x * kDiscStats + threadIdx.x] = v;
    }
  }

  // ---------------- backward
  int z = 0;
  for (int l = L - 1; l >= 0; --l) {
    const int din = d.dims[l], dout = d.dims[l + 1];
    __syncthreads();
    // H^T image of this layer's input: HT[i][r] for i < pad32(din)
    {
      const int C = pad32(din);
      for (int e = threadIdx.x; e < C * ROWS; e += blockDim.x) {
        const int i = e / ROWS, r = e - i * ROWS;
        HT[i * p.ld_ht + r] = Hs[l][r * p.ld_h + i];
      }
    }
    if (l > 0 || dX != nullptr) stage_w(Wb, d.W[l] + grp * d.gs_w[l], dout, din, true);
    __syncthreads();

    // db_l: reduce wave partials
    for (int c = threadIdx.x; c < dout; c += blockDim.x) {
      float s = 0.f;
      for (int ww = 0; ww < NW; ++ww) s += dbs[(z * NW + ww) * p.dmax_pad + c];
      if (direct) {
        float* dst = g.db[l] + grp * d.gs_b[l] + c;
        *dst = g.accumulate ? *dst + s : s;
      } else {
        slab_row[p.param_off[2 * l + 1] + c] = s;
      }
    }
    // dW_l = dZ^T (out x rows) . H (rows x in), tiles spread over waves
    {
      const int mt = pad16(dout) / 16, ntl = pad16(din) / 16;
      for (int t = w; t < mt * ntl; t += NW) {
        const int tm = t / ntl, tn = t - tm * ntl;
        f32x4 acc = mma_16x16(dZT[z] + tm * 16 * p.ld_ht, p.ld_ht, HT + tn * 16 * p.ld_ht, p.ld_ht, ROWS, zero4());
        const int in = tn * 16 + acc_col();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int o = tm * 16 + acc_row(i);
          if (o < dout && in < din) {
            if (direct) {
              float* dst = g.dW[l] + grp * d.gs_w[l] + o * din + in;
              *dst = g.accumulate ? *dst + acc[i] : acc[i];
            } else {
              slab_row[p.param_off[2 * l] + o * din + in] = acc[i];
            }
          }
        }
      }
    }
    // G = dZ_l . W_l (rows x in) -> dZ_{l-1} = G * act'(H_l), or dX for l == 0
    __syncthreads();
    if (l > 0 || dX != nullptr) {
      const int K = pad32(dout), ldw = ld_for_k(dout);
      const int act_prev = l > 0 ? layer_act(d, l - 1) : ACT_IDENTITY;
      const bf16* A = dZ[z] + w * 16 * p.ld_h;
      const int ntiles = pad32(din) / 16;
      for (int nt = 0; nt < ntiles; ++nt) {
        f32x4 acc = mma_16x16(A, p.ld_h, Wb + nt * 16 * ldw, ldw, K, zero4());
        const int col = nt * 16 + acc_col();
        if (l > 0) {
          float colsum = 0.f;
          float dzv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = w * 16 + acc_row(i);
            const float h = from_bf16(Hs[l][r * p.ld_h + col]);
            const float dz = col < din ? acc[i] * act_grad_from_out(act_prev, h) : 0.f;
            dzv[i] = dz;
            colsum += dz;
            dZ[z ^ 1][r * p.ld_h + col] = to_bf16(dz);
          }
          const int r0 = w * 16 + acc_row(0);
          bf16x4 v4 = {to_bf16(dzv[0]), to_bf16(dzv[1]), to_bf16(dzv[2]), to_bf16(dzv[3])};
          *reinterpret_cast<bf16x4*>(&dZT[z ^ 1][col * p.ld_ht + r0]) = v4;
          colsum = wave_colsum(colsum);
          if (lane_id() < 16) dbs[((z ^ 1) * NW + w) * p.dmax_pad + col] = colsum;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int gr = row0 + w * 16 + acc_row(i);
            if (gr < B && col < din) {
              float gx = acc[i];
              if (d.norm_mean) {
                const long long go = grp * d.gs_norm;
                const float sc = rsqrtf(d.norm_var[go + col] + d.norm_eps);
                if (d.norm_clip > 0.f) {
                  const float xn = (X[(size_t)gr * din + col] - d.norm_mean[go + col]) * sc;
                  if (xn <= -d.norm_clip || xn >= d.norm_clip) gx = 0.f;
                }
                gx *= sc;
              }
              dX[(size_t)gr * din + col] = gx;
            }
          }
        }
      }
    }
    z ^= 1;
  }
}

// grads[p] (+)= sum_b slab[b][p]  (fixed order -> deterministic)
__global__ void tmlp_grad_reduce_kernel(const float* __restrict__ slab, int nblk, TmlpPlan p, MLPDesc d, MLPGrads g) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.n_params) return;
  const long long grp = blockIdx.y;
  slab += (size_t)grp * nblk * p.n_params;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += slab[(size_t)b * p.n_params + e];
  // locate parameter tensor
  for (int l = d.n_layers - 1; l >= 0; --l) {
    if (e >= p.param_off[2 * l + 1]) {
      float* dst = g.db[l] + grp * d.gs_b[l] + (e - p.param_off[2 * l + 1]);
      *dst = g.accumulate ? *dst + s : s;
      return;
    }
    if (e >= p.param_off[2 * l]) {
      float* dst = g.dW[l] + grp * d.gs_w[l] + (e - p.param_off[2 * l]);
      *dst = g.accumulate ? *dst + s : s;
      return;
    }
  }
}

}  // namespace

int tmlp_disc_blocks(const MLPDesc& d, int B) {
  const TmlpPlan p = plan_tmlp(d, tmlp_waves_for(d));
  return (B + p.rows - 1) / p.rows;
}

hipError_t tmlp_disc_fwd_bwd(const MLPDesc& d, const float* X, int B, const DiscLoss& dl, float* slab, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (d.dims[d.n_layers] != 1 || d.out_act != ACT_IDENTITY) return hipErrorInvalidValue;
  const int nw = tmlp_waves_for(d);
  TmlpPlan p = plan_tmlp(d, nw);
  const int nblk = (B + p.rows - 1) / p.rows;
  const MLPGrads g{};
  if (nw == 4)
    hipLaunchKernelGGL((tmlp_bwd_kernel<4, true>), dim3(nblk), dim3(256), p.bwd_lds, s, d, p, X, nullptr, B, nullptr, g,
                       slab, dl);
  else
    hipLaunchKernelGGL((tmlp_bwd_kernel<2, true>), dim3(nblk), dim3(128), p.bwd_lds, s, d, p, X, nullptr, B, nullptr, g,
                       slab, dl);
  return hipGetLastError();
}

int tmlp_waves_for(const MLPDesc& d) {
  TmlpPlan p4 = plan_tmlp(d, 4);
  return p4.bwd_lds <= 160 * 1024 ? 4 : 2;
}

size_t tmlp_slab_floats(const MLPDesc& d, int B) {
  const int nw = tmlp_waves_for(d);
  TmlpPlan p = plan_tmlp(d, nw);
  const int nblk = (B + p.rows - 1) / p.rows;
  return nblk > 1 ? (size_t)nblk * p.n_params : 0;
}

hipError_t tmlp_forward(const MLPDesc& d, const float* X, int B, float* Y, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  // forward-only: 4 waves unless the forward image itself is too large
  TmlpPlan p = plan_tmlp(d, 4);
  if (p.fwd_lds > 160 * 1024) p = plan_tmlp(d, 2);
  const int nblk = (B + p.rows - 1) / p.rows;
  const unsigned G = d.groups > 1 ? (unsigned)d.groups : 1u;
  if (p.waves == 4)
    hipLaunchKernelGGL(tmlp_fwd_kernel<4>, dim3(nblk, G), dim3(256), p.fwd_lds, s, d, p, X, B, Y);
  else
    hipLaunchKernelGGL(tmlp_fwd_kernel<2>, dim3(nblk, G), dim3(128), p.fwd_lds, s, d, p, X, B, Y);
  return hipGetLastError();
}

hipError_t tmlp_backward(const MLPDesc& d, const float* X, const float* dY, int B, float* dX, const MLPGrads& g,
                         float* slab, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const int nw = tmlp_waves_for(d);
  TmlpPlan p = plan_tmlp(d, nw);
  const int nblk = (B + p.rows - 1) / p.rows;
  if (nblk > 1 && slab == nullptr) return hipErrorInvalidValue;
  const DiscLoss none{};
  const unsigned G = d.groups > 1 ? (unsigned)d.groups : 1u;
  if (nw == 4)
    hipLaunchKernelGGL((tmlp_bwd_kernel<4, false>), dim3(nblk, G), dim3(256), p.bwd_lds, s, d, p, X, dY, B, dX, g, slab,
                       none);
  else
    hipLaunchKernelGGL((tmlp_bwd_kernel<2, false>), dim3(nblk, G), dim3(128), p.bwd_lds, s, d, p, X, dY, B, dX, g, slab,
                       none);
  if (nblk > 1) {
    hipLaunchKernelGGL(tmlp_grad_reduce_kernel, dim3((p.n_params + 255) / 256, G), dim3(256), 0, s, slab, nblk, p, d, g);
  }
  return hipGetLastError();
}

}  // namespace ia

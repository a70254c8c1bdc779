// Block-level MLP building blocks shared by the fused discriminator / reward-model kernels
// (airl_disc.hip, pref_rm.hip): a 64-row block of 4 waves stages bf16 row and weight images
// in LDS, runs the forward with each wave on its own 16 rows (no barrier between layers),
// and the backward writes dW / db of the block into one gradient slab row (fixed-order
// reductions only, so replicas are bitwise reproducible). v_mfma_f32_16x16x32_bf16 with
// fp32 accumulation (ia/mfma.h).
#pragma once
#include <hip/hip_runtime.h>

#include "ia/mfma.h"
#include "launchers.h"

namespace ia {
namespace dmlp {

constexpr int kRows = 64;  // rows per block (4 waves x 16)
constexpr int kNW = 4;

__device__ inline void chan_merge(float* rmean, float* rvar, int count, int c, float bmean, float bvar, int n) {
  // RunningNorm.update_stats (networks.py:94-111), same fp32 operation order
  const float fc = (float)count, fn = (float)n, tot = (float)(count + n);
  const float delta = bmean - rmean[c];
  rmean[c] += delta * fn / tot;
  float v = rvar[c] * fc;
  v += bvar * fn;
  v += delta * delta * fc * fn / tot;
  rvar[c] = v / tot;
}


// LDS images are bf16 [row][k] with row stride ld (K-contiguous MFMA operands, mfma.h).

// rows [row0, row0 + 64) of X [B][din] -> image H (normalised with nrm slot: mean, rstd)
__device__ inline void stage_rows(lbf* H, int ld, const float* __restrict__ X, int din, int B, int row0, const float* nrm) {
  const int kp = pad32(din);
  for (int e = threadIdx.x; e < kRows * kp; e += blockDim.x) {
    const int r = e / kp, c = e - r * kp;
    const int gr = row0 + r;
    float v = 0.f;
    if (gr < B && c < din) v = (X[(size_t)gr * din + c] - nrm[c]) * nrm[128 + c];
    H[r * ld + c] = to_bf16(v);
  }
}

// weight image: [o][i] (forward B^T operand) or [i][o] (transposed, backward), zero padded
__device__ inline void stage_weights(lbf* dst, const float* __restrict__ W, int dout, int din, bool transposed) {
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

__device__ inline float act_apply(int act, float x) { return apply_act(act, x); }

// Forward of an MLP over the staged input Hs[0] (64 rows); hidden outputs go to Hs[l + 1]
// (kept for the backward pass), the last layer's (fp32, bias added, identity) outputs to
// out[row * out_ld + col] for col < dims[L] (<= 16). Wf[l]: pre-staged weight images.
// Each wave works on its own 16 rows only, so layers need no barrier between them.
// Hs / Wf (and Wt / dZ / dZT below): anything indexable by layer -- pointer arrays, or
// accessors that compute the image address (pref_rm.hip: a run-time-indexed array of LDS
// pointers would live in scratch).
template <class HA, class WA>
__device__ inline void mlp_forward(const AirlNet& net, const HA& Hs, int ld, const WA& Wf, lfl* out, int out_ld) {
  const int w = wave_id();
  for (int l = 0; l < net.n_layers; ++l) {
    const int din = net.dims[l], dout = net.dims[l + 1];
    const lbf* Wimg = Wf[l];
    const int K = pad32(din), ldw = ld_for_k(din);
    const bool last = l == net.n_layers - 1;
    const int ntiles = last ? 1 : pad32(dout) / 16;
    const lbf* A = Hs[l] + w * 16 * ld;
    for (int nt = 0; nt < ntiles; ++nt) {
      f32x4 acc = mma_16x16(A, ld, Wimg + nt * 16 * ldw, ldw, K, zero4());
      const int col = nt * 16 + acc_col();
      const float bv = col < dout ? net.b[l][col] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = w * 16 + acc_row(i);
        if (last) {
          if (col < dout) out[r * out_ld + col] = acc[i] + bv;
        } else {
          Hs[l + 1][r * ld + col] = to_bf16(col < dout ? act_apply(net.hidden_act, acc[i] + bv) : 0.f);
        }
      }
    }
  }
}

__device__ inline float wave_colsum(float s) {
  s += __shfl_xor(s, 16);
  s += __shfl_xor(s, 32);
  return s;
}

// Backward of an MLP (identity output, dout = 1) from per-row output gradients dy[64]:
// dW / db into slab[param offsets] (acc: add to what an earlier pass of this block wrote).
// Scratch: HT [feature][row] (ld_ht), dZ [row][k] (ld) and dZT [k][row] (ld_ht), x2.
template <class HA, class WA, class ZA>
__device__ inline void mlp_backward(const AirlNet& net, const HA& Hs, int ld, const WA& Wt, const lfl* dy, lbf* HT, int ld_ht,
                             const ZA& dZ, const ZA& dZT, lfl* dbs, int dmax_pad, float* slab, bool acc_mode) {
  const int w = wave_id(), lane = lane_id();
  const int L = net.n_layers;
  // last layer: dZ = dy (identity head, one output column)
  for (int e = threadIdx.x; e < kRows * 32; e += blockDim.x) {
    const int r = e >> 5, c = e & 31;
    const float v = c == 0 ? dy[r] : 0.f;
    dZ[0][r * ld + c] = to_bf16(v);
    dZT[0][c * ld_ht + r] = to_bf16(v);
  }
  lfl* dbs_head = dbs + 2 * kNW * dmax_pad;
  if (threadIdx.x == 0) {  // db of the head: fixed-order sum over rows (fp32)
    float s = 0.f;
    for (int r = 0; r < kRows; ++r) s += dy[r];
    *dbs_head = s;
  }
  int z = 0;
  bool head = true;
  for (int l = L - 1; l >= 0; --l) {
    const int din = net.dims[l], dout = net.dims[l + 1];
    __syncthreads();
    {  // H^T image of this layer's input
      const int C = pad32(din);
      for (int e = threadIdx.x; e < C * kRows; e += blockDim.x) {
        const int i = e / kRows, r = e - i * kRows;
        HT[i * ld_ht + r] = Hs[l][r * ld + i];
      }
    }
    __syncthreads();
    // db_l
    float* sb = slab + net.param_off + net.b_off[l];
    for (int c = threadIdx.x; c < dout; c += blockDim.x) {
      float s;
      if (head) {
        s = *dbs_head;
      } else {
        s = 0.f;
        for (int ww = 0; ww < kNW; ++ww) s += dbs[(z * kNW + ww) * dmax_pad + c];
      }
      sb[c] = acc_mode ? sb[c] + s : s;
    }
    // dW_l = dZ^T . H
    {
      float* sw = slab + net.param_off + net.w_off[l];
      const int mt = pad16(dout) / 16, ntl = pad16(din) / 16;
      for (int t = w; t < mt * ntl; t += kNW) {
        const int tm = t / ntl, tn = t - tm * ntl;
        f32x4 accv = mma_16x16(dZT[z] + tm * 16 * ld_ht, ld_ht, HT + tn * 16 * ld_ht, ld_ht, kRows, zero4());
        const int in = tn * 16 + acc_col();
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int o = tm * 16 + acc_row(i);
          if (o < dout && in < din) {
            float* p = sw + o * din + in;
            *p = acc_mode ? *p + accv[i] : accv[i];
          }
        }
      }
    }
    __syncthreads();
    if (l == 0) break;
    // dZ_{l-1} = (dZ_l . W_l) * act'(H_l)
    {
      const int K = pad32(dout), ldw = ld_for_k(dout);
      const lbf* A = dZ[z] + w * 16 * ld;
      const lbf* Wimg = Wt[l];
      const int ntiles = pad32(din) / 16;
      for (int nt = 0; nt < ntiles; ++nt) {
        f32x4 accv = mma_16x16(A, ld, Wimg + nt * 16 * ldw, ldw, K, zero4());
        const int col = nt * 16 + acc_col();
        float colsum = 0.f;
        float dzv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = w * 16 + acc_row(i);
          const float h = from_bf16(Hs[l][r * ld + col]);
          const float dzval = col < din ? accv[i] * act_grad_from_out(net.hidden_act, h) : 0.f;
          dzv[i] = dzval;
          colsum += dzval;
          dZ[z ^ 1][r * ld + col] = to_bf16(dzval);
        }
        const int r0 = w * 16 + acc_row(0);
        bf16x4 v4 = {to_bf16(dzv[0]), to_bf16(dzv[1]), to_bf16(dzv[2]), to_bf16(dzv[3])};
        *(lbf4*)(&dZT[z ^ 1][col * ld_ht + r0]) = v4;
        colsum = wave_colsum(colsum);
        if (lane < 16) dbs[((z ^ 1) * kNW + w) * dmax_pad + col] = colsum;
      }
    }
    z ^= 1;
    head = false;
  }
  __syncthreads();
}


}  // namespace dmlp
}  // namespace ia

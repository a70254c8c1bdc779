// Tiny-MLP (TMLP) descriptors + LDS planning shared by host launchers and kernels.
//
// A TMLP is the network shape used by every reward net / policy / value net in
// the reference: build_mlp (src/imitation/util/networks.py:204-283), SB3
// MlpExtractor + action/value heads, BasicRewardNet hid (32,32)
// (src/imitation/rewards/reward_nets.py:431), FeedForward32Policy [32,32]
// (src/imitation/policies/base.py:208-220), AIRL/PC [64,64] policies.
// Widths <= 128 go through these fused kernels; anything wider is a plain
// library GEMM (torch.nn.Linear -> hipBLASLt).
#pragma once
#include "ia/common.h"

namespace ia {

constexpr int kMaxLayers = 4;
constexpr int kMaxDim = 128;

struct MLPDesc {
  int n_layers;
  int dims[kMaxLayers + 1];
  int hidden_act;
  int out_act;
  const float* W[kMaxLayers];
  const float* b[kMaxLayers];
  const float* norm_mean;  // optional input normalisation (x - mean) * rsqrt(var + eps)
  const float* norm_var;
  float norm_eps;
  float norm_clip;  // >0: clamp normalised input to [-clip, clip]
  // Grouped launches (reward ensembles): blockIdx.y = group g reads W_l + g * gs_w[l],
  // b_l + g * gs_b[l], norm + g * gs_norm, X + g * gs_x and writes Y + g * gs_y (strides in
  // floats; 0 = shared by every group, e.g. one input batch for all members).
  int groups;
  long long gs_w[kMaxLayers], gs_b[kMaxLayers], gs_norm, gs_x, gs_y;
};

struct MLPGrads {
  float* dW[kMaxLayers];
  float* db[kMaxLayers];
  int accumulate;  // 1: add into existing grads, 0: overwrite
};

// Discriminator loss fused into the backward pass (GAIL/AIRL train_disc): the MLP output
// is the logit z of "expert"; rows [0, n_expert) are expert (label 1), the rest generator
// (label 0). dL/dz = (sigmoid(z) - y) * scale, and per-block sums of the statistics the
// reference logs (common.py compute_train_stats) go to stats_slab[block][kDiscStats].
constexpr int kDiscStats = 8;  // loss, correct, gen_pred, exp_correct, gen_correct, entropy, -, -
struct DiscLoss {
  int n_expert;
  float scale;
  float* stats_slab;
};

struct TmlpPlan {
  int rows;       // rows per block = 16 * waves
  int waves;
  int ld_h;       // ld of row-major activation images [rows][ld_h]
  int ld_ht;      // ld of transposed activation images [max_dim_pad][ld_ht]
  int dmax_pad;   // pad32 of the widest dimension
  int w_bytes, h_bytes, ht_bytes;
  int fwd_lds;    // bytes for the forward-only kernel
  int bwd_lds;    // bytes for the forward-recompute + backward kernel
  int n_params;
  int param_off[kMaxLayers * 2];  // flat offsets of W_l, b_l inside a gradient slab row
};

__host__ __device__ inline int layer_act(const MLPDesc& d, int l) {
  return l == d.n_layers - 1 ? d.out_act : d.hidden_act;
}

__host__ inline TmlpPlan plan_tmlp(const MLPDesc& d, int waves) {
  TmlpPlan p{};
  p.waves = waves;
  p.rows = 16 * waves;
  int dm = 0;
  for (int l = 0; l <= d.n_layers; ++l) dm = dm > d.dims[l] ? dm : d.dims[l];
  p.dmax_pad = pad32(dm);
  p.ld_h = ld_for_k(dm);
  p.ld_ht = ld_for_k(p.rows);
  p.w_bytes = p.dmax_pad * ld_for_k(dm) * 2;          // one weight image (W or W^T)
  p.h_bytes = p.rows * p.ld_h * 2;                    // one [rows][d] image
  p.ht_bytes = p.dmax_pad * p.ld_ht * 2;              // one [d][rows] image
  p.fwd_lds = p.w_bytes + 2 * p.h_bytes;
  // bwd: W image, L activation images (layer inputs), H^T scratch, 2x (dZ, dZ^T), db scratch
  p.bwd_lds = p.w_bytes + d.n_layers * p.h_bytes + p.ht_bytes + 2 * (p.h_bytes + p.ht_bytes) + 2 * waves * p.dmax_pad * 4;
  int off = 0;
  for (int l = 0; l < d.n_layers; ++l) {
    p.param_off[2 * l] = off;
    off += d.dims[l + 1] * d.dims[l];
    p.param_off[2 * l + 1] = off;
    off += d.dims[l + 1];
  }
  p.n_params = off;
  return p;
}

}  // namespace ia

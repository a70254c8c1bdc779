// Fused AIRL discriminator update for the device adversarial engine.
//
// Reference semantics (one minibatch of AdversarialTrainer.train_disc,
// src/imitation/algorithms/adversarial/common.py:317-389 + _make_disc_train_batches
// :521-632, AIRL logits airl.py:114-119, ShapedRewardNet reward_nets.py:674-809):
//
//   1. expert rows then generator rows -> obs s, acts a, next_obs s', dones d
//   2. log pi(a|s) of the generator policy under no_grad, in training mode: the policy's
//      features RunningNorm merges the batch moments of s first (networks.py:79-91)
//   3. r = base([s, a, ...]) with its input RunningNorm merging the batch moments of its
//      input columns first;  Phi(s') then Phi(s) with the potential's RunningNorm merging
//      the moments of s' and then of s (two train-mode calls, in that order)
//   4. logit = r + gamma (1 - d) Phi(s') - Phi(s) - log pi;  BCE(logit, expert = 1) * mb / B
//   5. backward into the base and potential MLPs (the potential gets both passes), Adam
//
// which the autograd path runs as ~60 launches per update. Here it is four:
//
//   airl_gather     rows gathered by index into S, S', actions, dones and the base-net
//                   input X; per-block shifted column sums of X, S', S for the moments
//   airl_norm       fixed-order (fp64) reduction of the block sums -> batch moments; the
//                   Chan merges of the policy, base and potential RunningNorms (the
//                   potential twice: s', then s) and the (mean, rsqrt(var + eps)) each
//                   forward pass normalises with
//   airl_fwd_bwd    per 64-row block: policy forward -> log pi, base forward, potential
//                   forward on s' and on s, logit / BCE / statistics, backward of the base
//                   and of both potential passes -> one gradient slab row per block
//   disc_adam       (disc.hip) fixed-order slab reduction + torch Adam on the flat params
//
// Matrix work is v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulation), as in the
// GAIL discriminator (tmlp.hip); every reduction has a fixed order, so replicas are
// bitwise reproducible.
#include <hip/hip_runtime.h>

#include "ia/dmlp.h"
#include "ia/mfma.h"
#include "launchers.h"

namespace ia {
namespace {

using namespace dmlp;  // kRows / kNW, staging, MLP forward / backward (ia/dmlp.h)
constexpr int kGatherRows = 16;  // 8 rows per thread: >= 256 blocks for a 2 x 2048-row batch
constexpr int kNormPhases = 8;

// ------------------------------------------------------------------ gather
__device__ __forceinline__ float act_val(const AirlDiscArgs& a, bool expert, int64_t src, int j) {
  if (a.act_discrete) {
    const int64_t* acts = expert ? a.e_acts_i : a.g_acts_i;
    return (int)acts[src] == j ? 1.f : 0.f;
  }
  return (expert ? a.e_acts : a.g_acts)[src * a.A + j];
}

// column c of the base-net input for source row src
__device__ __forceinline__ float base_col(const AirlDiscArgs& a, bool expert, int64_t src, int c) {
  const int D = a.D;
  if (a.use_state) {
    if (c < D) return (expert ? a.e_obs : a.g_obs)[src * D + c];
    c -= D;
  }
  if (a.use_action) {
    if (c < a.aw) return act_val(a, expert, src, c);
    c -= a.aw;
  }
  if (a.use_next_state) {
    if (c < D) return (expert ? a.e_next_obs : a.g_next_obs)[src * D + c];
    c -= D;
  }
  return (expert ? a.e_dones : a.g_dones)[src] ? 1.f : 0.f;
}

// statistics columns: [0, din_b) base input, [din_b, din_b + D) s', [din_b + D, din_b + 2D) s
__global__ __launch_bounds__(256) void airl_gather_kernel(AirlDiscArgs a, int k) {
  __shared__ float red[2][2][128];
  const int c = threadIdx.x & 127, ph = threadIdx.x >> 7;
  const int n = 2 * a.mb, D = a.D, nb = a.din_b;
  const int ncol = nb + 2 * D;
  const int r0 = blockIdx.x * kGatherRows;
  const int64_t* e_idx = a.e_idx + (size_t)k * a.mb;
  const int64_t* g_idx = a.g_idx + (size_t)k * a.mb;
  const bool col_ok = c < ncol;
  float shift = 0.f;
  if (col_ok) {
    if (c < nb) shift = a.b_mean ? a.b_mean[c] : 0.f;
    else shift = a.p_mean ? a.p_mean[(c - nb) % D] : 0.f;
  }
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int rr = ph; rr < kGatherRows; rr += 2) {
    const int r = r0 + rr;
    if (r >= n) break;
    const bool expert = r < a.mb;
    const int64_t src = expert ? e_idx[r] : g_idx[r - a.mb];
    float v = 0.f;
    if (col_ok) {
      if (c < nb) {
        v = base_col(a, expert, src, c);
        a.Xb[(size_t)r * nb + c] = v;
      } else if (c < nb + D) {
        v = (expert ? a.e_next_obs : a.g_next_obs)[src * D + (c - nb)];
        a.S2[(size_t)r * D + (c - nb)] = v;
      } else {
        v = (expert ? a.e_obs : a.g_obs)[src * D + (c - nb - D)];
        a.S[(size_t)r * D + (c - nb - D)] = v;
      }
      const float dv = v - shift;
      s1 += dv;
      s2 += dv * dv;
    }
    // raw actions for log pi (Gaussian values / categorical index) and dones (each row is
    // handled by one phase)
    if (c < a.aw_pi) {
      float av;
      if (a.act_discrete) av = (float)(expert ? a.e_acts_i : a.g_acts_i)[src];
      else av = (expert ? a.e_acts : a.g_acts)[src * a.A + c];
      a.Act[(size_t)r * a.aw_pi + c] = av;
    }
    if (c == 127) a.Done[r] = (expert ? a.e_dones : a.g_dones)[src] ? 1.f : 0.f;
  }
  red[ph][0][c] = s1;
  red[ph][1][c] = s2;
  __syncthreads();
  if (ph == 0 && col_ok) {
    float* out = a.partials + (size_t)blockIdx.x * 2 * ncol;
    out[c] = red[0][0][c] + red[1][0][c];
    out[ncol + c] = red[0][1][c] + red[1][1][c];
  }
}

// ------------------------------------------------------------------ norms
__device__ __forceinline__ void put_nrm(float* nrm, int slot, int c, const float* mean, const float* var, float eps) {
  nrm[slot * 256 + c] = mean ? mean[c] : 0.f;
  nrm[slot * 256 + 128 + c] = mean ? rsqrtf(var[c] + eps) : 1.f;
}

// 1024 threads = 8 block-phases x 128 columns (fixed-order reduction, as disc_norm_kernel)
__global__ __launch_bounds__(128 * kNormPhases) void airl_norm_kernel(AirlDiscArgs a, int mode, int n_total) {
  __shared__ double red[kNormPhases][2][128];
  __shared__ float bm[128], bv[128];
  const int c = threadIdx.x & 127, ph = threadIdx.x >> 7;
  const int D = a.D, nb = a.din_b, ncol = nb + 2 * D;
  const int n = mode == 2 ? n_total : 2 * a.mb;
  if (mode != 2) {
    double s1 = 0.0, s2 = 0.0;
    if (c < ncol)
      for (int b = ph; b < a.gather_blocks; b += kNormPhases) {
        const float* p = a.partials + (size_t)b * 2 * ncol;
        s1 += (double)p[c];
        s2 += (double)p[ncol + c];
      }
    red[ph][0][c] = s1;
    red[ph][1][c] = s2;
    __syncthreads();
  }
  if (ph == 0 && c < ncol) {
    double S1 = 0.0, S2 = 0.0;
    if (mode == 2) {
      S1 = a.sums[c];
      S2 = a.sums[ncol + c];
    } else {
      for (int q = 0; q < kNormPhases; ++q) {
        S1 += red[q][0][c];
        S2 += red[q][1][c];
      }
    }
    if (mode == 1) {
      a.sums[c] = S1;
      a.sums[ncol + c] = S2;
    } else {
      float shift = 0.f;
      if (c < nb) shift = a.b_mean ? a.b_mean[c] : 0.f;
      else shift = a.p_mean ? a.p_mean[(c - nb) % D] : 0.f;
      const double m = S1 / n;
      double var = S2 / n - m * m;
      if (var < 0.0) var = 0.0;
      bm[c] = (float)((double)shift + m);
      bv[c] = (float)var;
    }
  }
  if (mode == 1) return;
  __syncthreads();
  if (threadIdx.x < 128) {
    const int bc = a.b_count ? *a.b_count : 0;
    const int pc = a.p_count ? *a.p_count : 0;
    const int qc = a.q_count ? *a.q_count : 0;
    // base input norm over its own columns
    if (c < nb) {
      if (a.merge_b && a.b_mean) chan_merge(a.b_mean, a.b_var, bc, c, bm[c], bv[c], n);
      put_nrm(a.nrm, 1, c, a.b_mean, a.b_var, a.eps_b);
    }
    if (c < D) {
      // potential: s' first (Phi(s') is evaluated first), then s
      if (a.merge_p && a.p_mean) chan_merge(a.p_mean, a.p_var, pc, c, bm[nb + c], bv[nb + c], n);
      put_nrm(a.nrm, 2, c, a.p_mean, a.p_var, a.eps_p);
      if (a.merge_p && a.p_mean) chan_merge(a.p_mean, a.p_var, pc + n, c, bm[nb + D + c], bv[nb + D + c], n);
      put_nrm(a.nrm, 3, c, a.p_mean, a.p_var, a.eps_p);
      // policy features norm: moments of s (deferred: kept for airl_q_merge, which writes row 0)
      const bool defer = a.merge_q && a.q_mean && a.q_defer;
      if (defer) {
        a.q_defer[c] = bm[nb + D + c];
        a.q_defer[128 + c] = bv[nb + D + c];
      } else {
        if (a.merge_q && a.q_mean) chan_merge(a.q_mean, a.q_var, qc, c, bm[nb + D + c], bv[nb + D + c], n);
        put_nrm(a.nrm, 0, c, a.q_mean, a.q_var, a.eps_q);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (a.merge_b && a.b_count) *a.b_count += n;
    if (a.merge_p && a.p_count) *a.p_count += 2 * n;
    if (a.merge_q && a.q_count && !a.q_defer) *a.q_count += n;
  }
}

// The policy-norm merges airl_norm deferred, in staging order: the same chan_merge sequence on
// the same moments as merging in airl_norm (bitwise), so the staging itself (gathers, base and
// potential merges) can run while PPO still uses the policy norm. One thread per column.
__global__ __launch_bounds__(128) void airl_q_merge_kernel(AirlDiscArgs a, int count, long long stride, int n) {
  const int c = threadIdx.x;
  const int qc = *a.q_count;
  __syncthreads();
  if (c < a.D) {
    for (int j = 0; j < count; ++j) {
      float* nrm = a.nrm + (size_t)j * stride;
      const float* dq = a.q_defer + (size_t)j * stride;
      chan_merge(a.q_mean, a.q_var, qc + j * n, c, dq[c], dq[128 + c], n);
      put_nrm(nrm, 0, c, a.q_mean, a.q_var, a.eps_q);
    }
  }
  if (c == 0) *a.q_count = qc + count * n;
}

__global__ __launch_bounds__(64 * kNW) void airl_fwd_bwd_kernel(AirlDiscArgs a, AirlPlan p, int k) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ float fl[6][kRows];  // log pi, r, Phi(s'), Phi(s), grads
  __shared__ float heads[kRows][17];
  __shared__ float st_w[kNW][kDiscStats];
  lbf* Wf[3][kAirlMaxLayers];
  lbf* Wt[3][kAirlMaxLayers];
  for (int q = 0; q < 3; ++q)
    for (int l = 0; l < kAirlMaxLayers; ++l) {
      Wf[q][l] = (lbf*)(smem + p.wf_off[q][l]);
      Wt[q][l] = (lbf*)(smem + p.wt_off[q][l]);
    }
  lbf* Pimg[2] = {(lbf*)(smem + p.scratch_off), (lbf*)(smem + p.scratch_off + p.pimg_bytes)};
  lbf* Bh[kAirlMaxLayers];
  lbf* Qh[kAirlMaxLayers];
  lbf* Rh[kAirlMaxLayers];
  {
    const int nb = a.base.n_layers, np = a.pot.n_layers;
    for (int l = 0; l < kAirlMaxLayers; ++l) {
      Bh[l] = (lbf*)(smem + p.rimg_off + (size_t)min(l, nb - 1) * p.rimg_bytes);
      Qh[l] = (lbf*)(smem + p.rimg_off + (size_t)(nb + min(l, np - 1)) * p.rimg_bytes);
      Rh[l] = (lbf*)(smem + p.rimg_off + (size_t)(nb + np + min(l, np - 1)) * p.rimg_bytes);
    }
  }
  // backward scratch aliases the policy images (the policy pass is over by then)
  char* sc = smem + p.scratch_off;
  lbf* HT = (lbf*)(sc);
  lbf* dZ[2] = {(lbf*)(sc + p.ht_bytes), (lbf*)(sc + p.ht_bytes + p.rimg_bytes)};
  lbf* dZT[2] = {(lbf*)(sc + p.ht_bytes + 2 * p.rimg_bytes), (lbf*)(sc + p.ht_bytes + 2 * p.rimg_bytes + p.ht_bytes)};
  lfl* dbs = (lfl*)(sc + 3 * p.ht_bytes + 2 * p.rimg_bytes);

  const int n = 2 * a.mb;
  const int row0 = blockIdx.x * kRows;
  const int tid = threadIdx.x, w = wave_id(), lane = lane_id();
  // optional phase timestamps (block 0, thread 0): a.prof[0..7]
  const bool stamp = a.prof != nullptr && blockIdx.x == 0 && threadIdx.x == 0;
  unsigned long long t_0 = stamp ? clock64() : 0;
  lds_zero(smem, p.lds_bytes);
  __syncthreads();
  // every weight image once, up front (forward [o][i]; transposed [i][o] for the backward of
  // the reward nets' layers >= 1), all loads in flight together
  {
    const AirlNet* nets[3] = {&a.pol, &a.base, &a.pot};
    for (int q = 0; q < 3; ++q)
      for (int l = 0; l < nets[q]->n_layers; ++l) {
        stage_weights(Wf[q][l], nets[q]->W[l], nets[q]->dims[l + 1], nets[q]->dims[l], false);
        if (q > 0 && l > 0) stage_weights(Wt[q][l], nets[q]->W[l], nets[q]->dims[l + 1], nets[q]->dims[l], true);
      }
  }
  stage_rows(Pimg[0], p.ldp, a.S, a.D, n, row0, a.nrm + 0 * 256);
  stage_rows(Bh[0], p.ldr, a.Xb, a.din_b, n, row0, a.nrm + 1 * 256);
  stage_rows(Qh[0], p.ldr, a.S2, a.D, n, row0, a.nrm + 2 * 256);
  stage_rows(Rh[0], p.ldr, a.S, a.D, n, row0, a.nrm + 3 * 256);
  __syncthreads();

  unsigned long long t_1 = stamp ? clock64() : 0;
  // ---- policy forward -> log pi(a|s)  (each wave on its own 16 rows)
  {
    const AirlNet& pn = a.pol;
    // ping-pong: layer l reads Pimg[l & 1], writes Pimg[(l + 1) & 1]
    for (int l = 0; l < pn.n_layers; ++l) {
      const int din = pn.dims[l], dout = pn.dims[l + 1];
      const lbf* Wimg = Wf[0][l];
      const int K = pad32(din), ldw = ld_for_k(din);
      const bool last = l == pn.n_layers - 1;
      const int ntiles = last ? 1 : pad32(dout) / 16;
      const lbf* A = Pimg[l & 1] + w * 16 * p.ldp;
      lbf* O = Pimg[(l + 1) & 1];
      for (int nt = 0; nt < ntiles; ++nt) {
        f32x4 acc = mma_16x16(A, p.ldp, Wimg + nt * 16 * ldw, ldw, K, zero4());
        const int col = nt * 16 + acc_col();
        const float bv = col < dout ? pn.b[l][col] : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = w * 16 + acc_row(i);
          if (last) heads[r][col] = col < dout ? acc[i] + bv : 0.f;
          else O[r * p.ldp + col] = to_bf16(col < dout ? act_apply(pn.hidden_act, acc[i] + bv) : 0.f);
        }
      }
    }
    __syncthreads();
    if (tid < kRows) {
      const int r = tid, gr = row0 + r;
      float lp = 0.f;
      if (gr < n) {
        const int A = a.A;
        if (a.act_discrete) {
          float mx = -INFINITY;
          for (int j = 0; j < A; ++j) mx = fmaxf(mx, heads[r][j]);
          float zs = 0.f;
          for (int j = 0; j < A; ++j) zs += expf(heads[r][j] - mx);
          const int ai = (int)a.Act[(size_t)gr * a.aw_pi];
          lp = heads[r][ai] - mx - logf(zs);
        } else {
          for (int j = 0; j < A; ++j) {
            const float ls = a.log_std[j];
            const float zz = (a.Act[(size_t)gr * a.aw_pi + j] - heads[r][j]) * expf(-ls);
            lp += -0.5f * zz * zz - ls - 0.91893853320467274f;
          }
        }
      }
      fl[0][r] = lp;
    }
  }

  unsigned long long t_2 = stamp ? clock64() : 0;
  // ---- reward nets forward: base r, potential Phi(s'), Phi(s)
  mlp_forward(a.base, Bh, p.ldr, Wf[1], (lfl*)&fl[1][0], 1);
  mlp_forward(a.pot, Qh, p.ldr, Wf[2], (lfl*)&fl[2][0], 1);
  mlp_forward(a.pot, Rh, p.ldr, Wf[2], (lfl*)&fl[3][0], 1);
  __syncthreads();

  unsigned long long t_3 = stamp ? clock64() : 0;
  // ---- logit, BCE gradient, statistics (one row per thread of wave 0)
  float st[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (tid < kRows) {
    const int r = tid, gr = row0 + r;
    float g_b = 0.f, g_p1 = 0.f, g_p2 = 0.f;
    if (gr < n) {
      const float d = a.Done[gr];
      const float h = fl[1][r] + a.gamma * (1.f - d) * fl[2][r] - fl[3][r] - fl[0][r];
      const float y = gr < a.mb ? 1.f : 0.f;
      const float sg = 1.f / (1.f + expf(-h));
      const float sp = fmaxf(h, 0.f) + log1pf(expf(-fabsf(h)));  // softplus(z)
      const float dl = (sg - y) * a.scale;
      g_b = dl;
      g_p1 = a.gamma * (1.f - d) * dl;
      g_p2 = -dl;
      const bool gen_pred = h < 0.f, gen_true = y == 0.f, correct = gen_pred == gen_true;
      st[0] = sp - h * y;
      st[1] = correct ? 1.f : 0.f;
      st[2] = gen_pred ? 1.f : 0.f;
      st[3] = (!gen_true && correct) ? 1.f : 0.f;
      st[4] = (gen_true && correct) ? 1.f : 0.f;
      st[5] = sp - h * sg;
    }
    fl[4][r] = g_b;
    fl[5][r] = g_p1;
    fl[1][r] = g_p2;  // (r is no longer needed)
  }
  if (w == 0) {
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      float v = st[q];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) st_w[0][q] = v;
    }
  }
  __syncthreads();
  if (tid < kDiscStats) a.stats_slab[((size_t)k * gridDim.x + blockIdx.x) * kDiscStats + tid] = tid < 6 ? st_w[0][tid] : 0.f;

  unsigned long long t_4 = stamp ? clock64() : 0;
  // ---- backward: base, potential on s' (writes), potential on s (adds)
  float* slab_row = a.slab + ((size_t)k * gridDim.x + blockIdx.x) * a.n_params;
  mlp_backward(a.base, Bh, p.ldr, Wt[1], (const lfl*)&fl[4][0], HT, p.ld_ht, dZ, dZT, dbs, p.dmax_pad, slab_row, false);
  mlp_backward(a.pot, Qh, p.ldr, Wt[2], (const lfl*)&fl[5][0], HT, p.ld_ht, dZ, dZT, dbs, p.dmax_pad, slab_row, false);
  unsigned long long t_5 = stamp ? clock64() : 0;
  mlp_backward(a.pot, Rh, p.ldr, Wt[2], (const lfl*)&fl[1][0], HT, p.ld_ht, dZ, dZT, dbs, p.dmax_pad, slab_row, true);
  if (stamp) {
    const unsigned long long t_6 = clock64();
    a.prof[0] += t_1 - t_0;  // zero + stage
    a.prof[1] += t_2 - t_1;  // policy fwd + log pi
    a.prof[2] += t_3 - t_2;  // reward fwds
    a.prof[3] += t_4 - t_3;  // loss
    a.prof[4] += t_5 - t_4;  // base bwd + pot(s') bwd
    a.prof[5] += t_6 - t_5;  // pot(s) bwd
    a.prof[6] += 1;
  }
}

}  // namespace

int airl_gather_blocks(int mb) { return (2 * mb + kGatherRows - 1) / kGatherRows; }
int airl_fwd_blocks(int mb) { return (2 * mb + kRows - 1) / kRows; }

bool airl_plan(const AirlDiscArgs& a, AirlPlan& p) {
  p = AirlPlan{};
  const AirlNet* nets[3] = {&a.pol, &a.base, &a.pot};
  int rmax = 0, pmax = 0;
  for (int q = 0; q < 3; ++q) {
    const AirlNet& n = *nets[q];
    if (n.n_layers < 1 || n.n_layers > kAirlMaxLayers) return false;
    for (int l = 0; l <= n.n_layers; ++l) {
      if (n.dims[l] <= 0 || n.dims[l] > 64) return false;
      if (q == 0) pmax = pmax > n.dims[l] ? pmax : n.dims[l];
      else rmax = rmax > n.dims[l] ? rmax : n.dims[l];
    }
  }
  if (a.base.dims[a.base.n_layers] != 1 || a.pot.dims[a.pot.n_layers] != 1) return false;
  if (a.pol.dims[a.pol.n_layers] != a.A || a.A > 16) return false;
  if (a.din_b + 2 * a.D > 128) return false;
  p.ldp = ld_for_k(pmax);
  p.ldr = ld_for_k(rmax);
  p.ld_ht = ld_for_k(kRows);
  p.dmax_pad = pad32(rmax);
  const int wmax = pmax > rmax ? pmax : rmax;
  p.pimg_bytes = kRows * p.ldp * 2;
  p.rimg_bytes = kRows * p.ldr * 2;
  p.ht_bytes = pad32(rmax) * p.ld_ht * 2;
  if (p.ht_bytes < kRows * 32 * 2) p.ht_bytes = kRows * 32 * 2;
  (void)wmax;
  int off = 0;
  for (int q = 0; q < 3; ++q)
    for (int l = 0; l < kAirlMaxLayers; ++l) {
      p.wf_off[q][l] = p.wt_off[q][l] = 0;
      if (l >= nets[q]->n_layers) continue;
      const int din = nets[q]->dims[l], dout = nets[q]->dims[l + 1];
      p.wf_off[q][l] = off;
      off += (pad32(dout) * ld_for_k(din) * 2 + 15) & ~15;
      if (q > 0 && l > 0) {
        p.wt_off[q][l] = off;
        off += (pad32(din) * ld_for_k(dout) * 2 + 15) & ~15;
      }
    }
  p.rimg_off = off;
  off += (a.base.n_layers + 2 * a.pot.n_layers) * p.rimg_bytes;
  p.scratch_off = off;
  const int pol_scratch = 2 * p.pimg_bytes;
  const int bwd_scratch = 3 * p.ht_bytes + 2 * p.rimg_bytes + (2 * kNW * p.dmax_pad + 16) * 4;
  // dZT images are [k][row] with k < 32 here (pad32(dout) of the backward operand <= pad32(rmax))
  off += ((pol_scratch > bwd_scratch ? pol_scratch : bwd_scratch) + 15) & ~15;
  p.lds_bytes = off;
  return p.lds_bytes <= 144 * 1024;
}

hipError_t airl_gather(const AirlDiscArgs& a, int k, hipStream_t s) {
  hipLaunchKernelGGL(airl_gather_kernel, dim3(airl_gather_blocks(a.mb)), dim3(256), 0, s, a, k);
  return hipGetLastError();
}

hipError_t airl_norm(const AirlDiscArgs& a, int mode, int n_total, hipStream_t s) {
  hipLaunchKernelGGL(airl_norm_kernel, dim3(1), dim3(128 * kNormPhases), 0, s, a, mode, n_total);
  return hipGetLastError();
}

hipError_t airl_q_merge(const AirlDiscArgs& a, int count, long long stride, int n, hipStream_t s) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(airl_q_merge_kernel, dim3(1), dim3(128), 0, s, a, count, stride, n);
  return hipGetLastError();
}

hipError_t airl_fwd_bwd(const AirlDiscArgs& a, const AirlPlan& p, int k, hipStream_t s) {
  hipLaunchKernelGGL(airl_fwd_bwd_kernel, dim3(airl_fwd_blocks(a.mb)), dim3(64 * kNW), p.lds_bytes, s, a, p, k);
  return hipGetLastError();
}

}  // namespace ia

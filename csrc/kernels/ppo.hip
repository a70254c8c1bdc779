// PPO update on one persistent workgroup (SB3 PPO.train semantics).
//
// mode 0 runs ALL epochs x minibatches of one PPO.train() call inside ONE launch:
// parameters and gradients live in LDS for the whole update (a 32-wide actor-critic
// is ~3.5K params), the Adam moments in global memory (L2-resident), and every
// minibatch does
//   gather rows -> RunningNorm train-mode update (Chan merge) -> normalise ->
//   actor fwd -> Gaussian/categorical log-prob, ratio, clipped surrogate, entropy ->
//   actor bwd -> critic fwd -> value MSE -> critic bwd -> global-norm clip -> Adam
// with the GEMM-shaped pieces on v_mfma_f32_16x16x4_f32 (exact fp32 numerics, same
// as the fp32 reference; these tiles are latency-bound, not FLOP-bound).
// Data parallel (mode 1/2): mode 1 computes one minibatch's gradients into the flat
// grad vector (after the host all-reduced the normaliser moments), the host
// all-reduces the flat gradient with RCCL, mode 2 applies clip + Adam.
#include <hip/hip_runtime.h>

#include "ia/engine.h"
#include "ia/mfma.h"
#include "launchers.h"

namespace ia {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = 4;
constexpr int kMaxB = 128;

__device__ __forceinline__ int p16(int x) { return (x + 15) & ~15; }
__device__ __forceinline__ int ldp(int x) { return p16(x) + 2; }  // ≡ 2 mod 16 -> conflict-light fp32 MFMA reads

// C[16x16] += A(i,k) * B(k,j), K multiple of 4.
__device__ __forceinline__ f32x4 mm_tile(const float* A, int a_si, int a_sk, const float* B, int b_sk, int b_sj, int K,
                                         f32x4 acc) {
  const int l = threadIdx.x & 63;
  const int i = l & 15, kk = l >> 4;
  const float* ap = A + i * a_si + kk * a_sk;
  const float* bp = B + i * b_sj + kk * b_sk;
  for (int k = 0; k < K; k += 4) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ap[k * a_sk], bp[k * b_sk], acc, 0, 0, 0);
  }
  return acc;
}

struct Net {
  int L;
  int dims[kWaveMaxLayers + 1];
  float* W[kWaveMaxLayers];  // LDS images [p16(dout)][ldp(din)]
  float* b[kWaveMaxLayers];  // [p16(dout)]
  float* gW[kWaveMaxLayers];
  float* gb[kWaveMaxLayers];
  int w_off[kWaveMaxLayers], b_off[kWaveMaxLayers];  // flat offsets
};

struct Smem {
  Net pi, vf;
  float* X;        // [B][ldx] normalised input
  float* H[kWaveMaxLayers + 1];  // activations (H[0] aliases X)
  float* dZ[2];
  float* raw_obs;  // [B][D]
  float* acts;     // [B][A]
  float* rowv;     // per-row scratch: [5][B]: old_logp, adv, ret, g(dlogp), V
  float* red;      // reductions [64]
  float* log_std;  // [16]
  float* g_log_std;
  float* nmean;    // [64] normaliser
  float* nvar;
  float* ncount;
};

__device__ float* carve_net(Net& n, const int* dims, int L, float* p) {
  n.L = L;
  for (int l = 0; l <= L; ++l) n.dims[l] = dims[l];
  for (int l = 0; l < L; ++l) {
    const int sz = p16(dims[l + 1]) * ldp(dims[l]);
    n.W[l] = p;
    p += sz;
    n.b[l] = p;
    p += p16(dims[l + 1]);
    n.gW[l] = p;
    p += sz;
    n.gb[l] = p;
    p += p16(dims[l + 1]);
  }
  return p;
}

__device__ int net_floats(const int* dims, int L) {
  int f = 0;
  for (int l = 0; l < L; ++l) f += 2 * (p16(dims[l + 1]) * ldp(dims[l]) + p16(dims[l + 1]));
  return f;
}

__device__ void net_load(Net& n, const float* params) {
  for (int l = 0; l < n.L; ++l) {
    const int din = n.dims[l], dout = n.dims[l + 1], ld = ldp(din);
    const int R = p16(dout);
    for (int e = threadIdx.x; e < R * ld; e += kThreads) {
      const int o = e / ld, i = e - o * ld;
      n.W[l][e] = (o < dout && i < din) ? params[n.w_off[l] + o * din + i] : 0.f;
      n.gW[l][e] = 0.f;
    }
    for (int o = threadIdx.x; o < R; o += kThreads) {
      n.b[l][o] = o < dout ? params[n.b_off[l] + o] : 0.f;
      n.gb[l][o] = 0.f;
    }
  }
}

__device__ void net_store(const Net& n, float* params) {
  for (int l = 0; l < n.L; ++l) {
    const int din = n.dims[l], dout = n.dims[l + 1], ld = ldp(din);
    for (int e = threadIdx.x; e < dout * din; e += kThreads) {
      const int o = e / din, i = e - o * din;
      params[n.w_off[l] + e] = n.W[l][o * ld + i];
    }
    for (int o = threadIdx.x; o < dout; o += kThreads) params[n.b_off[l] + o] = n.b[l][o];
  }
}

__device__ void net_store_grads(const Net& n, float* grads) {
  for (int l = 0; l < n.L; ++l) {
    const int din = n.dims[l], dout = n.dims[l + 1], ld = ldp(din);
    for (int e = threadIdx.x; e < dout * din; e += kThreads) {
      const int o = e / din, i = e - o * din;
      grads[n.w_off[l] + e] = n.gW[l][o * ld + i];
    }
    for (int o = threadIdx.x; o < dout; o += kThreads) grads[n.b_off[l] + o] = n.gb[l][o];
  }
}

__device__ void net_load_grads(Net& n, const float* grads) {
  for (int l = 0; l < n.L; ++l) {
    const int din = n.dims[l], dout = n.dims[l + 1], ld = ldp(din);
    for (int e = threadIdx.x; e < dout * din; e += kThreads) {
      const int o = e / din, i = e - o * din;
      n.gW[l][o * ld + i] = grads[n.w_off[l] + e];
    }
    for (int o = threadIdx.x; o < dout; o += kThreads) n.gb[l][o] = grads[n.b_off[l] + o];
  }
}

// Forward of the whole net over B rows. Layer inputs kept in H[l] (H[0] = X), output in H[L].
__device__ void net_forward(const Net& n, float** H, int B, int hidden_act) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int l = 0; l < n.L; ++l) {
    const int din = n.dims[l], dout = n.dims[l + 1];
    const int ldi = ldp(din), ldo = ldp(dout), ldw = ldp(din);
    const int mt = B / 16, ntl = p16(dout) / 16;
    const int act = l == n.L - 1 ? ACT_IDENTITY : hidden_act;
    const int K = (din + 3) & ~3;
    for (int t = w; t < mt * ntl; t += kWaves) {
      const int tm = t / ntl, tn = t - tm * ntl;
      f32x4 acc = zero4();
      acc = mm_tile(H[l] + tm * 16 * ldi, ldi, 1, n.W[l] + tn * 16 * ldw, 1, ldw, K, acc);
      const int col = tn * 16 + (lane & 15);
      const float bv = n.b[l][col];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = tm * 16 + (lane >> 4) * 4 + i;
        H[l + 1][r * ldo + col] = col < dout ? apply_act(act, acc[i] + bv) : 0.f;
      }
    }
    __syncthreads();
  }
}

// Backward: dZ of the output layer in dZbuf[0] ([B][ldp(dout_L)]); accumulates gW/gb.
__device__ void net_backward(Net& n, float** H, float** dZ, int B, int hidden_act) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int z = 0;
  for (int l = n.L - 1; l >= 0; --l) {
    const int din = n.dims[l], dout = n.dims[l + 1];
    const int ldi = ldp(din), ldo = ldp(dout), ldw = ldp(din);
    const float* dz = dZ[z];
    // dW[o][i] = sum_r dz[r][o] * H[r][i]
    const int mt = p16(dout) / 16, ntl = p16(din) / 16;
    for (int t = w; t < mt * ntl; t += kWaves) {
      const int tm = t / ntl, tn = t - tm * ntl;
      f32x4 acc = zero4();
      acc = mm_tile(dz + tm * 16, 1, ldo, H[l] + tn * 16, ldi, 1, B, acc);
      const int i = tn * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int o = tm * 16 + (lane >> 4) * 4 + q;
        n.gW[l][o * ldw + i] += (o < dout && i < din) ? acc[q] : 0.f;
      }
    }
    // db[o] = sum_r dz[r][o]
    for (int o = threadIdx.x; o < dout; o += kThreads) {
      float s = 0.f;
      for (int r = 0; r < B; ++r) s += dz[r * ldo + o];
      n.gb[l][o] += s;
    }
    if (l > 0) {
      // G[r][i] = sum_o dz[r][o] W[o][i];  dz_{l-1} = G * act'(H_l)
      float* dzo = dZ[z ^ 1];
      const int mt2 = B / 16, nt2 = p16(din) / 16;
      const int K = (dout + 3) & ~3;
      for (int t = w; t < mt2 * nt2; t += kWaves) {
        const int tm = t / nt2, tn = t - tm * nt2;
        f32x4 acc = zero4();
        acc = mm_tile(dz + tm * 16 * ldo, ldo, 1, n.W[l] + tn * 16, ldw, 1, K, acc);
        const int col = tn * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = tm * 16 + (lane >> 4) * 4 + q;
          const float h = H[l][r * ldi + col];
          dzo[r * ldi + col] = col < din ? acc[q] * act_grad_from_out(hidden_act, h) : 0.f;
        }
      }
    }
    __syncthreads();
    z ^= 1;
  }
}

__device__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < kWaves; ++i) s += red[i];
  __syncthreads();
  return s;
}

struct Layout {
  int B, D, A;
};

// gather + normalise + advantages; returns nothing (fills smem)
__device__ void load_minibatch(const PPOArgs& a, Smem& s, const int* idx, bool update_norm) {
  const int B = a.batch, D = a.D;
  const int Aact = a.discrete ? 1 : a.A;
  const int ldx = ldp(D);
  for (int e = threadIdx.x; e < B * D; e += kThreads) {
    const int r = e / D, c = e - r * D;
    s.raw_obs[e] = a.obs[(size_t)idx[r] * D + c];
  }
  for (int e = threadIdx.x; e < B * Aact; e += kThreads) {
    const int r = e / Aact, c = e - r * Aact;
    s.acts[e] = a.acts[(size_t)idx[r] * Aact + c];
  }
  for (int r = threadIdx.x; r < B; r += kThreads) {
    s.rowv[0 * kMaxB + r] = a.old_logp[idx[r]];
    s.rowv[1 * kMaxB + r] = a.adv[idx[r]];
    s.rowv[2 * kMaxB + r] = a.returns[idx[r]];
  }
  __syncthreads();
  if (a.has_norm && update_norm) {
    // RunningNorm.update_stats (Chan et al.) with this minibatch (biased batch var)
    for (int c = threadIdx.x; c < D; c += kThreads) {
      float m = 0.f;
      for (int r = 0; r < B; ++r) m += s.raw_obs[r * D + c];
      m /= (float)B;
      float v = 0.f;
      for (int r = 0; r < B; ++r) {
        const float d = s.raw_obs[r * D + c] - m;
        v += d * d;
      }
      v /= (float)B;
      const float cnt = s.ncount[0];
      const float tot = cnt + (float)B;
      const float delta = m - s.nmean[c];
      s.nmean[c] += delta * (float)B / tot;
      float rv = s.nvar[c] * cnt + v * (float)B + delta * delta * cnt * (float)B / tot;
      s.nvar[c] = rv / tot;
    }
    __syncthreads();
    if (threadIdx.x == 0) s.ncount[0] += (float)B;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < B * ldx; e += kThreads) {
    const int r = e / ldx, c = e - r * ldx;
    float v = 0.f;
    if (c < D) {
      v = s.raw_obs[r * D + c];
      if (a.has_norm) v = (v - s.nmean[c]) * rsqrtf(s.nvar[c] + a.norm_eps);
    }
    s.X[e] = v;
  }
  // advantage normalisation: (adv - mean) / (std_unbiased + 1e-8)
  if (a.normalize_advantage && B > 1) {
    float v = threadIdx.x < B ? s.rowv[1 * kMaxB + threadIdx.x] : 0.f;
    const float mean = block_sum(v, s.red) / (float)B;
    const float d = threadIdx.x < B ? v - mean : 0.f;
    const float var = block_sum(d * d, s.red) / (float)(B - 1);
    const float inv = 1.f / (sqrtf(var) + 1e-8f);
    if (threadIdx.x < B) s.rowv[1 * kMaxB + threadIdx.x] = d * inv;
  }
  __syncthreads();
}

// Policy head -> per-row dlogp (rowv[3]) and dZ of the head; accumulates log_std grads and stats.
__device__ void policy_loss(const PPOArgs& a, Smem& s, float** H, float** dZ) {
  const int B = a.batch;
  const int L = s.pi.L;
  const int dout = s.pi.dims[L];
  const int ldo = ldp(dout);
  const float* head = H[L];
  const float invB = 1.f / (float)B;
  const float half_log2pi = 0.91893853320467274f;
  float pg = 0.f, clipf = 0.f, kl = 0.f;
  const int r = threadIdx.x;
  // per-row log prob and ratio (one thread per row)
  float dlogp = 0.f;
  if (r < B) {
    float logp = 0.f;
    if (a.discrete) {
      float mx = -INFINITY;
      for (int k = 0; k < dout; ++k) mx = fmaxf(mx, head[r * ldo + k]);
      float z = 0.f;
      for (int k = 0; k < dout; ++k) z += expf(head[r * ldo + k] - mx);
      const int act = (int)s.acts[r];
      logp = head[r * ldo + act] - mx - logf(z);
    } else {
      for (int k = 0; k < a.A; ++k) {
        const float ls = s.log_std[k];
        const float zz = (s.acts[r * a.A + k] - head[r * ldo + k]) * expf(-ls);
        logp += -0.5f * zz * zz - ls - half_log2pi;
      }
    }
    const float adv = s.rowv[1 * kMaxB + r];
    const float lr_ = logp - s.rowv[0 * kMaxB + r];
    const float ratio = expf(lr_);
    const float lo = 1.f - a.clip_range, hi = 1.f + a.clip_range;
    const float rc = fminf(fmaxf(ratio, lo), hi);
    const float pl1 = adv * ratio, pl2 = adv * rc;
    float c1, c2;  // torch.min tie-splitting
    if (pl1 < pl2) { c1 = 1.f; c2 = 0.f; } else if (pl2 < pl1) { c1 = 0.f; c2 = 1.f; } else { c1 = 0.5f; c2 = 0.5f; }
    const float inside = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
    const float dratio = -invB * (c1 * adv + c2 * adv * inside);
    dlogp = dratio * ratio;
    pg = -fminf(pl1, pl2);
    clipf = fabsf(ratio - 1.f) > a.clip_range ? 1.f : 0.f;
    kl = (ratio - 1.f) - lr_;
  }
  // head gradient
  float* dz = dZ[0];
  if (r < B) {
    if (a.discrete) {
      float mx = -INFINITY;
      for (int k = 0; k < dout; ++k) mx = fmaxf(mx, head[r * ldo + k]);
      float z = 0.f;
      for (int k = 0; k < dout; ++k) z += expf(head[r * ldo + k] - mx);
      const int act = (int)s.acts[r];
      // entropy: H = -sum p log p ; dH/dlogit_k = -p_k (log p_k + H)
      float ent = 0.f;
      for (int k = 0; k < dout; ++k) {
        const float lp = head[r * ldo + k] - mx - logf(z);
        ent -= expf(lp) * lp;
      }
      for (int k = 0; k < ldo; ++k) {
        float g = 0.f;
        if (k < dout) {
          const float lp = head[r * ldo + k] - mx - logf(z);
          const float pk = expf(lp);
          g = dlogp * ((k == act ? 1.f : 0.f) - pk);
          // entropy loss = -ent_coef * mean(H)
          g += -a.ent_coef * invB * (-pk * (lp + ent));
        }
        dz[r * ldo + k] = g;
      }
      s.rowv[4 * kMaxB + r] = ent;
    } else {
      for (int k = 0; k < ldo; ++k) {
        float g = 0.f;
        if (k < a.A) {
          const float ls = s.log_std[k];
          const float zz = (s.acts[r * a.A + k] - head[r * ldo + k]) * expf(-ls);
          g = dlogp * zz * expf(-ls);
        }
        dz[r * ldo + k] = g;
      }
    }
    s.rowv[3 * kMaxB + r] = dlogp;
  }
  __syncthreads();
  // log_std gradient: sum_r dlogp_r (z^2 - 1)  - ent_coef (entropy = sum log_std + const)
  float ent_loss;
  if (!a.discrete) {
    for (int k = threadIdx.x; k < a.A; k += kThreads) {
      const float ls = s.log_std[k];
      float g = 0.f;
      for (int rr = 0; rr < B; ++rr) {
        const float zz = (s.acts[rr * a.A + k] - head[rr * ldo + k]) * expf(-ls);
        g += s.rowv[3 * kMaxB + rr] * (zz * zz - 1.f);
      }
      s.g_log_std[k] += g - a.ent_coef;
    }
    float sl = 0.f;
    for (int k = 0; k < a.A; ++k) sl += s.log_std[k];
    ent_loss = -(sl + a.A * (0.5f + half_log2pi));
  } else {
    const float e = r < B ? s.rowv[4 * kMaxB + r] : 0.f;
    ent_loss = -block_sum(e, s.red) * invB;
  }
  const float pg_s = block_sum(pg, s.red) * invB;
  const float cf_s = block_sum(clipf, s.red) * invB;
  const float kl_s = block_sum(kl, s.red) * invB;
  if (threadIdx.x == 0) {
    a.stats[0] += ent_loss;
    a.stats[1] += pg_s;
    a.stats[3] += cf_s;
    a.stats[4] += kl_s;
  }
}

__device__ void value_loss(const PPOArgs& a, Smem& s, float** H, float** dZ) {
  const int B = a.batch;
  const int L = s.vf.L;
  const float* v = H[L];
  const int ldo = ldp(1);
  const int r = threadIdx.x;
  float sq = 0.f;
  if (r < B) {
    const float d = v[r * ldo] - s.rowv[2 * kMaxB + r];
    sq = d * d;
    for (int k = 0; k < ldo; ++k) dZ[0][r * ldo + k] = k == 0 ? a.vf_coef * 2.f * d / (float)B : 0.f;
  }
  __syncthreads();
  const float vl = block_sum(sq, s.red) / (float)B;
  if (threadIdx.x == 0) a.stats[2] += vl;
}

__device__ void zero_grads(Smem& s, const PPOArgs& a) {
  Net* nets[2] = {&s.pi, &s.vf};
  for (int q = 0; q < 2; ++q) {
    Net& n = *nets[q];
    for (int l = 0; l < n.L; ++l) {
      const int sz = p16(n.dims[l + 1]) * ldp(n.dims[l]);
      for (int e = threadIdx.x; e < sz; e += kThreads) n.gW[l][e] = 0.f;
      for (int e = threadIdx.x; e < p16(n.dims[l + 1]); e += kThreads) n.gb[l][e] = 0.f;
    }
  }
  for (int k = threadIdx.x; k < 16; k += kThreads) s.g_log_std[k] = 0.f;
  __syncthreads();
}

// clip_grad_norm_(max_norm) + torch Adam on every parameter (LDS images, moments in global)
__device__ void clip_and_adam(const PPOArgs& a, Smem& s, float step) {
  Net* nets[2] = {&s.pi, &s.vf};
  float ss = 0.f;
  for (int q = 0; q < 2; ++q) {
    Net& n = *nets[q];
    for (int l = 0; l < n.L; ++l) {
      const int sz = p16(n.dims[l + 1]) * ldp(n.dims[l]);
      for (int e = threadIdx.x; e < sz; e += kThreads) ss += n.gW[l][e] * n.gW[l][e];
      for (int e = threadIdx.x; e < n.dims[l + 1]; e += kThreads) ss += n.gb[l][e] * n.gb[l][e];
    }
  }
  if (!a.discrete && a.log_std_off >= 0)
    for (int k = threadIdx.x; k < a.A; k += kThreads) ss += s.g_log_std[k] * s.g_log_std[k];
  const float norm = sqrtf(block_sum(ss, s.red));
  const float coef = fminf(1.f, a.max_grad_norm / (norm + 1e-6f));
  const float bc1 = 1.f - powf(a.beta1, step);
  const float bc2 = 1.f - powf(a.beta2, step);
  const float step_size = a.lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (int q = 0; q < 2; ++q) {
    Net& n = *nets[q];
    for (int l = 0; l < n.L; ++l) {
      const int din = n.dims[l], dout = n.dims[l + 1], ld = ldp(din);
      for (int e = threadIdx.x; e < dout * din; e += kThreads) {
        const int o = e / din, i = e - o * din;
        const int gi = n.w_off[l] + e;
        const float g = n.gW[l][o * ld + i] * coef;
        const float m = a.beta1 * a.exp_avg[gi] + (1.f - a.beta1) * g;
        const float v = a.beta2 * a.exp_avg_sq[gi] + (1.f - a.beta2) * g * g;
        a.exp_avg[gi] = m;
        a.exp_avg_sq[gi] = v;
        n.W[l][o * ld + i] -= step_size * m / (sqrtf(v) / bc2s + a.adam_eps);
      }
      for (int o = threadIdx.x; o < dout; o += kThreads) {
        const int gi = n.b_off[l] + o;
        const float g = n.gb[l][o] * coef;
        const float m = a.beta1 * a.exp_avg[gi] + (1.f - a.beta1) * g;
        const float v = a.beta2 * a.exp_avg_sq[gi] + (1.f - a.beta2) * g * g;
        a.exp_avg[gi] = m;
        a.exp_avg_sq[gi] = v;
        n.b[l][o] -= step_size * m / (sqrtf(v) / bc2s + a.adam_eps);
      }
    }
  }
  if (!a.discrete && a.log_std_off >= 0) {
    for (int k = threadIdx.x; k < a.A; k += kThreads) {
      const int gi = a.log_std_off + k;
      const float g = s.g_log_std[k] * coef;
      const float m = a.beta1 * a.exp_avg[gi] + (1.f - a.beta1) * g;
      const float v = a.beta2 * a.exp_avg_sq[gi] + (1.f - a.beta2) * g * g;
      a.exp_avg[gi] = m;
      a.exp_avg_sq[gi] = v;
      s.log_std[k] -= step_size * m / (sqrtf(v) / bc2s + a.adam_eps);
    }
  }
  __syncthreads();
}

__device__ void setup(const PPOArgs& a, Smem& s, float* lds) {
  float* p = lds;
  for (int l = 0; l < kWaveMaxLayers; ++l) {
    s.pi.w_off[l] = a.pi_w_off[l];
    s.pi.b_off[l] = a.pi_b_off[l];
    s.vf.w_off[l] = a.vf_w_off[l];
    s.vf.b_off[l] = a.vf_b_off[l];
  }
  p = carve_net(s.pi, a.pi_dims, a.n_pi, p);
  p = carve_net(s.vf, a.vf_dims, a.n_vf, p);
  int maxd = a.D;
  for (int l = 0; l <= a.n_pi; ++l) maxd = max(maxd, a.pi_dims[l]);
  for (int l = 0; l <= a.n_vf; ++l) maxd = max(maxd, a.vf_dims[l]);
  const int img = a.batch * ldp(maxd);
  const int nh = a.n_pi > a.n_vf ? a.n_pi : a.n_vf;
  s.X = p;
  p += img;
  for (int l = 1; l <= kWaveMaxLayers; ++l) {
    s.H[l] = p;
    if (l <= nh) p += img;
  }
  s.H[0] = s.X;
  s.dZ[0] = p;
  p += img;
  s.dZ[1] = p;
  p += img;
  s.raw_obs = p;
  p += kMaxB * a.D;
  s.acts = p;
  p += kMaxB * (a.discrete ? 1 : a.A);
  s.rowv = p;
  p += 5 * kMaxB;
  s.red = p;
  p += 64;
  s.log_std = p;
  p += 16;
  s.g_log_std = p;
  p += 16;
  s.nmean = p;
  p += 64;
  s.nvar = p;
  p += 64;
  s.ncount = p;
  p += 4;
}

__global__ __launch_bounds__(kThreads) void ppo_kernel(PPOArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  __shared__ Smem s;
  if (threadIdx.x == 0) setup(a, s, lds);
  __syncthreads();
  Smem sm = s;  // private copy of the pointer table
  net_load(sm.pi, a.params);
  net_load(sm.vf, a.params);
  for (int k = threadIdx.x; k < 16; k += kThreads) {
    sm.log_std[k] = (a.log_std_off >= 0 && k < a.A && !a.discrete) ? a.params[a.log_std_off + k] : 0.f;
    sm.g_log_std[k] = 0.f;
  }
  if (a.has_norm) {
    for (int c = threadIdx.x; c < a.D; c += kThreads) {
      sm.nmean[c] = a.norm_mean[c];
      sm.nvar[c] = a.norm_var[c];
    }
    if (threadIdx.x == 0) sm.ncount[0] = a.norm_count[0];
  }
  __syncthreads();
  const int n_mb = a.rows / a.batch;
  float step = a.adam_step[0];
  const int first = a.mode == 1 ? a.mb_index : 0;
  const int last = a.mode == 1 ? a.mb_index + 1 : (a.mode == 2 ? 0 : a.n_epochs * n_mb);
  for (int it = first; it < last; ++it) {
    const int e = it / n_mb, mb = it - e * n_mb;
    const int* idx = a.perm + (size_t)e * a.rows + (size_t)mb * a.batch;
    zero_grads(sm, a);
    load_minibatch(a, sm, idx, a.mode == 0);
    // actor
    float* Hp[kWaveMaxLayers + 1];
    for (int l = 0; l <= kWaveMaxLayers; ++l) Hp[l] = sm.H[l];
    net_forward(sm.pi, Hp, a.batch, a.hidden_act);
    policy_loss(a, sm, Hp, sm.dZ);
    __syncthreads();
    net_backward(sm.pi, Hp, sm.dZ, a.batch, a.hidden_act);
    // critic (reuses the activation images)
    net_forward(sm.vf, Hp, a.batch, a.hidden_act);
    value_loss(a, sm, Hp, sm.dZ);
    __syncthreads();
    net_backward(sm.vf, Hp, sm.dZ, a.batch, a.hidden_act);
    if (a.mode == 0) {
      step += 1.f;
      clip_and_adam(a, sm, step);
    }
  }
  if (a.mode == 2) {
    // apply: grads from global (already all-reduced), clip + Adam
    net_load_grads(sm.pi, a.grads);
    net_load_grads(sm.vf, a.grads);
    for (int k = threadIdx.x; k < a.A; k += kThreads)
      if (a.log_std_off >= 0 && !a.discrete) sm.g_log_std[k] = a.grads[a.log_std_off + k];
    __syncthreads();
    step += 1.f;
    clip_and_adam(a, sm, step);
  }
  __syncthreads();
  if (a.mode == 1) {
    net_store_grads(sm.pi, a.grads);
    net_store_grads(sm.vf, a.grads);
    for (int k = threadIdx.x; k < a.A; k += kThreads)
      if (a.log_std_off >= 0 && !a.discrete) a.grads[a.log_std_off + k] = sm.g_log_std[k];
  } else {
    net_store(sm.pi, a.params);
    net_store(sm.vf, a.params);
    for (int k = threadIdx.x; k < a.A; k += kThreads)
      if (a.log_std_off >= 0 && !a.discrete) a.params[a.log_std_off + k] = sm.log_std[k];
    if (threadIdx.x == 0) a.adam_step[0] = step;
  }
  if (a.has_norm && a.mode == 0) {
    for (int c = threadIdx.x; c < a.D; c += kThreads) {
      a.norm_mean[c] = sm.nmean[c];
      a.norm_var[c] = sm.nvar[c];
    }
    if (threadIdx.x == 0) a.norm_count[0] = sm.ncount[0];
  }
}

}  // namespace

size_t ppo_lds_bytes(const PPOArgs& a) {
  auto p16h = [](int x) { return (x + 15) & ~15; };
  auto ldph = [&](int x) { return p16h(x) + 2; };
  int f = 0;
  for (int l = 0; l < a.n_pi; ++l) f += 2 * (p16h(a.pi_dims[l + 1]) * ldph(a.pi_dims[l]) + p16h(a.pi_dims[l + 1]));
  for (int l = 0; l < a.n_vf; ++l) f += 2 * (p16h(a.vf_dims[l + 1]) * ldph(a.vf_dims[l]) + p16h(a.vf_dims[l + 1]));
  int maxd = a.D;
  for (int l = 0; l <= a.n_pi; ++l) maxd = maxd > a.pi_dims[l] ? maxd : a.pi_dims[l];
  for (int l = 0; l <= a.n_vf; ++l) maxd = maxd > a.vf_dims[l] ? maxd : a.vf_dims[l];
  const int nh = a.n_pi > a.n_vf ? a.n_pi : a.n_vf;
  f += (1 + nh + 2) * a.batch * ldph(maxd);
  f += kMaxB * a.D + kMaxB * (a.discrete ? 1 : a.A) + 5 * kMaxB + 64 + 16 + 16 + 64 + 64 + 4;
  return (size_t)f * sizeof(float);
}

hipError_t ppo_launch(const PPOArgs& a, hipStream_t s) {
  if (a.batch % 16 != 0 || a.batch > kMaxB || a.rows % a.batch != 0) return hipErrorInvalidValue;
  const size_t lds = ppo_lds_bytes(a);
  if (lds > 150 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ppo_kernel, dim3(1), dim3(kThreads), lds, s, a);
  return hipGetLastError();
}

}  // namespace ia

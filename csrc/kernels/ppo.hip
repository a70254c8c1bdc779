// PPO update on one persistent workgroup (SB3 PPO.train semantics,
// reference call site: src/imitation/algorithms/adversarial/common.py train_gen ->
// PPO.learn -> PPO.train).
//
// mode 0 runs ALL epochs x minibatches of one PPO.train() call inside ONE launch.
// Everything the update touches lives in LDS for the whole launch: parameters,
// gradients and both Adam moments (padded [16-row][din+2] images) plus the
// minibatch activation images. Each minibatch does
//   rows (prefetched into registers one minibatch ahead) -> RunningNorm train-mode
//   update (Chan merge) -> normalise -> {actor fwd, critic fwd} -> {policy loss,
//   value loss} -> {actor bwd, critic bwd} -> global-norm clip -> Adam
// The actor and the critic are independent until the shared gradient norm, so
// waves 0-3 run the actor while waves 4-7 run the critic, in lock-step stages
// separated by workgroup barriers. Every GEMM-shaped piece runs on
// v_mfma_f32_16x16x4_f32 (exact fp32, the reference is fp32). Bias gradients ride
// in the dW MFMA tiles through a constant-1 column appended to every layer input
// image; backward reuses the forward activation images in place for dZ.
//
// Register/LDS discipline: no per-thread arrays or pointer tables are indexed at run
// time (the previous version kept a struct of LDS pointers indexed by layer, which
// the compiler placed in scratch memory -- every layer access was a global-memory
// round trip). Layer geometry is recomputed from the kernel arguments with
// compile-time layer indices (fully unrolled loops over kWaveMaxLayers).
//
// Data parallel: mode 1 computes one minibatch's gradients into the flat grad
// vector (the host all-reduced the normaliser moments first), the host all-reduces
// the flat gradient with RCCL, mode 2 applies clip + Adam.
#include <hip/hip_runtime.h>

#include "ia/engine.h"
#include "ia/mfma.h"
#include "launchers.h"

namespace ia {
namespace {

constexpr int kThreads = 512;
constexpr int kWaves = kThreads / 64;
constexpr int kGroup = 4;   // waves per net (actor group = waves 0-3, critic = 4-7)
constexpr int kMaxB = 64;   // rows per minibatch (one row per lane in reductions)
constexpr int kPfObs = 8;   // prefetch slots per thread: B*D <= 64*64 = kThreads*8
constexpr int kPfAct = 2;   // B*A <= 64*16
constexpr int kL = kWaveMaxLayers;

// LDS pointers are typed address_space(3): 32-bit, ds_read/ds_write, and cheap to keep live
typedef __attribute__((address_space(3))) float lf;

__host__ __device__ __forceinline__ int p16(int x) { return (x + 15) & ~15; }
__host__ __device__ __forceinline__ int ldp(int x) { return p16(x) + 2; }
__host__ __device__ inline int layer_floats(int din, int dout) { return p16(dout) * ldp(din) + p16(dout); }

// C[16x16] += A(i,k) * B(k,j), K multiple of 4 (runtime). Operands for 8 k-steps are
// issued together so one LDS latency covers 8 MFMAs.
__device__ __forceinline__ f32x4 mm_tile(const lf* A, int a_si, int a_sk, const lf* B, int b_sk, int b_sj, int K,
                                         f32x4 acc) {
  const int l = threadIdx.x & 63;
  const int i = l & 15, kk = l >> 4;
  const lf* ap = A + i * a_si + kk * a_sk;
  const lf* bp = B + i * b_sj + kk * b_sk;
  int k = 0;
  for (; k + 32 <= K; k += 32) {
    float av[8], bv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      av[u] = ap[(k + 4 * u) * a_sk];
      bv[u] = bp[(k + 4 * u) * b_sk];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
  }
  for (; k < K; k += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ap[k * a_sk], bp[k * b_sk], acc, 0, 0, 0);
  return acc;
}

__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------- LDS geometry
// [actor layers][critic layers] each {W,b | gW,gb | mW,mb | vW,vb}, then
// H0 | actor H1..HL | critic H1..HL | dZ actor | dZ critic | raw | acts | rowv | ls | norm | red
struct Lay {
  lf *W, *b, *gW, *gb;
  int din, dout, n, w_off, b_off;
};

template <int Q>
__device__ __forceinline__ const int* dims_of(const PPOArgs& a) { return Q ? a.vf_dims : a.pi_dims; }
template <int Q>
__device__ __forceinline__ int nl_of(const PPOArgs& a) { return Q ? a.n_vf : a.n_pi; }

// floats of all padded parameter images (actor layers then critic layers)
__host__ __device__ inline int param_floats(const PPOArgs& a) {
  int f = 0;
  for (int l = 0; l < kL; ++l) {
    if (l < a.n_pi) f += layer_floats(a.pi_dims[l], a.pi_dims[l + 1]);
    if (l < a.n_vf) f += layer_floats(a.vf_dims[l], a.vf_dims[l + 1]);
  }
  return f;
}

template <int Q>
__device__ __forceinline__ Lay lay(lf* lds, const PPOArgs& a, int li) {
  int off = 0;
  if (Q == 1) {
#pragma unroll
    for (int l = 0; l < kL; ++l)
      if (l < a.n_pi) off += layer_floats(a.pi_dims[l], a.pi_dims[l + 1]);
  }
  const int* d = dims_of<Q>(a);
#pragma unroll
  for (int l = 0; l < kL; ++l)
    if (l < li) off += layer_floats(d[l], d[l + 1]);
  Lay y;
  y.din = d[li];
  y.dout = d[li + 1];
  y.n = layer_floats(y.din, y.dout);
  const int sw = p16(y.dout) * ldp(y.din);
  y.W = lds + off;
  y.b = y.W + sw;
  y.gW = y.W + param_floats(a);  // gradient image region mirrors the parameter region
  y.gb = y.gW + sw;
  y.w_off = Q ? a.vf_w_off[li] : a.pi_w_off[li];
  y.b_off = Q ? a.vf_b_off[li] : a.pi_b_off[li];
  return y;
}


__host__ __device__ inline int max_dim(const PPOArgs& a) {
  int m = a.D;
  for (int l = 0; l <= kL; ++l) {
    if (l <= a.n_pi) m = m > a.pi_dims[l] ? m : a.pi_dims[l];
    if (l <= a.n_vf) m = m > a.vf_dims[l] ? m : a.vf_dims[l];
  }
  return m;
}
// activation image (also holds dZ in place during backward); +16 tail slack for tile over-read
__host__ __device__ inline int img_floats(const PPOArgs& a) { return a.batch * ldp(max_dim(a)) + 16; }
__host__ __device__ inline int head_ld(const PPOArgs& a) {
  const int hp = a.pi_dims[a.n_pi], hv = a.vf_dims[a.n_vf];
  return ldp(hp > hv ? hp : hv);
}
__host__ __device__ inline int dz_floats(const PPOArgs& a) { return a.batch * head_ld(a) + 16; }

struct Bufs {
  lf* H0;
  lf* Ha;  // actor H1 = Ha, H_l = Ha + (l-1)*img
  lf* Hc;
  lf* dZa;
  lf* dZc;
  lf* raw;   // [B][D]
  lf* acts;  // [B][Aw]
  lf* rowv;  // [6][kMaxB]: old_logp, adv, ret, dlogp, ent / value err, pg
  lf* ls;    // log_std [16], grad [16], m [16], v [16]
  lf* norm;  // mean [64], var [64], count
  lf* red;   // [32]: 0-7 wave partials, 8-12 stats accumulators
  int img;
};

__device__ __forceinline__ Bufs bufs(lf* lds, const PPOArgs& a) {
  Bufs b;
  b.img = img_floats(a);
  lf* p = lds + 2 * param_floats(a);  // Wall | Gall
  b.H0 = p; p += b.img;
  b.Ha = p; p += a.n_pi * b.img;
  b.Hc = p; p += a.n_vf * b.img;
  b.dZa = p; p += dz_floats(a);
  b.dZc = p; p += dz_floats(a);
  b.raw = p; p += kMaxB * a.D;
  b.acts = p; p += kMaxB * (a.discrete ? 1 : a.A);
  b.rowv = p; p += 6 * kMaxB;
  b.ls = p; p += 64;
  b.norm = p; p += 132;
  b.red = p; p += 32;
  return b;
}
__host__ __device__ inline int total_floats(const PPOArgs& a) {
  return 2 * param_floats(a) + img_floats(a) * (1 + a.n_pi + a.n_vf) + 2 * dz_floats(a) + kMaxB * a.D +
         kMaxB * (a.discrete ? 1 : a.A) + 6 * kMaxB + 64 + 132 + 32 + 2 * kL * 8;
}

template <int Q>
__device__ __forceinline__ lf* Hq(const Bufs& b, int l) {
  return l == 0 ? b.H0 : (Q ? b.Hc : b.Ha) + (l - 1) * b.img;
}

// flat (torch layout) <-> padded image
__device__ __forceinline__ void img_load(lf* img, lf* bimg, const float* flat, const Lay& y) {
  const int ld = ldp(y.din), R = p16(y.dout);
  for (int e = threadIdx.x; e < R * ld; e += kThreads) {
    const int o = e / ld, i = e - o * ld;
    img[e] = (o < y.dout && i < y.din) ? flat[y.w_off + o * y.din + i] : 0.f;
  }
  for (int o = threadIdx.x; o < R; o += kThreads) bimg[o] = o < y.dout ? flat[y.b_off + o] : 0.f;
}
__device__ __forceinline__ void img_zero(lf* img, int n) {
  for (int e = threadIdx.x; e < n; e += kThreads) img[e] = 0.f;
}
__device__ __forceinline__ void img_store(const lf* img, const lf* bimg, float* flat, const Lay& y) {
  const int ld = ldp(y.din);
  for (int e = threadIdx.x; e < y.dout * y.din; e += kThreads) {
    const int o = e / y.din, i = e - o * y.din;
    flat[y.w_off + e] = img[o * ld + i];
  }
  for (int o = threadIdx.x; o < y.dout; o += kThreads) flat[y.b_off + o] = bimg[o];
}

// ---------------------------------------------------------------- per-net stages
// Layer table in LDS, built once per launch: one 8-int record per (net, layer).
// Stages read their record at a wave-uniform address and readfirstlane it into
// SGPRs, so one copy of each stage body serves every layer of both nets (no
// per-layer inlined copies whose hoisted invariants spill registers).
typedef __attribute__((address_space(3))) int li32;
enum { LT_OFF = 0, LT_DIN, LT_DOUT, LT_ACT, LT_HIN, LT_HOUT, LT_DZIN, LT_N };
struct LT {
  int off, din, dout, act, hin, hout, dzin, n;
};
__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ LT load_lt(const li32* tab, int e) {
  const li32* r = tab + e * 8;
  LT t;
  t.off = rfl(r[LT_OFF]);
  t.din = rfl(r[LT_DIN]);
  t.dout = rfl(r[LT_DOUT]);
  t.act = rfl(r[LT_ACT]);
  t.hin = rfl(r[LT_HIN]);
  t.hout = rfl(r[LT_HOUT]);
  t.dzin = rfl(r[LT_DZIN]);
  t.n = rfl(r[LT_N]);
  return t;
}

template <int Q>
__device__ __forceinline__ void write_lt(li32* tab, lf* lds, const PPOArgs& a, const Bufs& bf) {
  const int L = nl_of<Q>(a);
#pragma unroll
  for (int li = 0; li < kL; ++li) {
    if (li < L) {
      const Lay y = lay<Q>(lds, a, li);
      li32* r = tab + (Q * kL + li) * 8;
      r[LT_OFF] = (int)(y.W - lds);
      r[LT_DIN] = y.din;
      r[LT_DOUT] = y.dout;
      r[LT_ACT] = li == L - 1 ? ACT_IDENTITY : a.hidden_act;
      r[LT_HIN] = (int)(Hq<Q>(bf, li) - lds);
      r[LT_HOUT] = (int)(Hq<Q>(bf, li + 1) - lds);
      r[LT_DZIN] = (int)((li == L - 1 ? (Q ? bf.dZc : bf.dZa) : Hq<Q>(bf, li + 2)) - lds);
      r[LT_N] = param_floats(a);
    }
  }
}

// gw: wave index within the net's group (0..3).
__device__ __forceinline__ void fwd_stage(lf* lds, const LT& t, int B, int gw) {
  const int lane = threadIdx.x & 63;
  const lf* W = lds + t.off;
  const lf* bias = W + p16(t.dout) * ldp(t.din);
  const lf* Hin = lds + t.hin;
  lf* Hout = lds + t.hout;
  const int ldi = ldp(t.din), ldo = ldp(t.dout);
  const int mt = B / 16, ntl = p16(t.dout) / 16;
  const int K = (t.din + 3) & ~3;
  for (int tt = gw; tt < mt * ntl; tt += kGroup) {
    const int tm = tt / ntl, tn = tt - tm * ntl;
    f32x4 acc = mm_tile(Hin + tm * 16 * ldi, ldi, 1, W + tn * 16 * ldi, 1, ldi, K, zero4());
    const int col = tn * 16 + (lane & 15);
    const float bv = bias[col];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = tm * 16 + (lane >> 4) * 4 + q;
      Hout[r * ldo + col] = col < t.dout ? apply_act(t.act, acc[q] + bv) : (col == t.dout ? 1.f : 0.f);
    }
  }
  if (t.dout % 16 == 0)  // ones column outside the written tiles
    for (int r = gw * 64 + lane; r < B; r += kGroup * 64) Hout[r * ldo + t.dout] = 1.f;
}

// Backward stage of one layer: dW (+ bias grad via the ones column) and, if
// `lower`, dZ of the layer below. dZ of this layer lives in the head dZ image or in
// place in H[li+2]; dZ of the layer below is written in place into H[li+1] (free:
// its last reader was the previous backward stage).
__device__ __forceinline__ void bwd_stage(lf* lds, const LT& t, int B, int gw, bool lower, int hidden_act) {
  const int lane = threadIdx.x & 63;
  const lf* W = lds + t.off;
  const int sw = p16(t.dout) * ldp(t.din);
  lf* gW = lds + t.off + t.n;  // t.n = size of the parameter region
  lf* gb = gW + sw;
  const int ldi = ldp(t.din), ldo = ldp(t.dout);
  const lf* dz = lds + t.dzin;
  const lf* Hin = lds + t.hin;
  {
    const int mt = p16(t.dout) / 16, ntl = p16(t.din + 1) / 16;
    for (int tt = gw; tt < mt * ntl; tt += kGroup) {
      const int tm = tt / ntl, tn = tt - tm * ntl;
      f32x4 acc = mm_tile(dz + tm * 16, 1, ldo, Hin + tn * 16, ldi, 1, B, zero4());
      const int i = tn * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int o = tm * 16 + (lane >> 4) * 4 + q;
        if (o < t.dout) {
          if (i < t.din) gW[o * ldi + i] = acc[q];
          else if (i == t.din) gb[o] = acc[q];
        }
      }
    }
  }
  if (lower) {
    lf* dzo = lds + t.hout;  // H[li+1]
    const int mt2 = B / 16, nt2 = p16(t.din) / 16;
    const int K = (t.dout + 3) & ~3;
    for (int tt = gw; tt < mt2 * nt2; tt += kGroup) {
      const int tm = tt / nt2, tn = tt - tm * nt2;
      f32x4 acc = mm_tile(dz + tm * 16 * ldo, ldo, 1, W + tn * 16, ldi, 1, K, zero4());
      const int col = tn * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = tm * 16 + (lane >> 4) * 4 + q;
        dzo[r * ldi + col] = col < t.din ? acc[q] * act_grad_from_out(hidden_act, Hin[r * ldi + col]) : 0.f;
      }
    }
  }
}

// ---------------------------------------------------------------- minibatch rows
struct Prefetch {
  float ob[kPfObs];
  float ac[kPfAct];
  float lp, adv, ret;
};

__device__ __forceinline__ void prefetch_rows(const PPOArgs& a, const int* idx, Prefetch& pf) {
  const int B = a.batch, D = a.D, Aw = a.discrete ? 1 : a.A;
#pragma unroll
  for (int u = 0; u < kPfObs; ++u) {
    const int e = threadIdx.x + u * kThreads;
    if (e < B * D) {
      const int r = e / D, c = e - r * D;
      pf.ob[u] = a.obs[(size_t)idx[r] * D + c];
    }
  }
#pragma unroll
  for (int u = 0; u < kPfAct; ++u) {
    const int e = threadIdx.x + u * kThreads;
    if (e < B * Aw) {
      const int r = e / Aw, c = e - r * Aw;
      pf.ac[u] = a.acts[(size_t)idx[r] * Aw + c];
    }
  }
  if (threadIdx.x < B) {
    const int r = idx[threadIdx.x];
    pf.lp = a.old_logp[r];
    pf.adv = a.adv[r];
    pf.ret = a.returns[r];
  }
}

__device__ __forceinline__ void stage_rows(const PPOArgs& a, const Bufs& bf, const Prefetch& pf) {
  const int B = a.batch, D = a.D, Aw = a.discrete ? 1 : a.A;
#pragma unroll
  for (int u = 0; u < kPfObs; ++u) {
    const int e = threadIdx.x + u * kThreads;
    if (e < B * D) bf.raw[e] = pf.ob[u];
  }
#pragma unroll
  for (int u = 0; u < kPfAct; ++u) {
    const int e = threadIdx.x + u * kThreads;
    if (e < B * Aw) bf.acts[e] = pf.ac[u];
  }
  if (threadIdx.x < B) {
    bf.rowv[0 * kMaxB + threadIdx.x] = pf.lp;
    bf.rowv[1 * kMaxB + threadIdx.x] = pf.adv;
    bf.rowv[2 * kMaxB + threadIdx.x] = pf.ret;
  }
}

// normaliser update + advantage normalisation + normalised input image H0
__device__ __forceinline__ void prepare_minibatch(const PPOArgs& a, const Bufs& bf, bool update_norm) {
  const int B = a.batch, D = a.D;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  lf* nmean = bf.norm;
  lf* nvar = bf.norm + 64;
  lf* ncount = bf.norm + 128;
  if (a.has_norm && update_norm) {
    const float cnt = ncount[0];
    const float tot = cnt + (float)B;
    for (int c = w; c < D; c += kWaves) {  // one feature per wave, one row per lane
      const float v = lane < B ? bf.raw[lane * D + c] : 0.f;
      const float m = wsum(v) / (float)B;
      const float d = lane < B ? v - m : 0.f;
      const float var = wsum(d * d) / (float)B;
      if (lane == 0) {
        const float delta = m - nmean[c];
        nmean[c] += delta * (float)B / tot;
        nvar[c] = (nvar[c] * cnt + var * (float)B + delta * delta * cnt * (float)B / tot) / tot;
      }
    }
  }
  // advantage normalisation (last wave): (adv - mean) / (std_unbiased + 1e-8)
  if (w == kWaves - 1 && a.normalize_advantage && B > 1) {
    const float v = lane < B ? bf.rowv[1 * kMaxB + lane] : 0.f;
    const float m = wsum(v) / (float)B;
    const float d = lane < B ? v - m : 0.f;
    const float sd = sqrtf(wsum(d * d) / (float)(B - 1));
    if (lane < B) bf.rowv[1 * kMaxB + lane] = d / (sd + 1e-8f);
  }
  __syncthreads();
  if (a.has_norm && update_norm && threadIdx.x == 0) ncount[0] += (float)B;
  const int ldx = ldp(D);
  for (int e = threadIdx.x; e < B * ldx; e += kThreads) {
    const int r = e / ldx, c = e - r * ldx;
    float v = c == D ? 1.f : 0.f;
    if (c < D) {
      v = bf.raw[r * D + c];
      if (a.has_norm) v = (v - nmean[c]) * rsqrtf(nvar[c] + a.norm_eps);
    }
    bf.H0[e] = v;
  }
}

// ---------------------------------------------------------------- losses (one wave each)
// Actor head -> dZa, log-std gradient, statistics. Runs on wave 0 only: B <= 64 rows,
// one row per lane, every row reduction is a wave shuffle.
__device__ __forceinline__ void policy_loss(const PPOArgs& a, const Bufs& bf, int dout) {
  const int B = a.batch;
  const int lane = threadIdx.x & 63;
  const int ldo = ldp(dout);
  const lf* head = Hq<0>(bf, a.n_pi);
  const float invB = 1.f / (float)B;
  const float c_half_log2pi = 0.91893853320467274f;
  const lf* log_std = bf.ls;
  const bool valid = lane < B;
  const int r = valid ? lane : 0;
  lf* dz = bf.dZa;
  float logp = 0.f, ent = 0.f, mx = 0.f, lz = 0.f;
  if (a.discrete) {
    mx = -INFINITY;
    for (int k = 0; k < dout; ++k) mx = fmaxf(mx, head[r * ldo + k]);
    float zsum = 0.f;
    for (int k = 0; k < dout; ++k) zsum += expf(head[r * ldo + k] - mx);
    lz = logf(zsum);
    logp = head[r * ldo + (int)bf.acts[r]] - mx - lz;
    for (int k = 0; k < dout; ++k) {
      const float lp = head[r * ldo + k] - mx - lz;
      ent -= expf(lp) * lp;
    }
  } else {
    for (int k = 0; k < a.A; ++k) {
      const float zz = (bf.acts[r * a.A + k] - head[r * ldo + k]) * expf(-log_std[k]);
      logp += -0.5f * zz * zz - log_std[k] - c_half_log2pi;
    }
  }
  const float adv = bf.rowv[1 * kMaxB + r];
  const float lr_ = logp - bf.rowv[0 * kMaxB + r];
  const float ratio = expf(lr_);
  const float lo = 1.f - a.clip_range, hi = 1.f + a.clip_range;
  const float pl1 = adv * ratio, pl2 = adv * fminf(fmaxf(ratio, lo), hi);
  float c1, c2;  // torch.min sends the gradient to the smaller operand, half each on ties
  if (pl1 < pl2) { c1 = 1.f; c2 = 0.f; } else if (pl2 < pl1) { c1 = 0.f; c2 = 1.f; } else { c1 = 0.5f; c2 = 0.5f; }
  const float inside = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
  const float dlogp = valid ? -invB * (c1 * adv + c2 * adv * inside) * ratio : 0.f;
  if (a.discrete) {
    const int act = (int)bf.acts[r];
    for (int k = 0; k < ldo; ++k) {
      float g = 0.f;
      if (k < dout) {
        const float lp = head[r * ldo + k] - mx - lz;
        const float pk = expf(lp);
        g = dlogp * ((k == act ? 1.f : 0.f) - pk) - a.ent_coef * invB * (-pk * (lp + ent));
      }
      if (valid) dz[r * ldo + k] = g;
    }
  } else {
    for (int k = 0; k < ldo; ++k) {
      float g = 0.f;
      if (k < a.A) {
        const float is = expf(-log_std[k]);
        const float df = bf.acts[r * a.A + k] - head[r * ldo + k];
        g = dlogp * df * is * is;
        // d/dlog_std_k: sum_r dlogp_r (z^2 - 1) - ent_coef
        const float zz = df * is;
        const float gl = wsum(valid ? dlogp * (zz * zz - 1.f) : 0.f);
        if (lane == 0) bf.ls[16 + k] = gl - a.ent_coef;
      }
      if (valid) dz[r * ldo + k] = g;
    }
  }
  // statistics
  float ent_l;
  if (a.discrete) {
    ent_l = -wsum(valid ? ent : 0.f) * invB;
  } else {
    float sl = 0.f;
    for (int k = 0; k < a.A; ++k) sl += log_std[k];
    ent_l = -(sl + a.A * (0.5f + c_half_log2pi));
  }
  const float pg = wsum(valid ? -fminf(pl1, pl2) : 0.f) * invB;
  const float cf = wsum(valid && fabsf(ratio - 1.f) > a.clip_range ? 1.f : 0.f) * invB;
  const float kl = wsum(valid ? (ratio - 1.f) - lr_ : 0.f) * invB;
  if (lane == 0) {
    bf.red[8] += ent_l;
    bf.red[9] += pg;
    bf.red[11] += cf;
    bf.red[12] += kl;
  }
}

__device__ __forceinline__ void value_loss(const PPOArgs& a, const Bufs& bf) {
  const int B = a.batch;
  const int lane = threadIdx.x & 63;
  const lf* v = Hq<1>(bf, a.n_vf);
  const int ldo = ldp(1);
  float d = 0.f;
  if (lane < B) {
    d = v[lane * ldo] - bf.rowv[2 * kMaxB + lane];
    for (int k = 0; k < ldo; ++k) bf.dZc[lane * ldo + k] = k == 0 ? a.vf_coef * 2.f * d / (float)B : 0.f;
  }
  const float vl = wsum(d * d) / (float)B;
  if (lane == 0) bf.red[10] += vl;
}

// ---------------------------------------------------------------- clip_grad_norm_ + Adam
// Adam moments live in registers for the whole launch: thread t owns parameter-image
// elements t, t + kThreads, ... (kSlots of them) of the concatenated Wall/Gall
// regions, so the elementwise update touches LDS only for W and G.
template <int kSlots>
__device__ __forceinline__ void clip_and_adam(lf* lds, const PPOArgs& a, const Bufs& bf, float step, bool has_ls, float (&m)[kSlots],
                              float (&v)[kSlots]) {
  const int n_all = param_floats(a);
  lf* W = lds;
  const lf* G = lds + n_all;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < kSlots; ++j) {
    const int e = threadIdx.x + j * kThreads;
    if (e < n_all) ss += G[e] * G[e];
  }
  if (has_ls && threadIdx.x < a.A) ss += bf.ls[16 + threadIdx.x] * bf.ls[16 + threadIdx.x];
  ss = wsum(ss);
  if ((threadIdx.x & 63) == 0) bf.red[threadIdx.x >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) tot += bf.red[w];
  const float norm = sqrtf(tot);
  const float coef = fminf(1.f, a.max_grad_norm / (norm + 1e-6f));
  const float bc1 = 1.f - powf(a.beta1, step);
  const float bc2s = sqrtf(1.f - powf(a.beta2, step));
  const float step_size = a.lr / bc1;
  const float b1 = a.beta1, b2 = a.beta2, eps = a.adam_eps;
#pragma unroll
  for (int j = 0; j < kSlots; ++j) {
    const int e = threadIdx.x + j * kThreads;
    if (e < n_all) {
      const float g = G[e] * coef;
      m[j] = b1 * m[j] + (1.f - b1) * g;
      v[j] = b2 * v[j] + (1.f - b2) * g * g;
      W[e] -= step_size * m[j] / (sqrtf(v[j]) / bc2s + eps);
    }
  }
  if (has_ls && threadIdx.x < a.A) {
    lf* ls = bf.ls;
    const int k = threadIdx.x;
    const float g = ls[16 + k] * coef;
    const float mm = b1 * ls[32 + k] + (1.f - b1) * g;
    const float vv = b2 * ls[48 + k] + (1.f - b2) * g * g;
    ls[32 + k] = mm;
    ls[48 + k] = vv;
    ls[k] -= step_size * mm / (sqrtf(vv) / bc2s + eps);
  }
  __syncthreads();
}

// Moments: global flat vector <-> registers, staged through the gradient region.
template <int kSlots>
__device__ __forceinline__ void moments_in(lf* lds, const PPOArgs& a, const float* flat, float (&r)[kSlots]) {
  const int n_all = param_floats(a);
#pragma unroll
  for (int li = 0; li < kL; ++li) {
    if (li < a.n_pi) { const Lay y = lay<0>(lds, a, li); img_load(y.gW, y.gb, flat, y); }
    if (li < a.n_vf) { const Lay y = lay<1>(lds, a, li); img_load(y.gW, y.gb, flat, y); }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSlots; ++j) {
    const int e = threadIdx.x + j * kThreads;
    r[j] = e < n_all ? lds[n_all + e] : 0.f;
  }
  __syncthreads();
}
template <int kSlots>
__device__ __forceinline__ void moments_out(lf* lds, const PPOArgs& a, float* flat, const float (&r)[kSlots]) {
  const int n_all = param_floats(a);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kSlots; ++j) {
    const int e = threadIdx.x + j * kThreads;
    if (e < n_all) lds[n_all + e] = r[j];
  }
  __syncthreads();
#pragma unroll
  for (int li = 0; li < kL; ++li) {
    if (li < a.n_pi) { const Lay y = lay<0>(lds, a, li); img_store(y.gW, y.gb, flat, y); }
    if (li < a.n_vf) { const Lay y = lay<1>(lds, a, li); img_store(y.gW, y.gb, flat, y); }
  }
}

template <int kSlots>
__global__ __launch_bounds__(kThreads) void ppo_kernel(PPOArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_raw[];
  lf* lds = (lf*)lds_raw;
  const Bufs bf = bufs(lds, a);
  li32* tab = (li32*)(bf.red + 32);  // [2][kL][8]
  const int w = threadIdx.x >> 6;
  const int grp = w / kGroup, gw = w - grp * kGroup;
  const bool has_ls = a.log_std_off >= 0 && !a.discrete;
  const bool need_moments = a.mode != 1;

  float mom1[kSlots], mom2[kSlots];
#pragma unroll
  for (int j = 0; j < kSlots; ++j) mom1[j] = mom2[j] = 0.f;
  if (need_moments) {
    moments_in(lds, a, a.exp_avg, mom1);
    moments_in(lds, a, a.exp_avg_sq, mom2);
  }
#pragma unroll
  for (int li = 0; li < kL; ++li) {
    if (li < a.n_pi) {
      const Lay y = lay<0>(lds, a, li);
      img_load(y.W, y.b, a.params, y);
      if (a.mode == 2) img_load(y.gW, y.gb, a.grads, y);
    }
    if (li < a.n_vf) {
      const Lay y = lay<1>(lds, a, li);
      img_load(y.W, y.b, a.params, y);
      if (a.mode == 2) img_load(y.gW, y.gb, a.grads, y);
    }
  }
  // gradient padding must stay zero (backward only writes the valid entries)
  if (a.mode != 2) img_zero(lds + param_floats(a), param_floats(a));
  if (threadIdx.x == 0) write_lt<0>(tab, lds, a, bf);
  if (threadIdx.x == 64) write_lt<1>(tab, lds, a, bf);
  if (threadIdx.x < 16) {
    const int k = threadIdx.x;
    const bool ok = has_ls && k < a.A;
    bf.ls[k] = ok ? a.params[a.log_std_off + k] : 0.f;
    bf.ls[16 + k] = (ok && a.mode == 2) ? a.grads[a.log_std_off + k] : 0.f;
    bf.ls[32 + k] = (ok && need_moments) ? a.exp_avg[a.log_std_off + k] : 0.f;
    bf.ls[48 + k] = (ok && need_moments) ? a.exp_avg_sq[a.log_std_off + k] : 0.f;
  }
  if (threadIdx.x < 32) bf.red[threadIdx.x] = 0.f;
  if (a.has_norm) {
    for (int c = threadIdx.x; c < a.D; c += kThreads) {
      bf.norm[c] = a.norm_mean[c];
      bf.norm[64 + c] = a.norm_var[c];
    }
    if (threadIdx.x == 0) bf.norm[128] = a.norm_count_i ? (float)a.norm_count_i[0] : a.norm_count[0];
  }

  const int n_mb = a.rows / a.batch;
  float step = a.adam_step[0];
  int first = 0, last = 0;
  if (a.mode == 0) last = a.n_epochs * n_mb;
  if (a.mode == 1) { first = a.mb_index; last = a.mb_index + 1; }
  const int L = a.n_pi > a.n_vf ? a.n_pi : a.n_vf;
  const int myL = grp == 0 ? a.n_pi : a.n_vf;  // layer count of this wave's net
  const int pi_out = a.pi_dims[a.n_pi];
  const int B = a.batch;
  Prefetch pf;
  if (first < last) prefetch_rows(a, a.perm + (size_t)first * a.batch, pf);
  unsigned long long prof[6] = {0, 0, 0, 0, 0, 0};
  __syncthreads();
  for (int it = first; it < last; ++it) {
    unsigned long long t0 = clock64(), t1;
#define IA_PROF(i)       \
  if (a.prof) {          \
    t1 = clock64();      \
    prof[i] += t1 - t0;  \
    t0 = t1;             \
  }
    stage_rows(a, bf, pf);
    __syncthreads();
    if (it + 1 < last) prefetch_rows(a, a.perm + (size_t)(it + 1) * a.batch, pf);  // perm is [epochs][rows]
    IA_PROF(0)
    prepare_minibatch(a, bf, a.mode == 0);
    __syncthreads();
    IA_PROF(1)
    for (int li = 0; li < L; ++li) {  // actor (waves 0-3) and critic (waves 4-7) in lock-step
      if (li < myL) fwd_stage(lds, load_lt(tab, grp * kL + li), B, gw);
      __syncthreads();
    }
    IA_PROF(2)
    if (w == 0) policy_loss(a, bf, pi_out);
    if (w == kGroup) value_loss(a, bf);
    __syncthreads();
    IA_PROF(3)
    for (int t = 0; t < L; ++t) {
      const int li = myL - 1 - t;
      if (li >= 0) bwd_stage(lds, load_lt(tab, grp * kL + li), B, gw, li > 0, a.hidden_act);
      __syncthreads();
    }
    IA_PROF(4)
    if (a.mode == 0) {
      step += 1.f;
      clip_and_adam<kSlots>(lds, a, bf, step, has_ls, mom1, mom2);
    }
    IA_PROF(5)
#undef IA_PROF
  }
  if (a.mode == 2) {
    step += 1.f;
    clip_and_adam<kSlots>(lds, a, bf, step, has_ls, mom1, mom2);
  }
  __syncthreads();
#pragma unroll
  for (int li = 0; li < kL; ++li) {
    if (li < a.n_pi) {
      const Lay y = lay<0>(lds, a, li);
      if (a.mode == 1) img_store(y.gW, y.gb, a.grads, y);
      else img_store(y.W, y.b, a.params, y);
    }
    if (li < a.n_vf) {
      const Lay y = lay<1>(lds, a, li);
      if (a.mode == 1) img_store(y.gW, y.gb, a.grads, y);
      else img_store(y.W, y.b, a.params, y);
    }
  }
  if (need_moments) {
    moments_out(lds, a, a.exp_avg, mom1);
    moments_out(lds, a, a.exp_avg_sq, mom2);
  }
  if (threadIdx.x < a.A && has_ls) {
    const int k = threadIdx.x;
    if (a.mode == 1) {
      a.grads[a.log_std_off + k] = bf.ls[16 + k];
    } else {
      a.params[a.log_std_off + k] = bf.ls[k];
      a.exp_avg[a.log_std_off + k] = bf.ls[32 + k];
      a.exp_avg_sq[a.log_std_off + k] = bf.ls[48 + k];
    }
  }
  if (threadIdx.x < 5) a.stats[threadIdx.x] += bf.red[8 + threadIdx.x];
  if (a.mode != 1 && threadIdx.x == 0) a.adam_step[0] = step;
  if (a.has_norm && a.mode == 0) {
    for (int c = threadIdx.x; c < a.D; c += kThreads) {
      a.norm_mean[c] = bf.norm[c];
      a.norm_var[c] = bf.norm[64 + c];
    }
    if (threadIdx.x == 0) {
      if (a.norm_count_i) a.norm_count_i[0] = (int)bf.norm[128];
      else a.norm_count[0] = bf.norm[128];
    }
  }
  if (a.prof && threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < 6; ++i) a.prof[i] += prof[i];
  }
}

}  // namespace

size_t ppo_lds_bytes(const PPOArgs& a) { return (size_t)total_floats(a) * sizeof(float); }

hipError_t ppo_launch(const PPOArgs& a, hipStream_t s) {
  if (a.batch % 16 != 0 || a.batch > kMaxB || a.rows % a.batch != 0 || a.D > 64 || a.A > 16) return hipErrorInvalidValue;
  const size_t lds = ppo_lds_bytes(a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int slots = (param_floats(a) + kThreads - 1) / kThreads;
  if (slots <= 8) hipLaunchKernelGGL(ppo_kernel<8>, dim3(1), dim3(kThreads), lds, s, a);
  else if (slots <= 16) hipLaunchKernelGGL(ppo_kernel<16>, dim3(1), dim3(kThreads), lds, s, a);
  else if (slots <= 32) hipLaunchKernelGGL(ppo_kernel<32>, dim3(1), dim3(kThreads), lds, s, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace ia

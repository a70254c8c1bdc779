// NHWC implicit-GEMM convolutions on CDNA4 MFMA (bf16 operands, fp32 accumulate) for the
// NatureCNN trunk of the Atari policies (SB3 NatureCNN used via the reference's
// `cnn_policy`, scripts/ingredients/policy.py:48-50; DAgger-Pong, BASELINE config 4) and
// the reward CNNs (reward_nets.py:535-600 via util/networks.py:286-357 build_cnn).
//
// Frames arrive channel-last from the native Atari env ([B, 84, 84, 4]), so every kernel
// works on NHWC and the GEMM contraction index k = (kh, kw, c) has c fastest: for a fixed
// kh the KW*C taps of a row are CONTIGUOUS in memory. One MFMA operand fragment is 8
// consecutive k (v_mfma_f32_16x16x32_bf16: lane l holds A[m = l&15][k = 8*(l>>4) + j]),
// i.e. one 16-byte (bf16) / 32-byte (fp32) load straight from the activation tensor -- the
// forward and the data-gradient kernels need no LDS staging and no barrier at all:
//
//   conv_fwd    Y[m][n]  = act(sum_k X(m, k) W[n][k] + b[n])            m = (b, oh, ow)
//   conv_dgrad  dZp[p][c] = [Xp > 0] * sum_{tap, n} dZ(p, tap)[n] Wt[c][tap][n]   p = (b, ih, iw)
//                (tiles hold pixels of one stride phase, which only the KH*KW/S^2 taps of that
//                phase reach; border misses are skipped per wave with a ballot)
//   conv_wgrad  dW[n][k] = sum_m dZ[m][n] X(m, k),  db[n] = sum_m dZ[m][n]
//                (contraction over m needs m-contiguous operands: 32-row chunks of dZ and
//                of the im2col rows are staged transposed in LDS; each block reduces a
//                contiguous m range into fp32 partials, conv_reduce sums them in block
//                order -- deterministic, no atomics)
//
// dZ = dY * [Y > 0] (ReLU of the layer's own output) is formed on load when relu_out is
// set, so no separate mask kernel runs.
//
// Zero padding (g.P > 0: the reward CNNs' 3x3 stride-1 "same" convs, reward_nets.py:535-600
// / networks.py:286-357) needs C % 8 == 0, so a fragment's 8 consecutive k = (kh, kw, c..c+7)
// stay inside one tap: the fragment is loaded if that tap's input pixel is inside the image
// and is zero otherwise. K = KH*KW*C is padded to Kp (a multiple of 32) with zero weight
// columns; fragments past K read as zero too.
#include <hip/hip_runtime.h>

#include "ia/mfma.h"
#include "gather_body.h"
#include "wgrad_reduce.h"
#include "launchers.h"

namespace ia {
namespace {

// rows per wgrad chunk: 128 (or 64 where the chunk's LDS images would not fit) once a layer
// has at least kWgradBigM GEMM rows, else 32
constexpr int kWgradBigM = 1 << 14;
__host__ __device__ __forceinline__ int wgrad_chunk(const ConvGeo& g) {
  if (g.B * g.OH * g.OW < kWgradBigM) return 32;
  const int rows = g.Kp + g.N;  // LDS image rows (bf16)
  if (rows * (128 + 8) * 2 <= 160 * 1024) return 128;
  if (rows * (64 + 8) * 2 <= 160 * 1024) return 64;
  return 32;
}

__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
  return z;
}

// 8 consecutive input elements -> bf16x8 (scaled)
__device__ __forceinline__ bf16x8 load8(const bf16* p, float) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ bf16x8 load8(const float* p, float s) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  bf16x8 v;
  v[0] = (bf16)(a.x * s); v[1] = (bf16)(a.y * s); v[2] = (bf16)(a.z * s); v[3] = (bf16)(a.w * s);
  v[4] = (bf16)(b.x * s); v[5] = (bf16)(b.y * s); v[6] = (bf16)(b.z * s); v[7] = (bf16)(b.w * s);
  return v;
}
__device__ __forceinline__ bf16x8 load8(const uint8_t* p, float s) {
  const uint32_t a = *reinterpret_cast<const uint32_t*>(p);
  const uint32_t b = *reinterpret_cast<const uint32_t*>(p + 4);
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = (bf16)((float)((a >> (8 * j)) & 0xffu) * s);
    v[4 + j] = (bf16)((float)((b >> (8 * j)) & 0xffu) * s);
  }
  return v;
}

// dZ fragment of 8 consecutive channels: dY * [Y > 0] when relu_out
__device__ __forceinline__ bf16x8 load_dz8(const bf16* dY, const bf16* Y, size_t off, int relu_out) {
  bf16x8 d = *reinterpret_cast<const bf16x8*>(dY + off);
  if (relu_out) {
    const bf16x8 y = *reinterpret_cast<const bf16x8*>(Y + off);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!((float)y[j] > 0.f)) d[j] = (bf16)0.f;
  }
  return d;
}

// ------------------------------------------------------------------ forward
// tap-checked fragment of a padded conv: 8 consecutive k at k (k % 8 == 0, C % 8 == 0)
template <typename TIn>
__device__ __forceinline__ bf16x8 load8_pad(const TIn* X, const ConvGeo& g, int b, int oh, int ow, int k, bool mv,
                                            float in_scale) {
  const int tap = k / g.C, c = k - tap * g.C;
  const int kh = tap / g.KW, kw = tap - kh * g.KW;
  const int ih = oh * g.S - g.P + kh, iw = ow * g.S - g.P + kw;
  if (!mv || kh >= g.KH || (unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return zero8();
  return load8(X + ((size_t)(b * g.H + ih) * g.W + iw) * g.C + c, in_scale);
}

// RT row tiles (16 output pixels each) per wave share every weight fragment: at large M the
// per-wave weight re-reads from L2, not the MFMAs, set the forward's time.
template <typename TIn, int NT, bool PADDED = false, int RT = 1>
__device__ __forceinline__ void conv_fwd_tile(const TIn* __restrict__ X, const bf16* __restrict__ Wb,
                                              const float* __restrict__ bias, bf16* __restrict__ Y, const ConvGeo& g,
                                              float in_scale, int relu, int bx, int by) {
  const int l = threadIdx.x & 63;
  const int m0 = (bx * 4 + (threadIdx.x >> 6)) * 16 * RT;
  const int OHW = g.OH * g.OW;
  const int M = g.B * OHW;
  if (m0 >= M) return;
  const int K = g.Kp;
  const int n_base = by * 16 * NT;  // split-N grids (small batches): this block's channels
  const int rowlen = g.KW * g.C;
  const int r = l & 15, kq = (l >> 4) * 8;
  const size_t xrow = (size_t)g.W * g.C;
  int rb[RT], roh[RT], row_[RT];
  bool rmv[RT];
  const TIn* xb[RT];
#pragma unroll
  for (int ri = 0; ri < RT; ++ri) {
    const int m = m0 + ri * 16 + r;
    rmv[ri] = m < M;
    const int mm = rmv[ri] ? m : M - 1;
    const int b = mm / OHW, pix = mm - b * OHW, oh = pix / g.OW, ow = pix - oh * g.OW;
    rb[ri] = b;
    roh[ri] = oh;
    row_[ri] = ow;
    xb[ri] = PADDED ? X : X + ((size_t)(b * g.H + oh * g.S) * g.W + (size_t)ow * g.S) * g.C;
  }
  f32x4 acc[RT][NT];
#pragma unroll
  for (int ri = 0; ri < RT; ++ri)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[ri][t] = zero4();
  const bf16* wr = Wb + (size_t)(n_base + r) * K + kq;
  // KB k-steps' operand loads are issued before their MFMAs: at the small batches (collector,
  // BC) a wave's time is its chain of per-k-step load round trips, so 8 in flight instead of 2
  // cuts the round trips per tile ~4x. Same MFMA sequence per accumulator (bitwise).
  constexpr int KB = NT * RT >= 8 ? 1 : 8 / (NT * RT);
  for (int k0 = 0; k0 < K; k0 += 32 * KB) {
    bf16x8 bv[KB][NT], av[KB][RT];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int ku = k0 + 32 * u;
      if (ku >= K) break;
      const int k = ku + kq;
#pragma unroll
      for (int t = 0; t < NT; ++t) bv[u][t] = *reinterpret_cast<const bf16x8*>(wr + (size_t)t * 16 * K + ku);
      int tap_c = 0, tap_kh = 0, tap_kw = 0;
      if constexpr (PADDED) {
        const int tap = k / g.C;
        tap_c = k - tap * g.C;
        tap_kh = tap / g.KW;
        tap_kw = tap - tap_kh * g.KW;
      }
#pragma unroll
      for (int ri = 0; ri < RT; ++ri) {
        if constexpr (PADDED) {
          const int ih = roh[ri] * g.S - g.P + tap_kh, iw = row_[ri] * g.S - g.P + tap_kw;
          const bool ok = rmv[ri] && tap_kh < g.KH && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
          av[u][ri] = ok ? load8(X + ((size_t)(rb[ri] * g.H + ih) * g.W + iw) * g.C + tap_c, in_scale) : zero8();
        } else {
          const int kh = k / rowlen, off = k - kh * rowlen;
          av[u][ri] = load8(xb[ri] + kh * xrow + off, in_scale);
          if (!rmv[ri]) av[u][ri] = zero8();
        }
      }
    }
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      if (k0 + 32 * u >= K) break;
#pragma unroll
      for (int ri = 0; ri < RT; ++ri)
#pragma unroll
        for (int t = 0; t < NT; ++t)
          acc[ri][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[u][ri], bv[u][t], acc[ri][t], 0, 0, 0);
    }
  }
  const int col = l & 15;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int n = n_base + t * 16 + col;
    const float bb = bias ? bias[n] : 0.f;
#pragma unroll
    for (int ri = 0; ri < RT; ++ri) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = m0 + ri * 16 + 4 * (l >> 4) + i;
        if (row < M) {
          float v = acc[ri][t][i] + bb;
          if (relu) v = fmaxf(v, 0.f);
          Y[(size_t)row * g.N + n] = (bf16)v;
        }
      }
    }
  }
}

template <typename TIn, int NT, bool PADDED = false, int RT = 1>
__global__ __launch_bounds__(256) void conv_fwd_kernel(const TIn* __restrict__ X, const bf16* __restrict__ Wb,
                                                       const float* __restrict__ bias, bf16* __restrict__ Y, ConvGeo g,
                                                       float in_scale, int relu) {
  conv_fwd_tile<TIn, NT, PADDED, RT>(X, Wb, bias, Y, g, in_scale, relu, blockIdx.x, blockIdx.y);
}

// Split-K forward for BC-size batches: one 16 x 16 output tile per block of KS waves, wave w taking
// k-steps [w * per, (w + 1) * per) with all of its operand loads issued at once, the KS partial tiles
// summed through LDS in wave order. conv_fwd_tile's waves walk the whole K in rounds of 8 k-steps: at
// batch 32 its few hundred waves each wait on 2-3 dependent load rounds. Different summation order from
// conv_fwd_tile (not bitwise with it); used where the caller asks for it (the fused BC step).
constexpr int kSkMaxSteps = 8;
template <typename TIn, int KS>
__global__ __launch_bounds__(64 * KS) void conv_fwd_sk_kernel(const TIn* __restrict__ X, const bf16* __restrict__ Wb,
                                                              const float* __restrict__ bias, bf16* __restrict__ Y,
                                                              ConvGeo g, float in_scale, int relu) {
  __shared__ f32x4 part[KS][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int OHW = g.OH * g.OW, M = g.B * OHW;
  const int m0 = blockIdx.x * 16, n0 = blockIdx.y * 16;
  const int K = g.Kp, steps = K / 32, per = (steps + KS - 1) / KS;
  const int s0 = w * per, s1 = min(steps, s0 + per);
  const int r = l & 15, kq = (l >> 4) * 8;
  const int m = m0 + r;
  const bool mv = m < M;
  const int mm = mv ? m : M - 1;
  const int b = mm / OHW, pix = mm - b * OHW, oh = pix / g.OW, ow = pix - oh * g.OW;
  const TIn* xb = X + ((size_t)(b * g.H + oh * g.S) * g.W + (size_t)ow * g.S) * g.C;
  const int rowlen = g.KW * g.C;
  const size_t xrow = (size_t)g.W * g.C;
  const bf16* wr = Wb + (size_t)(n0 + r) * K + kq;
  bf16x8 av[kSkMaxSteps], bv[kSkMaxSteps];
#pragma unroll
  for (int u = 0; u < kSkMaxSteps; ++u) {  // every k-step's operands in flight at once
    const int st = s0 + u;
    if (st < s1) {  // (wave-uniform)
      const int k = st * 32 + kq, kh = k / rowlen, off = k - kh * rowlen;
      av[u] = load8(xb + kh * xrow + off, in_scale);
      if (!mv) av[u] = zero8();
      bv[u] = *reinterpret_cast<const bf16x8*>(wr + st * 32);
    }
  }
  f32x4 acc = zero4();
#pragma unroll
  for (int u = 0; u < kSkMaxSteps; ++u)
    if (s0 + u < s1) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[u], bv[u], acc, 0, 0, 0);
  part[w][l] = acc;
  __syncthreads();
  if (w != 0) return;
  f32x4 sum = part[0][l];
#pragma unroll
  for (int v = 1; v < KS; ++v) {
    const f32x4 x = part[v][l];
    sum[0] += x[0];
    sum[1] += x[1];
    sum[2] += x[2];
    sum[3] += x[3];
  }
  const int n = n0 + (l & 15);
  const float bb = bias ? bias[n] : 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + 4 * (l >> 4) + i;
    if (row < M) {
      float v = sum[i] + bb;
      if (relu) v = fmaxf(v, 0.f);
      Y[(size_t)row * g.N + n] = (bf16)v;
    }
  }
}

// Two same-shape convolutions in one launch (blockIdx.z = which): the DAgger collector's
// expert and learner CNNs step the same frames, so each layer of both is one small-batch
// split-N grid of twice the blocks instead of two latency-bound launches.
template <typename TIn>
__global__ __launch_bounds__(256) void conv_fwd_pair_kernel(ConvPair p, ConvGeo g, float in_scale, int relu) {
  const int z = blockIdx.z;
  conv_fwd_tile<TIn, 1>(static_cast<const TIn*>(p.X[z]), static_cast<const bf16*>(p.W[z]), p.bias[z],
                        static_cast<bf16*>(p.Y[z]), g, in_scale, relu, blockIdx.x, blockIdx.y);
}

// ------------------------------------------------------------------ data gradient
// Pixels are grouped by stride phase (ih % S, iw % S) (blockIdx.y): every pixel of a phase
// is hit by the same kh = ph (mod S), kw = pw (mod S) taps, so a tile only walks those
// (1/S^2 of KH*KW) and only the image border still masks rows.
template <int CT, int RT = 1>
__global__ __launch_bounds__(256) void conv_dgrad_kernel(const bf16* __restrict__ dY, const bf16* __restrict__ Y,
                                                         const bf16* __restrict__ Wt, const bf16* __restrict__ Xp,
                                                         bf16* __restrict__ dZp, ConvGeo g, int relu_out, int relu_in) {
  const int l = threadIdx.x & 63;
  const int ph = blockIdx.y / g.S, pw = blockIdx.y - ph * g.S;
  const int Hc = (g.H - ph + g.S - 1) / g.S, Wc = (g.W - pw + g.S - 1) / g.S;
  const int HWc = Hc * Wc;
  const int P = g.B * HWc;  // pixels of this phase
  const int p0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 * RT;
  if (p0 >= P) return;
  const int Kp = g.KH * g.KW * g.N;
  const int r = l & 15, kq = (l >> 4) * 8;
  auto pix_of = [&](int q, int& b, int& ih, int& iw) {
    b = q / HWc;
    const int rem = q - b * HWc, i = rem / Wc, j = rem - i * Wc;
    ih = ph + g.S * i;
    iw = pw + g.S * j;
  };
  int pb[RT], pih[RT], piw[RT];
  bool pv[RT];
#pragma unroll
  for (int ri = 0; ri < RT; ++ri) {
    const int p = p0 + ri * 16 + r;
    pv[ri] = p < P;
    pix_of(pv[ri] ? p : P - 1, pb[ri], pih[ri], piw[ri]);
  }
  f32x4 acc[RT][CT];
#pragma unroll
  for (int ri = 0; ri < RT; ++ri)
#pragma unroll
    for (int t = 0; t < CT; ++t) acc[ri][t] = zero4();
  const bf16* wr = Wt + (size_t)r * Kp + kq;
  // (padded convs are stride 1: one phase, every tap; output pixel (ih + P - kh, iw + P - kw))
  for (int kh = ph; kh < g.KH; kh += g.S) {
    for (int kw = pw; kw < g.KW; kw += g.S) {
      bool valid[RT];
      size_t dzoff[RT];
      bool any = false;
#pragma unroll
      for (int ri = 0; ri < RT; ++ri) {
        const int th = pih[ri] + g.P - kh, tw = piw[ri] + g.P - kw;
        const int oh = th / g.S, ow = tw / g.S;
        valid[ri] = pv[ri] && th >= 0 && oh < g.OH && tw >= 0 && ow < g.OW;
        dzoff[ri] = valid[ri] ? ((size_t)(pb[ri] * g.OH + oh) * g.OW + ow) * g.N + kq : 0;
        any |= __ballot(valid[ri]) != 0ull;
      }
      if (!any) continue;  // this tap misses every pixel of the wave's tiles (border)
      const int kbase = (kh * g.KW + kw) * g.N;
      for (int n0 = 0; n0 < g.N; n0 += 32) {
        bf16x8 bv[CT];
#pragma unroll
        for (int t = 0; t < CT; ++t) bv[t] = *reinterpret_cast<const bf16x8*>(wr + (size_t)t * 16 * Kp + kbase + n0);
#pragma unroll
        for (int ri = 0; ri < RT; ++ri) {
          bf16x8 av = zero8();
          if (valid[ri]) av = load_dz8(dY, Y, dzoff[ri] + n0, relu_out);
#pragma unroll
          for (int t = 0; t < CT; ++t) acc[ri][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv[t], acc[ri][t], 0, 0, 0);
        }
      }
    }
  }
  const int col = l & 15;
#pragma unroll
  for (int ri = 0; ri < RT; ++ri) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = p0 + ri * 16 + 4 * (l >> 4) + i;
      if (q >= P) continue;
      int bb, hh, ww;
      pix_of(q, bb, hh, ww);
      const size_t row = ((size_t)bb * g.H + hh) * g.W + ww;
#pragma unroll
      for (int t = 0; t < CT; ++t) {
        const int c = t * 16 + col;
        float v = acc[ri][t][i];
        if (relu_in && !((float)Xp[row * g.C + c] > 0.f)) v = 0.f;
        dZp[row * g.C + c] = (bf16)v;
      }
    }
  }
}

// Small-batch data gradient (one 16-pixel tile per wave, N = 32 NN output channels): the same
// tap order and MFMA sequence per accumulator as conv_dgrad_kernel<CT, 1> (bitwise), but the
// loads of the next kDgDepth taps are in flight while a tap's MFMAs run. At BC batch sizes the
// grid is < 1 wave per CU and the kernel time is one wave's dependent chain of per-tap load
// round trips (NatureCNN conv3: 9 taps x 2 channel halves ~ 18 us); with 3 taps in flight it
// is about a third of that.
constexpr int kDgDepth = 3;

template <int CT, int NN>
struct DgTap {
  bool any, valid;
  bf16x8 a[NN];
  bf16x8 b[NN][CT];
};

template <int CT, int NN>
__global__ __launch_bounds__(256) void conv_dgrad_pf_kernel(const bf16* __restrict__ dY, const bf16* __restrict__ Y,
                                                            const bf16* __restrict__ Wt, const bf16* __restrict__ Xp,
                                                            bf16* __restrict__ dZp, ConvGeo g, int relu_out, int relu_in) {
  const int l = threadIdx.x & 63;
  const int ph = blockIdx.y / g.S, pw = blockIdx.y - ph * g.S;
  const int Hc = (g.H - ph + g.S - 1) / g.S, Wc = (g.W - pw + g.S - 1) / g.S;
  const int HWc = Hc * Wc;
  const int P = g.B * HWc;
  const int p0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16;
  if (p0 >= P) return;
  const int Kp = g.KH * g.KW * g.N;
  const int r = l & 15, kq = (l >> 4) * 8;
  auto pix_of = [&](int q, int& b, int& ih, int& iw) {
    b = q / HWc;
    const int rem = q - b * HWc, i = rem / Wc, j = rem - i * Wc;
    ih = ph + g.S * i;
    iw = pw + g.S * j;
  };
  int pb, pih, piw;
  const bool pv = p0 + r < P;
  pix_of(pv ? p0 + r : P - 1, pb, pih, piw);
  f32x4 acc[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) acc[t] = zero4();
  const bf16* wr = Wt + (size_t)r * Kp + kq;
  const int nkw = (g.KW - pw + g.S - 1) / g.S;
  const int ntap = ((g.KH - ph + g.S - 1) / g.S) * nkw;
  auto load_tap = [&](int tp, DgTap<CT, NN>& st) {
    const int kh = ph + g.S * (tp / nkw), kw = pw + g.S * (tp - (tp / nkw) * nkw);
    const int th = pih + g.P - kh, tw = piw + g.P - kw;
    const int oh = th / g.S, ow = tw / g.S;
    st.valid = pv && th >= 0 && oh < g.OH && tw >= 0 && ow < g.OW;
    st.any = __ballot(st.valid) != 0ull;
    const size_t dzoff = st.valid ? ((size_t)(pb * g.OH + oh) * g.OW + ow) * g.N + kq : 0;
    const int kbase = (kh * g.KW + kw) * g.N;
#pragma unroll
    for (int nn = 0; nn < NN; ++nn) {
#pragma unroll
      for (int t = 0; t < CT; ++t) st.b[nn][t] = *reinterpret_cast<const bf16x8*>(wr + (size_t)t * 16 * Kp + kbase + 32 * nn);
      st.a[nn] = st.valid ? load_dz8(dY, Y, dzoff + 32 * nn, relu_out) : zero8();
    }
  };
  auto run_tap = [&](const DgTap<CT, NN>& st) {
    if (!st.any) return;  // (the tap misses every pixel of the wave's tile: no MFMA, as before)
#pragma unroll
    for (int nn = 0; nn < NN; ++nn)
#pragma unroll
      for (int t = 0; t < CT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(st.a[nn], st.b[nn][t], acc[t], 0, 0, 0);
  };
  DgTap<CT, NN> ring[kDgDepth];
#pragma unroll
  for (int d = 0; d < kDgDepth; ++d)
    if (d < ntap) load_tap(d, ring[d]);
  for (int tp = 0; tp < ntap; tp += kDgDepth) {
#pragma unroll
    for (int d = 0; d < kDgDepth; ++d) {
      if (tp + d < ntap) {
        run_tap(ring[d]);
        if (tp + d + kDgDepth < ntap) load_tap(tp + d + kDgDepth, ring[d]);
      }
    }
  }
  const int col = l & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = p0 + 4 * (l >> 4) + i;
    if (q >= P) continue;
    int bb, hh, ww;
    pix_of(q, bb, hh, ww);
    const size_t row = ((size_t)bb * g.H + hh) * g.W + ww;
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int c = t * 16 + col;
      float v = acc[t][i];
      if (relu_in && !((float)Xp[row * g.C + c] > 0.f)) v = 0.f;
      dZp[row * g.C + c] = (bf16)v;
    }
  }
}

// Small-batch data gradient with the tap loop split over waves: a block is ONE 16-pixel tile and
// TS x NN waves, wave w = (tap group w / NN, channel half w % NN) accumulating its taps of one
// 32-channel half of dZ; the TS * NN partial tiles are summed through LDS in wave order. At BC
// batch sizes the grid of conv_dgrad_pf_kernel is a few hundred waves and each wave's time is its
// chain of per-tap load round trips (NatureCNN conv3: 9 taps x 2 halves, 19 us); here each wave
// issues all of its (<= kDgMaxTpg) taps' loads at once and the chain is one round trip deep.
constexpr int kDgMaxTpg = 4;

// the split-tap body for block (bx, by): by = stride phase, bx = 16-pixel tile; part = LDS
// [8 waves][CT][64 lanes] f32x4; blockDim.x = 512 (8 waves: tap groups x channel halves)
template <int CT, int NN>
__device__ __forceinline__ void conv_dgrad_split_body(const bf16* __restrict__ dY, const bf16* __restrict__ Y,
                                                      const bf16* __restrict__ Wt, const bf16* __restrict__ Xp,
                                                      bf16* __restrict__ dZp, const ConvGeo& g, int relu_out, int relu_in,
                                                      int tpg, int bx, int by, f32x4 (*part)[CT][64]) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const int ph = by / g.S, pw = by - ph * g.S;
  const int Hc = (g.H - ph + g.S - 1) / g.S, Wc = (g.W - pw + g.S - 1) / g.S;
  const int HWc = Hc * Wc;
  const int P = g.B * HWc;
  const int p0 = bx * 16;
  if (p0 >= P) return;  // (block-uniform)
  const int Kp = g.KH * g.KW * g.N;
  const int r = l & 15, kq = (l >> 4) * 8;
  const int q0 = p0 + r;
  const bool pv = q0 < P;
  const int qq = pv ? q0 : P - 1;
  const int pb = qq / HWc;
  const int rem = qq - pb * HWc, ii = rem / Wc, jj = rem - ii * Wc;
  const int pih = ph + g.S * ii, piw = pw + g.S * jj;
  const int nkw = (g.KW - pw + g.S - 1) / g.S;
  const int ntap = ((g.KH - ph + g.S - 1) / g.S) * nkw;
  const int tg = w / NN, nn = w - (w / NN) * NN;
  const int t0 = tg * tpg, t1 = min(ntap, t0 + tpg);
  const bf16* wr = Wt + (size_t)r * Kp + kq + 32 * nn;
  f32x4 acc[CT];
#pragma unroll
  for (int t = 0; t < CT; ++t) acc[t] = zero4();
  bf16x8 av[kDgMaxTpg], bv[kDgMaxTpg][CT];
  bool any[kDgMaxTpg];
  // every tap's operand loads first (one round trip), then the MFMAs
#pragma unroll
  for (int u = 0; u < kDgMaxTpg; ++u) {
    const int tp = t0 + u;
    any[u] = false;
    if (tp < t1) {  // (wave-uniform)
      const int kh = ph + g.S * (tp / nkw), kw = pw + g.S * (tp - (tp / nkw) * nkw);
      const int th = pih + g.P - kh, tw = piw + g.P - kw;
      const int oh = th / g.S, ow = tw / g.S;
      const bool valid = pv && th >= 0 && oh < g.OH && tw >= 0 && ow < g.OW;
      any[u] = __ballot(valid) != 0ull;
      const size_t dzoff = valid ? ((size_t)(pb * g.OH + oh) * g.OW + ow) * g.N + kq + 32 * nn : 0;
      const int kbase = (kh * g.KW + kw) * g.N;
#pragma unroll
      for (int t = 0; t < CT; ++t) bv[u][t] = *reinterpret_cast<const bf16x8*>(wr + (size_t)t * 16 * Kp + kbase);
      av[u] = valid ? load_dz8(dY, Y, dzoff, relu_out) : zero8();
    }
  }
#pragma unroll
  for (int u = 0; u < kDgMaxTpg; ++u) {
    if (!any[u]) continue;  // (wave-uniform: past this wave's taps, or a tap missing every pixel)
#pragma unroll
    for (int t = 0; t < CT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[u], bv[u][t], acc[t], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < CT; ++t) part[w][t][l] = acc[t];
  __syncthreads();
  if (w != 0) return;
  // fixed wave order (tap groups, then channel halves) for every output element
#pragma unroll
  for (int t = 0; t < CT; ++t) {
    f32x4 s = part[0][t][l];
    for (int v = 1; v < nw; ++v) {
      const f32x4 x = part[v][t][l];
      s[0] += x[0];
      s[1] += x[1];
      s[2] += x[2];
      s[3] += x[3];
    }
    acc[t] = s;
  }
  const int col = l & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = p0 + 4 * (l >> 4) + i;
    if (q >= P) continue;
    const int bb = q / HWc;
    const int rr = q - bb * HWc, i2 = rr / Wc, j2 = rr - i2 * Wc;
    const size_t row = ((size_t)bb * g.H + (ph + g.S * i2)) * g.W + (pw + g.S * j2);
#pragma unroll
    for (int t = 0; t < CT; ++t) {
      const int c = t * 16 + col;
      float v = acc[t][i];
      if (relu_in && !((float)Xp[row * g.C + c] > 0.f)) v = 0.f;
      dZp[row * g.C + c] = (bf16)v;
    }
  }
}

// tap groups of the split-tap data gradient: 8 waves = (8 / NN) tap groups x NN channel halves;
// 0 when a phase would need more than kDgMaxTpg taps per group (then the prefetching form runs)
__host__ __device__ __forceinline__ int dgrad_split_tpg(const ConvGeo& g) {
  const int nn = g.N / 32;
  if (nn != 1 && nn != 2) return 0;
  const int ntap_max = ((g.KH + g.S - 1) / g.S) * ((g.KW + g.S - 1) / g.S);
  const int ts = 8 / nn;
  const int tpg = (ntap_max + ts - 1) / ts;
  return tpg <= kDgMaxTpg ? tpg : 0;
}

template <int CT, int NN>
__global__ __launch_bounds__(512) void conv_dgrad_split_kernel(const bf16* __restrict__ dY, const bf16* __restrict__ Y,
                                                               const bf16* __restrict__ Wt, const bf16* __restrict__ Xp,
                                                               bf16* __restrict__ dZp, ConvGeo g, int relu_out, int relu_in,
                                                               int tpg) {
  __shared__ f32x4 part[8][CT][64];  // [wave][channel tile][lane]
  conv_dgrad_split_body<CT, NN>(dY, Y, Wt, Xp, dZp, g, relu_out, relu_in, tpg, blockIdx.x, blockIdx.y, part);
}

// ------------------------------------------------------------------ weight gradient (partials)
// 512 threads; wave w owns output tiles t = w + 8 i (t = nt * KT + kt), TPW >= ceil(NT*KT/8).
// Each block reduces a contiguous m range in chunks of CH rows staged transposed in LDS
// (row stride CH + 8 bf16): the im2col rows as 8-k fragments, dZ as 8-channel fragments
// (one 16-byte load per (row, 8 channels)); every tile then runs CH/32 MFMA k-steps per
// chunk. CH = 128 for large M (4x the MFMA work per barrier pair and per load round trip),
// 32 for the small BC batches, where more blocks matter more.
template <typename TIn, int NT, int TPW, int CH>
__device__ __forceinline__ void conv_wgrad_body(const TIn* __restrict__ X, const bf16* __restrict__ dY,
                                                const bf16* __restrict__ Y, float* __restrict__ slab, const ConvGeo& g,
                                                float in_scale, int relu_out, int m_per_block, int blk, char* smem) {
  constexpr int LD = CH + 8;
  const int K = g.Kp;
  bf16* At = reinterpret_cast<bf16*>(smem);  // [K][LD]   im2col chunk, m contiguous
  bf16* Zt = At + (size_t)K * LD;            // [N][LD]   dZ chunk, m contiguous
  const int OHW = g.OH * g.OW;
  const int N = g.N;
  const int KT = K / 16;
  const int n_tiles = NT * KT;
  const int rowlen = g.KW * g.C;
  const size_t xrow = (size_t)g.W * g.C;
  const bool tap_checked = g.P > 0 || g.Kp != g.KH * g.KW * g.C;
  const int tid = threadIdx.x;
  const int w = tid >> 6, l = tid & 63;
  const int mb = blk * m_per_block;
  const int me = min(g.B * OHW, mb + m_per_block);
  f32x4 acc[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) acc[i] = zero4();
  float bsum = 0.f;  // bias partial of channel tid (tid < N)
  const int n_items = (K / 8) * CH;
  for (int c0 = mb; c0 < me; c0 += CH) {
    // im2col fragments (k-group kg, row ml), transposed; kWgBatch fragments per thread are
    // loaded before any is stored, so their round trips overlap (small-batch chunks: one batch)
    constexpr int kWgBatch = 8;
    for (int base = tid; base < n_items; base += 512 * kWgBatch) {
      bf16x8 v[kWgBatch];
#pragma unroll
      for (int u = 0; u < kWgBatch; ++u) {
        const int it = base + 512 * u;
        v[u] = zero8();
        if (it >= n_items) continue;
        const int ml = it % CH, kg = it / CH;
        const int m = c0 + ml;
        if (m < me) {
          const int b = m / OHW, pix = m - b * OHW, oh = pix / g.OW, ow = pix - oh * g.OW;
          if (tap_checked) {
            v[u] = load8_pad(X, g, b, oh, ow, kg * 8, true, in_scale);
          } else {
            const int k = kg * 8, kh = k / rowlen, off = k - kh * rowlen;
            v[u] = load8(X + ((size_t)(b * g.H + oh * g.S) * g.W + (size_t)ow * g.S) * g.C + kh * xrow + off, in_scale);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kWgBatch; ++u) {
        const int it = base + 512 * u;
        if (it >= n_items) continue;
        const int ml = it % CH, kg = it / CH;
#pragma unroll
        for (int j = 0; j < 8; ++j) At[(size_t)(kg * 8 + j) * LD + ml] = v[u][j];
      }
    }
    // dZ fragments (8 channels ng, row ml): dY * [Y > 0] when relu_out, transposed
    for (int it = tid; it < (N / 8) * CH; it += 512) {
      const int ml = it % CH, ng = it / CH;
      const int m = c0 + ml;
      bf16x8 z = zero8();
      if (m < me) z = load_dz8(dY, Y, (size_t)m * N + ng * 8, relu_out);
#pragma unroll
      for (int j = 0; j < 8; ++j) Zt[(ng * 8 + j) * LD + ml] = z[j];
    }
    __syncthreads();
    if (tid < N) {
      const bf16x8* zr = reinterpret_cast<const bf16x8*>(Zt + tid * LD);
#pragma unroll
      for (int q = 0; q < CH / 8; ++q) {
        const bf16x8 z = zr[q];
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum += (float)z[j];
      }
    }
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = w + 8 * i;
      if (t < n_tiles) {
        const int nt = t / KT, kt = t - nt * KT;
        const bf16* za = Zt + (nt * 16 + (l & 15)) * LD + (l >> 4) * 8;
        const bf16* xa = At + (size_t)(kt * 16 + (l & 15)) * LD + (l >> 4) * 8;
#pragma unroll
        for (int s = 0; s < CH / 32; ++s) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(za + s * 32);
          const bf16x8 bb = *reinterpret_cast<const bf16x8*>(xa + s * 32);
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bb, acc[i], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // partial dW [N][K] then db [N] of this block
  float* out = slab + (size_t)blk * ((size_t)N * K + N);
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = w + 8 * i;
    if (t < n_tiles) {
      const int nt = t / KT, kt = t - nt * KT;
      const int k = kt * 16 + (l & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) out[(size_t)(nt * 16 + 4 * (l >> 4) + q) * K + k] = acc[i][q];
    }
  }
  if (tid < N) out[(size_t)N * K + tid] = bsum;
}

template <typename TIn, int NT, int TPW, int CH>
__global__ __launch_bounds__(512) void conv_wgrad_kernel(const TIn* __restrict__ X, const bf16* __restrict__ dY,
                                                         const bf16* __restrict__ Y, float* __restrict__ slab, ConvGeo g,
                                                         float in_scale, int relu_out, int m_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_wgrad_body<TIn, NT, TPW, CH>(X, dY, Y, slab, g, in_scale, relu_out, m_per_block, blockIdx.x, smem);
}

// One layer's two independent backward products in ONE launch (the BC step's conv2 / conv3): blocks
// [0, n_wg) are the weight-gradient partials (conv_wgrad_body), the rest the split-tap data
// gradient (conv_dgrad_split_body, block b -> tile b % dg_gx, phase b / dg_gx). Both read the same
// dY / Y; neither feeds the other, so the launch's critical path is the longer of the two instead
// of their sum plus a dispatch.
// RT: 16-pixel data-gradient tiles per block, one after another (LDS partials reused after a
// barrier; the same per-tile arithmetic, so the same bits whatever RT).
template <int NT, int TPW, int CH, int CT, int NN, int RT>
__global__ __launch_bounds__(512) void conv_back_pair_kernel(const bf16* __restrict__ X, const bf16* __restrict__ dY,
                                                             const bf16* __restrict__ Y, float* __restrict__ slab,
                                                             ConvGeo g, int relu_out, int m_per_block, int n_wg,
                                                             const bf16* __restrict__ Wt, bf16* __restrict__ dZp,
                                                             int relu_in, int tpg, int dg_gx) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  if (b < n_wg) {
    conv_wgrad_body<bf16, NT, TPW, CH>(X, dY, Y, slab, g, 1.f, relu_out, m_per_block, b, smem);
  } else {
    const int d = b - n_wg;
#pragma unroll 1
    for (int k = 0; k < RT; ++k) {
      // (waves 1..7 leave the body after its barrier; wave 0 after the tile's stores)
      conv_dgrad_split_body<CT, NN>(dY, Y, Wt, X, dZp, g, relu_out, relu_in, tpg, (d % dg_gx) * RT + k, d / dg_gx,
                                    reinterpret_cast<f32x4(*)[CT][64]>(smem));
      if (RT > 1) __syncthreads();  // wave 0's reads of the partials before the next tile's writes
    }
  }
}

// Fixed-order sum of the wgrad block partials: 4 independent accumulators (blocks b with
// b % 4 == j) keep 4 loads in flight per thread, combined in a fixed order at the end.
// The weight gradient is written in torch's [N][C][KH][KW] layout (GEMM column k = (kh, kw, c),
// columns past K = KH*KW*C are the zero padding of Kp and dropped), so no permute copy follows.
__global__ __launch_bounds__(256) void conv_reduce_kernel(const float* __restrict__ slab, int nblk, int len,
                                                          float* __restrict__ dW, float* __restrict__ db, int nk,
                                                          ConvGeo g) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= len) return;
  (void)nk;
  int wi, bi;
  const float s = slab_column(slab, nblk, g, i, &wi, &bi);
  if (wi >= 0) dW[wi] = s;
  else if (bi >= 0 && db) db[bi] = s;
}

template <typename TIn>
hipError_t launch_fwd(const TIn* X, const bf16* Wb, const float* bias, bf16* Y, const ConvGeo& g, float scale, int relu,
                      hipStream_t s) {
  const int M = g.B * g.OH * g.OW;
  const dim3 block(256);
  if (M >= (1 << 16)) {  // large M: 4 row tiles per wave
    const dim3 grid((M + 255) / 256);
    const bool pad = g.P > 0 || g.Kp != g.KH * g.KW * g.C;
#define IA_FWD4(NT)                                                                                                   \
  if (pad) hipLaunchKernelGGL((conv_fwd_kernel<TIn, NT, true, 4>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu); \
  else hipLaunchKernelGGL((conv_fwd_kernel<TIn, NT, false, 4>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu)
    switch (g.N / 16) {
      case 1: IA_FWD4(1); break;
      case 2: IA_FWD4(2); break;
      case 4: IA_FWD4(4); break;
      default: return hipErrorInvalidValue;
    }
#undef IA_FWD4
    return hipGetLastError();
  }
  if (g.P > 0 || g.Kp != g.KH * g.KW * g.C) {
    const dim3 grid((M + 63) / 64);
    switch (g.N / 16) {
      case 1: hipLaunchKernelGGL((conv_fwd_kernel<TIn, 1, true>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu); break;
      case 2: hipLaunchKernelGGL((conv_fwd_kernel<TIn, 2, true>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu); break;
      case 4: hipLaunchKernelGGL((conv_fwd_kernel<TIn, 4, true>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if ((M + 63) / 64 < 96) {
    // small batches (policy inference): one 16-channel slice per block row, so the grid has
    // N/16 x as many waves to hide the operand-load latency of the K loop
    const dim3 grid((M + 63) / 64, g.N / 16);
    hipLaunchKernelGGL((conv_fwd_kernel<TIn, 1>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu);
    return hipGetLastError();
  }
  const dim3 grid((M + 63) / 64);
  switch (g.N / 16) {
    case 1: hipLaunchKernelGGL((conv_fwd_kernel<TIn, 1>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu); break;
    case 2: hipLaunchKernelGGL((conv_fwd_kernel<TIn, 2>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu); break;
    case 4: hipLaunchKernelGGL((conv_fwd_kernel<TIn, 4>), grid, block, 0, s, X, Wb, bias, Y, g, scale, relu); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename TIn, int NT, int CH>
hipError_t launch_wgrad_ch(const TIn* X, const bf16* dY, const bf16* Y, float* slab, const ConvGeo& g, float scale,
                           int relu_out, int nblk, int mpb, hipStream_t s) {
  const int K = g.Kp;
  const int tiles = NT * (K / 16);
  const size_t lds = ((size_t)K + (size_t)g.N) * (CH + 8) * sizeof(bf16);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int tpw = (tiles + 7) / 8;
  const dim3 grid(nblk), block(512);
  if (tpw <= 4)
    hipLaunchKernelGGL((conv_wgrad_kernel<TIn, NT, 4, CH>), grid, block, lds, s, X, dY, Y, slab, g, scale, relu_out, mpb);
  else if (tpw <= 8)
    hipLaunchKernelGGL((conv_wgrad_kernel<TIn, NT, 8, CH>), grid, block, lds, s, X, dY, Y, slab, g, scale, relu_out, mpb);
  else if (tpw <= 12)
    hipLaunchKernelGGL((conv_wgrad_kernel<TIn, NT, 12, CH>), grid, block, lds, s, X, dY, Y, slab, g, scale, relu_out, mpb);
  else if (tpw <= 18)
    hipLaunchKernelGGL((conv_wgrad_kernel<TIn, NT, 18, CH>), grid, block, lds, s, X, dY, Y, slab, g, scale, relu_out, mpb);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <typename TIn, int NT>
hipError_t launch_wgrad_nt(const TIn* X, const bf16* dY, const bf16* Y, float* slab, const ConvGeo& g, float scale,
                           int relu_out, int nblk, int mpb, hipStream_t s) {
  switch (wgrad_chunk(g)) {
    case 128: return launch_wgrad_ch<TIn, NT, 128>(X, dY, Y, slab, g, scale, relu_out, nblk, mpb, s);
    case 64: return launch_wgrad_ch<TIn, NT, 64>(X, dY, Y, slab, g, scale, relu_out, nblk, mpb, s);
    default: return launch_wgrad_ch<TIn, NT, 32>(X, dY, Y, slab, g, scale, relu_out, nblk, mpb, s);
  }
}

template <typename TIn>
hipError_t launch_wgrad(const TIn* X, const bf16* dY, const bf16* Y, float* slab, float* dW, float* db, const ConvGeo& g,
                        float scale, int relu_out, hipStream_t s) {
  const int M = g.B * g.OH * g.OW;
  int nblk = 0, mpb = 0;
  conv_wgrad_blocks(g, &nblk, &mpb);
  hipError_t e;
  switch (g.N / 16) {
    case 1: e = launch_wgrad_nt<TIn, 1>(X, dY, Y, slab, g, scale, relu_out, nblk, mpb, s); break;
    case 2: e = launch_wgrad_nt<TIn, 2>(X, dY, Y, slab, g, scale, relu_out, nblk, mpb, s); break;
    case 4: e = launch_wgrad_nt<TIn, 4>(X, dY, Y, slab, g, scale, relu_out, nblk, mpb, s); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  (void)M;
  if (!dW) return hipSuccess;  // reduction deferred to conv_reduce_multi
  const int K = g.Kp;
  const int len = g.N * K + g.N;
  hipLaunchKernelGGL(conv_reduce_kernel, dim3((len + 255) / 256), dim3(256), 0, s, slab, nblk, len, dW, db, g.N * K, g);
  return hipGetLastError();
}

// the deferred reductions of several layers' wgrad slabs in one launch (blockIdx.y = layer)
__global__ __launch_bounds__(256) void conv_reduce_multi_kernel(ConvReduceMulti r) {
  const int l = blockIdx.y;
  const ConvGeo& g = r.g[l];
  const int len = g.N * g.Kp + g.N;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= len) return;
  // (same fixed-order sum as conv_reduce_kernel, and as the Adam launch that folds it: optim.hip)
  int wi, bi;
  const float s = slab_column(r.slab[l], r.nblk[l], g, i, &wi, &bi);
  if (wi >= 0) r.dW[l][wi] = s;
  else if (bi >= 0 && r.db[l]) r.db[l][bi] = s;
}

// fp32 torch-layout conv weights [N][C][KH][KW] of up to kMaxPack layers -> bf16 [N][KH][KW][C]
// (forward GEMM operand) and, where requested, the data-gradient operand: bf16 [C][KH][KW][N]
// (a 2-D transpose of the source viewed [N][C*KH*KW]) or, t_hwc, [KH][KW][C][N] (a 2-D
// transpose of the packed [N][KH*KW*C], read straight from the fp32 source: bf16 of the same
// value). Both passes are 32x32 LDS-tile transposes in ONE launch (the per-step weight refresh
// of the fused BC step: two launches were ~12.5 us of its ~145): blocks [0, nwb) the forward
// images (tile, output channel, layer), the rest the transposes (k tile, n tile, layer).
__device__ __forceinline__ void pack_wb_tile(const ConvPackLayer& L, int tile, int n, float (*t)[33]) {
  const int taps = L.KH * L.KW, C = L.C;
  const int tt = (taps + 31) / 32, nc = (C + 31) / 32;
  if (n >= L.N || tile >= tt * nc) return;
  const int c0 = (tile / tt) * 32, p0 = (tile % tt) * 32;
  const float* src = L.w + (size_t)n * C * taps;
  for (int i = threadIdx.x; i < 1024; i += 256) {  // src [c][tap], coalesced along tap
    const int r = i >> 5, q = i & 31, c = c0 + r, p = p0 + q;
    t[r][q] = (c < C && p < taps) ? src[(size_t)c * taps + p] : 0.f;
  }
  __syncthreads();
  bf16* dst = static_cast<bf16*>(L.wb) + (size_t)n * taps * C;
  for (int i = threadIdx.x; i < 1024; i += 256) {  // dst [tap][c], coalesced along c
    const int r = i >> 5, q = i & 31, p = p0 + r, c = c0 + q;
    if (p < taps && c < C) dst[(size_t)p * C + c] = (bf16)t[q][r];
  }
}

__device__ __forceinline__ void pack_wt_tile(const ConvPackLayer& L, int kt, int nt, float (*t)[33]) {
  if (!L.wt) return;
  const int taps = L.KH * L.KW, K = L.C * taps, N = L.N;
  const int n0 = nt * 32;
  if (n0 >= N) return;
  bf16* dst = static_cast<bf16*>(L.wt);
  if (!L.t_hwc) {
    // [C*KH*KW][N] = the source viewed [N][K], transposed: tiles of 32 k x 32 n
    const int k0 = kt * 32;
    if (k0 >= K) return;
    for (int i = threadIdx.x; i < 1024; i += 256) {  // [n][k] rows, coalesced along k
      const int r = i >> 5, q = i & 31, nn = n0 + r, k = k0 + q;
      t[r][q] = (nn < N && k < K) ? L.w[(size_t)nn * K + k] : 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 256) {  // [k][n], coalesced along n
      const int r = i >> 5, q = i & 31, k = k0 + r, nn = n0 + q;
      if (k < K && nn < N) dst[(size_t)k * N + nn] = (bf16)t[q][r];
    }
  } else {
    // [KH*KW][C][N]: per channel c a 32 tap x 32 n tile of source rows w[n][c][tap], coalesced
    // along tap on the read and along n on the write (a k tile of the packed row would read
    // 32 channels of one tap, one 4-B element per source line)
    const int ttl = (taps + 31) / 32, c = kt / ttl, p0 = (kt - c * ttl) * 32;
    if (c >= L.C) return;
    for (int i = threadIdx.x; i < 1024; i += 256) {  // [n][tap]
      const int r = i >> 5, q = i & 31, nn = n0 + r, p = p0 + q;
      t[r][q] = (nn < N && p < taps) ? L.w[((size_t)nn * L.C + c) * taps + p] : 0.f;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 256) {  // [tap][c][n]
      const int r = i >> 5, q = i & 31, p = p0 + r, nn = n0 + q;
      if (p < taps && nn < N) dst[((size_t)p * L.C + c) * N + nn] = (bf16)t[q][r];
    }
  }
}

// Row form (layers whose C x KH*KW fits one LDS image, e.g. all of NatureCNN): one block per
// output channel n transposes the whole [C][taps] row to [taps][C] (the FC: 3136 elements, 12
// loads per thread in flight), and the t_hwc transpose runs one block per (channel, 64 n): 64
// source rows of `taps` floats -> taps rows of 64 bf16. ~1250 blocks for the NatureCNN step
// instead of ~4400 32x32 tiles (each a load -> barrier -> store round trip). The LDS row stride
// is odd (taps | 1), so the column-order reads are bank-conflict free.
constexpr int kPackRowLds = 4224;  // floats: C * stride (forward image) or 64 * stride (t_hwc)
constexpr int kPackRowIt = 17;     // loads per thread: ceil(4224 / 256)

__device__ __forceinline__ int pack_stride(int taps) { return taps | 1; }

__device__ __forceinline__ void pack_wb_row(const ConvPackLayer& L, int n, float* t) {
  const int taps = L.KH * L.KW, C = L.C, K = C * taps, st = pack_stride(taps);
  const float* src = L.w + (size_t)n * K;
  float v[kPackRowIt];
#pragma unroll
  for (int u = 0; u < kPackRowIt; ++u) {  // all loads in flight before the LDS stores
    const int i = threadIdx.x + 256 * u;
    v[u] = i < K ? src[i] : 0.f;
  }
  // (integer divisions by runtime taps / C are ~40 VALU each: skipped where the layout allows --
  // odd taps (st == taps: the LDS index is i itself), power-of-two C (a shift))
  const bool odd = st == taps;
#pragma unroll
  for (int u = 0; u < kPackRowIt; ++u) {  // src [c][tap] -> t[c * st + tap]
    const int i = threadIdx.x + 256 * u;
    if (i < K) {
      if (odd) {
        t[i] = v[u];
      } else {
        const int c = i / taps;
        t[c * st + i - c * taps] = v[u];
      }
    }
  }
  __syncthreads();
  bf16* dst = static_cast<bf16*>(L.wb) + (size_t)n * K;
  if ((C & (C - 1)) == 0) {
    const int sh = __builtin_ctz(C);
    for (int i = threadIdx.x; i < K; i += 256) {  // dst [tap][c], coalesced along c
      const int p = i >> sh, c = i & (C - 1);
      dst[i] = (bf16)t[c * st + p];
    }
  } else {
    for (int i = threadIdx.x; i < K; i += 256) {
      const int p = i / C, c = i - p * C;
      dst[i] = (bf16)t[c * st + p];
    }
  }
}

__device__ __forceinline__ void pack_wt_row(const ConvPackLayer& L, int c, int nt, float* t) {
  const int taps = L.KH * L.KW, C = L.C, N = L.N, st = pack_stride(taps), n0 = nt * 64;
  const int cnt = 64 * taps;
  float v[kPackRowIt];
  const bool odd = st == taps;
  int nls[kPackRowIt];
#pragma unroll
  for (int u = 0; u < kPackRowIt; ++u) {  // 64 source rows w[n][c][0..taps)
    const int i = threadIdx.x + 256 * u;
    const int nl = i / taps, p = i - nl * taps;
    nls[u] = nl;
    v[u] = (i < cnt && n0 + nl < N) ? L.w[((size_t)(n0 + nl) * C + c) * taps + p] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kPackRowIt; ++u) {
    const int i = threadIdx.x + 256 * u;
    if (i < cnt) t[odd ? i : nls[u] * st + i - nls[u] * taps] = v[u];
  }
  __syncthreads();
  bf16* dst = static_cast<bf16*>(L.wt);
  for (int i = threadIdx.x; i < cnt; i += 256) {  // dst [tap][c][n0 .. n0 + 64), coalesced along n
    const int p = i >> 6, nl = i & 63;
    if (n0 + nl < N) dst[((size_t)p * C + c) * N + n0 + nl] = (bf16)t[nl * st + p];
  }
}

// Block ranges of one pack launch: per layer its forward-image tiles (tiles x N; row form: N)
// then, after all of those, its transpose tiles (kts x nts) -- exact counts, no idle blocks.
struct PackPlan {
  int off[2 * kMaxPack + 1];  // block offsets: [0, n) forward images, [n, 2n) transposes
  int tiles[kMaxPack], kts[kMaxPack];
  int row[kMaxPack];  // forward image in row form; t_hwc transpose in row form
};

// Blocks past the packing ranges: the BC step's minibatch gather (gather_body.h), ga.k fields x gx
// blocks -- independent of the packing, so it rides on this launch instead of a dispatch of its own.
__global__ __launch_bounds__(256) void conv_pack_kernel(ConvPackArgs a, PackPlan pl, GatherArgs ga, const int* perm,
                                                        const int* cursor, int gn, float* inc, int gx) {
  __shared__ float t[kPackRowLds];
  const int b = blockIdx.x;
  if (b >= pl.off[2 * a.n]) {
    const int r = b - pl.off[2 * a.n];
    gather_rows_cursor_block(ga, perm, cursor, gn, inc, r % gx, r / gx, gx);
    return;
  }
  int j = 0;
  while (j + 1 < 2 * a.n && b >= pl.off[j + 1]) ++j;  // (uniform)
  const int r = b - pl.off[j];
  float(*t32)[33] = reinterpret_cast<float(*)[33]>(t);
  if (j < a.n) {
    if (pl.row[j]) pack_wb_row(a.layer[j], r, t);
    else pack_wb_tile(a.layer[j], r % pl.tiles[j], r / pl.tiles[j], t32);
  } else {
    const int l = j - a.n;
    if (pl.row[l] && a.layer[l].t_hwc) pack_wt_row(a.layer[l], r % pl.kts[l], r / pl.kts[l], t);
    else pack_wt_tile(a.layer[l], r % pl.kts[l], r / pl.kts[l], t32);
  }
}

}  // namespace

hipError_t conv_pack_weights(const ConvPackArgs& a, hipStream_t s, const GatherArgs* ga, const int* perm, const int* cursor,
                             int gn, float* inc) {
  if (a.n <= 0) return hipSuccess;
  if (a.n > kMaxPack) return hipErrorInvalidValue;
  const bool gather = ga != nullptr && ga->k > 0 && gn > 0;
  if (gather && ga->k > kGatherMax) return hipErrorInvalidValue;
  PackPlan pl{};
  int total = 0;
  for (int i = 0; i < a.n; ++i) {  // forward images: (channel x tap) tiles per output channel, or rows
    const ConvPackLayer& L = a.layer[i];
    const int taps = L.KH * L.KW, st = taps | 1;
    pl.row[i] = L.C * st <= kPackRowLds && taps <= 64;  // (t_hwc row form: 64 x st floats)
    pl.tiles[i] = pl.row[i] ? 1 : ((taps + 31) / 32) * ((L.C + 31) / 32);
    pl.off[i] = total;
    total += pl.tiles[i] * L.N;
  }
  for (int i = 0; i < a.n; ++i) {  // transposes: k tiles (or channel x 32-tap tiles, t_hwc) x n tiles
    const ConvPackLayer& L = a.layer[i];
    const int taps = L.KH * L.KW;
    const bool row = pl.row[i] && L.t_hwc;  // one block per (channel, 64 n)
    pl.kts[i] = row ? L.C : L.t_hwc ? L.C * ((taps + 31) / 32) : (L.C * taps + 31) / 32;
    pl.off[a.n + i] = total;
    if (L.wt) total += pl.kts[i] * (row ? (L.N + 63) / 64 : (L.N + 31) / 32);
  }
  pl.off[2 * a.n] = total;
  const GatherArgs none{};
  const int gx = gather ? gather_cursor_blocks(*ga, gn) : 1;
  const int blocks = total + (gather ? gx * ga->k : 0);
  hipLaunchKernelGGL(conv_pack_kernel, dim3(blocks), dim3(256), 0, s, a, pl, gather ? *ga : none, perm, cursor, gn, inc, gx);
  return hipGetLastError();
}

hipError_t conv_fwd_pair(int in_kind, const ConvPair& p, const ConvGeo& g, float in_scale, int relu, hipStream_t s) {
  if (!conv_geo_ok(g) || g.P != 0 || g.Kp != g.KH * g.KW * g.C || g.N % 16 != 0) return hipErrorInvalidValue;
  const int M = g.B * g.OH * g.OW;
  const dim3 grid((M + 63) / 64, g.N / 16, 2), block(256);
  if (in_kind == 1)
    hipLaunchKernelGGL(conv_fwd_pair_kernel<bf16>, grid, block, 0, s, p, g, in_scale, relu);
  else if (in_kind == 2)
    hipLaunchKernelGGL(conv_fwd_pair_kernel<uint8_t>, grid, block, 0, s, p, g, in_scale, relu);
  else
    hipLaunchKernelGGL(conv_fwd_pair_kernel<float>, grid, block, 0, s, p, g, in_scale, relu);
  return hipGetLastError();
}

bool conv_geo_ok(const ConvGeo& g) {
  const int K = g.KH * g.KW * g.C;
  if (g.B <= 0 || g.OH <= 0 || g.OW <= 0 || g.P < 0) return false;
  if ((g.OH - 1) * g.S + g.KH > g.H + 2 * g.P || (g.OW - 1) * g.S + g.KW > g.W + 2 * g.P) return false;
  if (g.Kp != ((K + 31) & ~31)) return false;
  if (g.P > 0 || g.Kp != K) {  // tap-checked path
    if (g.C % 8 != 0 || g.S != 1) return false;
  } else if ((g.KW * g.C) % 8 != 0) {
    return false;
  }
  if (g.N % 16 != 0 || g.N > 64) return false;
  return true;
}

void conv_wgrad_blocks(const ConvGeo& g, int* nblk, int* mpb) {
  const int M = g.B * g.OH * g.OW;
  const int CH = wgrad_chunk(g);
  const int chunks = (M + CH - 1) / CH;
  const int K = g.Kp;
  // fp32 partial traffic (nblk x N x K, written then re-read by conv_reduce) vs parallelism:
  // small layers (BC batches) ~2M partial floats at most (the 256-block cap moved 24 MB per
  // NatureCNN BC step; 1M -> 2M: BC step 0.145 -> 0.140 ms, 4M 0.141, profiles/r6_bc_step.md);
  // large ones (>= 64K rows, e.g. full-resolution reward CNN batches, where the m loop is the
  // cost) up to 8M floats and 512 blocks -- 2 per CU
  const int len = g.N * K + g.N;
  const bool big = CH > 32;
  int cap = (big ? (8 << 20) : (2 << 20)) / len;
  const int hi = big ? 512 : 256;
  cap = cap < 16 ? 16 : (cap > hi ? hi : cap);
  int b = chunks < cap ? chunks : cap;
  const int cpb = (chunks + b - 1) / b;
  b = (chunks + cpb - 1) / cpb;
  *nblk = b;
  *mpb = cpb * CH;
}

hipError_t conv_reduce_multi(const ConvReduceMulti& r, hipStream_t s) {
  if (r.n <= 0) return hipSuccess;
  if (r.n > kMaxPack) return hipErrorInvalidValue;
  ConvReduceMulti rr = r;
  int maxlen = 0;
  for (int l = 0; l < r.n; ++l) {
    int mpb = 0;
    conv_wgrad_blocks(r.g[l], &rr.nblk[l], &mpb);
    const int len = r.g[l].N * r.g[l].Kp + r.g[l].N;
    maxlen = len > maxlen ? len : maxlen;
  }
  hipLaunchKernelGGL(conv_reduce_multi_kernel, dim3((maxlen + 255) / 256, r.n), dim3(256), 0, s, rr);
  return hipGetLastError();
}

size_t conv_wgrad_slab_floats(const ConvGeo& g) {
  int nblk = 0, mpb = 0;
  conv_wgrad_blocks(g, &nblk, &mpb);
  const int K = g.Kp;
  return (size_t)nblk * ((size_t)g.N * K + g.N);
}

hipError_t conv_forward(int in_kind, const void* X, const void* Wb, const float* bias, void* Y, const ConvGeo& g,
                        float in_scale, int relu, hipStream_t s) {
  if (!conv_geo_ok(g)) return hipErrorInvalidValue;
  const bf16* w = static_cast<const bf16*>(Wb);
  bf16* y = static_cast<bf16*>(Y);
  switch (in_kind) {
    case 0: return launch_fwd(static_cast<const float*>(X), w, bias, y, g, in_scale, relu, s);
    case 1: return launch_fwd(static_cast<const bf16*>(X), w, bias, y, g, in_scale, relu, s);
    case 2: return launch_fwd(static_cast<const uint8_t*>(X), w, bias, y, g, in_scale, relu, s);
    default: return hipErrorInvalidValue;
  }
}

bool conv_forward_sk_ok(const ConvGeo& g) {
  const int steps = g.Kp / 32;
  return conv_geo_ok(g) && g.P == 0 && g.Kp == g.KH * g.KW * g.C && g.Kp % 32 == 0 && g.N % 16 == 0 && steps >= 2 &&
         steps <= 4 * kSkMaxSteps;
}

hipError_t conv_forward_sk(int in_kind, const void* X, const void* Wb, const float* bias, void* Y, const ConvGeo& g,
                           float in_scale, int relu, hipStream_t s) {
  if (!conv_forward_sk_ok(g)) return hipErrorInvalidValue;
  const int M = g.B * g.OH * g.OW, steps = g.Kp / 32;
  const dim3 grid((M + 15) / 16, g.N / 16);
  const bf16* w = static_cast<const bf16*>(Wb);
  bf16* y = static_cast<bf16*>(Y);
  // 2 waves per tile up to 16 k-steps (<= 8 each), else 4
#define IA_SK(T, KS) \
  hipLaunchKernelGGL((conv_fwd_sk_kernel<T, KS>), grid, dim3(64 * KS), 0, s, static_cast<const T*>(X), w, bias, y, g, in_scale, relu)
#define IA_SK_K(T) \
  if (steps <= 8) IA_SK(T, 2); else IA_SK(T, 4)
  switch (in_kind) {
    case 0: IA_SK_K(float); break;
    case 1: IA_SK_K(bf16); break;
    case 2: IA_SK_K(uint8_t); break;
    default: return hipErrorInvalidValue;
  }
#undef IA_SK_K
#undef IA_SK
  return hipGetLastError();
}

hipError_t conv_wgrad(int in_kind, const void* X, const void* dY, const void* Y, float* slab, float* dW, float* db,
                      const ConvGeo& g, float in_scale, int relu_out, hipStream_t s) {
  if (!conv_geo_ok(g)) return hipErrorInvalidValue;
  const bf16* dy = static_cast<const bf16*>(dY);
  const bf16* y = static_cast<const bf16*>(Y);
  switch (in_kind) {
    case 0: return launch_wgrad(static_cast<const float*>(X), dy, y, slab, dW, db, g, in_scale, relu_out, s);
    case 1: return launch_wgrad(static_cast<const bf16*>(X), dy, y, slab, dW, db, g, in_scale, relu_out, s);
    case 2: return launch_wgrad(static_cast<const uint8_t*>(X), dy, y, slab, dW, db, g, in_scale, relu_out, s);
    default: return hipErrorInvalidValue;
  }
}

// compute units of the current device (cached; BC-size launch shapes are sized against it)
static int cu_count() {
  static int n = 0;
  if (n <= 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      n = v;
    if (n <= 0) n = 256;
  }
  return n;
}

bool conv_back_pair_ok(const ConvGeo& g) {
  if (!conv_geo_ok(g) || g.N % 32 != 0 || g.C % 16 != 0 || g.C > 64 || g.P != 0) return false;
  const int Hc = (g.H + g.S - 1) / g.S, Wc = (g.W + g.S - 1) / g.S;
  if (g.B * Hc * Wc >= (1 << 16) || dgrad_split_tpg(g) == 0) return false;  // small batches only
  if (wgrad_chunk(g) != 32) return false;
  const int tiles = (g.N / 16) * (g.Kp / 16);
  return (tiles + 7) / 8 <= 18;
}

hipError_t conv_back_pair(const void* X, const void* dY, const void* Y, float* slab, const void* Wt, void* dZp,
                          const ConvGeo& g, int relu_out, int relu_in, hipStream_t s) {
  if (!conv_back_pair_ok(g)) return hipErrorInvalidValue;
  int nblk = 0, mpb = 0;
  conv_wgrad_blocks(g, &nblk, &mpb);
  const int tpg = dgrad_split_tpg(g);
  const int Hc = (g.H + g.S - 1) / g.S, Wc = (g.W + g.S - 1) / g.S;
  // The kernel's VGPR budget is the weight-gradient body's (~240: one 512-thread block per CU), so
  // its short data-gradient blocks run ~one per CU. When the launch would need more than one round
  // of blocks (conv2 at batch 32: 41 + 800), each data-gradient block takes 4 tiles: 41 + 200.
  const int tiles16 = (g.B * Hc * Wc + 15) / 16;
  const int rt = nblk + tiles16 * g.S * g.S > cu_count() ? 4 : 1;
  const int gx = (tiles16 + rt - 1) / rt;
  const int n_dg = gx * g.S * g.S;
  constexpr int CH = 32;
  const size_t lds_wg = ((size_t)g.Kp + (size_t)g.N) * (CH + 8) * sizeof(bf16);
  const size_t lds_dg = (size_t)8 * (g.C / 16) * 64 * sizeof(f32x4);
  const size_t lds = lds_wg > lds_dg ? lds_wg : lds_dg;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int tpw = ((g.N / 16) * (g.Kp / 16) + 7) / 8;
  const bf16* x = static_cast<const bf16*>(X);
  const bf16* dy = static_cast<const bf16*>(dY);
  const bf16* y = static_cast<const bf16*>(Y);
  const bf16* wt = static_cast<const bf16*>(Wt);
  bf16* dz = static_cast<bf16*>(dZp);
  const dim3 grid(nblk + n_dg), block(512);
  const int nn = g.N / 32;
#define IA_BP(NT, TPW, CT, NN)                                                                                                 \
  do {                                                                                                                         \
    if (rt == 4)                                                                                                               \
      hipLaunchKernelGGL((conv_back_pair_kernel<NT, TPW, CH, CT, NN, 4>), grid, block, lds, s, x, dy, y, slab, g, relu_out, mpb, \
                         nblk, wt, dz, relu_in, tpg, gx);                                                                      \
    else                                                                                                                       \
      hipLaunchKernelGGL((conv_back_pair_kernel<NT, TPW, CH, CT, NN, 1>), grid, block, lds, s, x, dy, y, slab, g, relu_out, mpb, \
                         nblk, wt, dz, relu_in, tpg, gx);                                                                      \
  } while (0)
#define IA_BP_T(NT, CT, NN)         \
  if (tpw <= 4) IA_BP(NT, 4, CT, NN);      \
  else if (tpw <= 8) IA_BP(NT, 8, CT, NN); \
  else if (tpw <= 12) IA_BP(NT, 12, CT, NN); \
  else IA_BP(NT, 18, CT, NN)
  // NT = N / 16 (wgrad output tiles), CT = C / 16 (dgrad output tiles), NN = N / 32
  if (nn == 2 && g.C == 64) { IA_BP_T(4, 4, 2); }
  else if (nn == 2 && g.C == 32) { IA_BP_T(4, 2, 2); }
  else if (nn == 2 && g.C == 16) { IA_BP_T(4, 1, 2); }
  else if (nn == 1 && g.C == 64) { IA_BP_T(2, 4, 1); }
  else if (nn == 1 && g.C == 32) { IA_BP_T(2, 2, 1); }
  else if (nn == 1 && g.C == 16) { IA_BP_T(2, 1, 1); }
  else return hipErrorInvalidValue;
#undef IA_BP_T
#undef IA_BP
  return hipGetLastError();
}

hipError_t conv_dgrad(const void* dY, const void* Y, const void* Wt, const void* Xp, void* dZp, const ConvGeo& g,
                      int relu_out, int relu_in, hipStream_t s, int form) {
  if (!conv_geo_ok(g) || g.N % 32 != 0 || g.C % 16 != 0 || g.C > 64) return hipErrorInvalidValue;
  const int Hc = (g.H + g.S - 1) / g.S, Wc = (g.W + g.S - 1) / g.S;  // largest phase
  const int P = g.B * Hc * Wc;
  const bool big = P >= (1 << 16);  // large M: 4 pixel tiles per wave share the weight fragments
  const dim3 grid(big ? (P + 255) / 256 : (P + 63) / 64, g.S * g.S), block(256);
  const bf16* dy = static_cast<const bf16*>(dY);
  const bf16* y = static_cast<const bf16*>(Y);
  const bf16* wt = static_cast<const bf16*>(Wt);
  const bf16* xp = static_cast<const bf16*>(Xp);
  bf16* dz = static_cast<bf16*>(dZp);
  // small batches, N = 32 / 64: the split-tap form (one tile per block, its taps and channel
  // halves over waves), else the prefetching one-wave-per-tile form; `form` forces the
  // prefetching form or the plain loop (the bitwise / fp32 checks of tests/ops/test_conv.py)
  const int nn = g.N / 32;
  const bool small = !big && (nn == 1 || nn == 2);
  if (form != kDgradAuto && !small) return hipErrorInvalidValue;
  const bool pf = small && form != kDgradPlain;
  const int tpg = dgrad_split_tpg(g);  // (8 waves: the same tap grouping as conv_back_pair)
  if (form == kDgradSplit && tpg <= 0) return hipErrorInvalidValue;
  const bool split = pf && tpg > 0 && form != kDgradPrefetch;
  const dim3 sgrid((P + 15) / 16, g.S * g.S), sblock(512);
#define IA_DG(CT)                                                                                                         \
  if (big) hipLaunchKernelGGL((conv_dgrad_kernel<CT, 4>), grid, block, 0, s, dy, y, wt, xp, dz, g, relu_out, relu_in);     \
  else if (split && nn == 2) hipLaunchKernelGGL((conv_dgrad_split_kernel<CT, 2>), sgrid, sblock, 0, s, dy, y, wt, xp, dz, g, relu_out, relu_in, tpg); \
  else if (split) hipLaunchKernelGGL((conv_dgrad_split_kernel<CT, 1>), sgrid, sblock, 0, s, dy, y, wt, xp, dz, g, relu_out, relu_in, tpg); \
  else if (pf && nn == 2) hipLaunchKernelGGL((conv_dgrad_pf_kernel<CT, 2>), grid, block, 0, s, dy, y, wt, xp, dz, g, relu_out, relu_in); \
  else if (pf) hipLaunchKernelGGL((conv_dgrad_pf_kernel<CT, 1>), grid, block, 0, s, dy, y, wt, xp, dz, g, relu_out, relu_in); \
  else hipLaunchKernelGGL((conv_dgrad_kernel<CT, 1>), grid, block, 0, s, dy, y, wt, xp, dz, g, relu_out, relu_in)
  switch (g.C / 16) {
    case 1: IA_DG(1); break;
    case 2: IA_DG(2); break;
    case 4: IA_DG(4); break;
    default: return hipErrorInvalidValue;
  }
#undef IA_DG
  return hipGetLastError();
}

}  // namespace ia

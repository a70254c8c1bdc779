// Register-chained PPO update: host planning, the parallel prep kernel and the launch of the
// shape-specialised kernel instance (kernel template: ppo_rc_kernel.h; instances compiled in
// ppo_rc_inst*.hip, declared extern below).
#include <stdio.h>

#include "ppo_rc_kernel.h"
#include "ppo_rc_instances.h"

namespace ia {
namespace rc {

IA_RC_INSTANCES(IA_RC_EXTERN)

// ---------------------------------------------------------------- prep (parallel over minibatches)
// One workgroup per minibatch k = epoch * n_mb + mb, one wave per chunk (looping when the
// minibatch has more chunks than waves), one lane per row. Minibatch statistics (obs
// moments, advantage mean / std) are exact two-pass reductions over all its rows.
constexpr int kPrepWaves = 16;
constexpr int kPrepBatch = 16;  // obs loads of a row issued back to back (launch bounds: <= 128 VGPRs)

__device__ __forceinline__ int prep_idx(const PPOArgs& a, const PPORcGeo& g, int e, int mb, int c, int lane) {
  const int Bg = g.G * g.nch * g.cw;
  return a.perm[(size_t)e * a.rows + (size_t)mb * Bg + (size_t)c * g.cw + lane];
}

__global__ __launch_bounds__(64 * kPrepWaves) void ppo_rc_prep_kernel(PPOArgs a, PPORcGeo g) {
  __shared__ float red[kPrepWaves][64];
  __shared__ float stat[2][64];
  __shared__ float adv_stat[2];
  __shared__ float red_a[kPrepWaves];
  const int k = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int CH = g.G * g.nch, cw = g.cw, Bg = CH * cw, D = a.D;
  // the main kernel's arrival counters / flags start at zero (stream order: it runs after
  // this launch) -- replaces a separate memset launch per update
  if (k == 0 && threadIdx.x < 64) g.sync[threadIdx.x] = 0u;
  if (k == 0 && a.zero_stats && threadIdx.x < 5) a.stats[threadIdx.x] = 0.f;  // (and the stats)
  const int n_mb = a.rows / Bg;
  const int e = k / n_mb, mb = k - e * n_mb;
  const bool ok = lane < cw;
  // ---- pass 1: gather, feature sums, advantage sum
  float fs = 0.f, as = 0.f;  // lane c: this wave's sum of feature c; as: advantage sum (lane 0)
  for (int c = wv; c < CH; c += nw) {
    const int idx = ok ? prep_idx(a, g, e, mb, c, lane) : 0;
    const size_t slot = (size_t)k * CH + c;
    float* xr = g.xraw + (slot * 64 + lane) * g.dp;
    // batches of kPrepBatch features: all of a batch's loads are issued before its first store
    // (a store to xraw between two obs loads serialises them -- the buffers may alias as far as
    // the compiler knows: ~20 dependent L2 round trips per row before)
    for (int f0 = 0; f0 < g.dp; f0 += kPrepBatch) {
      float xv[kPrepBatch];
#pragma unroll
      for (int i = 0; i < kPrepBatch; ++i) xv[i] = (ok && f0 + i < D) ? a.obs[(size_t)idx * D + f0 + i] : 0.f;
#pragma unroll
      for (int i = 0; i < kPrepBatch; ++i) {
        const int f = f0 + i;
        if (f < g.dp) {
          if (ok) xr[f] = xv[i];
          if (f < D && a.has_norm) {
            const float s = wave_sum(xv[i]);
            if (lane == f) fs += s;
          }
        }
      }
    }
    float av16[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      float v = 0.f;
      if (ok) {
        if (a.discrete) v = j == 0 ? a.acts[idx] : 0.f;
        else v = j < a.A ? a.acts[(size_t)idx * a.A + j] : 0.f;
      }
      av16[j] = v;
    }
    const float adv = ok ? a.adv[idx] : 0.f;
    float* ac = g.acts + (slot * 64 + lane) * 16;
    if (ok)
#pragma unroll
      for (int j = 0; j < 16; ++j) ac[j] = av16[j];
    as += wave_sum(adv);
  }
  red[wv][lane] = fs;
  if (lane == 0) red_a[wv] = as;
  __syncthreads();
  if (wv == 0) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[i][lane];
    stat[0][lane] = s / (float)Bg;
    if (lane == 0) {
      float t = 0.f;
      for (int i = 0; i < nw; ++i) t += red_a[i];
      adv_stat[0] = t / (float)Bg;
    }
  }
  __syncthreads();
  const float am = adv_stat[0];
  // ---- pass 2: centred second moments
  float fv = 0.f, av = 0.f;
  for (int c = wv; c < CH; c += nw) {
    const int idx = ok ? prep_idx(a, g, e, mb, c, lane) : 0;
    if (a.has_norm) {
      for (int f0 = 0; f0 < D; f0 += kPrepBatch) {  // (batched loads, as in pass 1)
        float xv[kPrepBatch];
#pragma unroll
        for (int i = 0; i < kPrepBatch; ++i) xv[i] = (ok && f0 + i < D) ? a.obs[(size_t)idx * D + f0 + i] : 0.f;
#pragma unroll
        for (int i = 0; i < kPrepBatch; ++i) {
          const int f = f0 + i;
          if (f < D) {
            const float d = ok ? xv[i] - stat[0][f] : 0.f;
            const float s = wave_sum(d * d);
            if (lane == f) fv += s;
          }
        }
      }
    }
    const float d = ok ? a.adv[idx] - am : 0.f;
    av += wave_sum(d * d);
  }
  __syncthreads();
  red[wv][lane] = fv;
  __syncthreads();
  if (wv == 0) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red[i][lane];
    stat[1][lane] = s / (float)Bg;
  }
  __syncthreads();
  if (lane == 0) red_a[wv] = av;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int i = 0; i < nw; ++i) s += red_a[i];
    adv_stat[1] = sqrtf(s / (float)(Bg > 1 ? Bg - 1 : 1));
  }
  __syncthreads();
  if (a.has_norm && threadIdx.x < D) {
    g.mom[(size_t)k * 128 + threadIdx.x] = stat[0][threadIdx.x];
    g.mom[(size_t)k * 128 + 64 + threadIdx.x] = stat[1][threadIdx.x];
  }
  const float sd = adv_stat[1];
  // ---- pass 3: per-row (old_logp, normalised advantage, return)
  for (int c = wv; c < CH; c += nw) {
    if (!ok) continue;
    const int idx = prep_idx(a, g, e, mb, c, lane);
    float adv = a.adv[idx];
    if (a.normalize_advantage && Bg > 1) adv = (adv - am) / (sd + 1e-8f);
    const size_t slot = (size_t)k * CH + c;
    f4 rd = {a.old_logp[idx], adv, a.returns[idx], 0.f};
    *reinterpret_cast<f4*>(g.rowd + (slot * 64 + lane) * 4) = rd;
  }
}

}  // namespace rc

using namespace rc;

// Shape-specialised instances (0 = generic). Shared by the plan (which sizes chunks / waves
// for the instance that will run) and the launch. Every instance the plan can reach compiles
// without scratch (tools/kernel_resources.py, profiles/r4_kernel_resources.md).
enum RcInst : int {
  RC_GENERIC = 0,
  RC_NS_CHEETAH32,    // HalfCheetah / Walker2d FeedForward32Policy (tanh), net split
  RC_NS_CARTPOLE32,   // CartPole FeedForward32Policy, net split
  RC_NS_HOPPER64R,    // Hopper MlpPolicy [64, 64] ReLU (AIRL config)
  RC_NS_WALKER64R,    // Walker2d MlpPolicy [64, 64] ReLU (DRLHP config)
  RC_NS_64_D16,       // any 3-layer [64, 64] net, obs dim <= 16 (SB3 MlpPolicy default: CartPole, Hopper, ...)
  RC_NS_64_D32,       // any 3-layer [64, 64] net, obs dim <= 32 (HalfCheetah / Walker2d / Ant, ...)
  RC_CHEETAH32_64,    // both nets per workgroup, 64-row chunks
  RC_CHEETAH32_32,    // the same, 32-row chunks
  RC_HOPPER64R_32,
  RC_WALKER64R_32,
  RC_CARTPOLE32_64,
  RC_64_D16,          // both nets per workgroup, 32-row chunks: any 3-layer [64, 64] net, obs dim <= 16
  RC_64_D32,          // the same, obs dim <= 32, ReLU + Gaussian head
};

static bool rc_inst_is_bf3(int inst) {
  return inst == RC_NS_CHEETAH32 || inst == RC_NS_CARTPOLE32 || inst == RC_NS_HOPPER64R || inst == RC_NS_WALKER64R ||
         inst == RC_NS_64_D16 || inst == RC_NS_64_D32 || inst == RC_CHEETAH32_64 || inst == RC_CARTPOLE32_64;
}

static int rc_instance_raw(const PPOArgs& a, int kt, int cw, bool ns);

// IMITATION_AMD_PPO_BF3=0: exact-fp32 PPO products. The split-bf16 instances are not selected
// (the plan then takes a generic fp32 register-chained build, or the LDS kernel where no
// scratch-free generic build exists -- slower, bit-for-bit the fp32 formulation)
static int rc_instance(const PPOArgs& a, int kt, int cw, bool ns) {
  const int inst = rc_instance_raw(a, kt, cw, ns);
  const char* ev = getenv("IMITATION_AMD_PPO_BF3");
  if (ev && ev[0] == '0' && rc_inst_is_bf3(inst)) return RC_GENERIC;
  return inst;
}

static int rc_instance_raw(const PPOArgs& a, int kt, int cw, bool ns) {
  const int hw = a.pi_dims[1];
  bool uniform = a.n_pi == 3 && a.n_vf == 3;
  for (int l = 1; l < 3 && uniform; ++l) uniform = a.pi_dims[l] == hw && a.vf_dims[l] == hw;
  const int s0 = (a.D + 3) / 4;
  const bool gauss = !a.discrete;
  const bool act_ok = a.hidden_act == 1 || a.hidden_act == 2;
  if (ns) {
    if (uniform && hw == 32 && s0 == 5 && a.hidden_act == 2 && kt == 2 && gauss) return RC_NS_CHEETAH32;
    if (uniform && hw == 32 && s0 == 1 && a.hidden_act == 2 && kt == 2 && !gauss) return RC_NS_CARTPOLE32;
    if (uniform && hw == 64 && s0 == 3 && a.hidden_act == 1 && kt == 4 && gauss) return RC_NS_HOPPER64R;
    if (uniform && hw == 64 && s0 == 5 && a.hidden_act == 1 && kt == 4 && gauss) return RC_NS_WALKER64R;
    if (uniform && hw == 64 && kt == 4 && act_ok && a.D <= 16) return RC_NS_64_D16;
    if (uniform && hw == 64 && kt == 4 && act_ok && a.D <= 32) return RC_NS_64_D32;
    return RC_GENERIC;
  }
  if (uniform && hw == 32 && s0 == 5 && a.hidden_act == 2 && kt == 2 && cw == 64 && gauss) return RC_CHEETAH32_64;
  if (uniform && hw == 32 && s0 == 5 && a.hidden_act == 2 && kt == 2 && cw == 32 && gauss) return RC_CHEETAH32_32;
  if (uniform && hw == 64 && s0 == 3 && a.hidden_act == 1 && kt == 4 && cw == 32 && gauss) return RC_HOPPER64R_32;
  if (uniform && hw == 64 && s0 == 5 && a.hidden_act == 1 && kt == 4 && cw == 32 && gauss) return RC_WALKER64R_32;
  if (uniform && hw == 32 && s0 == 1 && a.hidden_act == 2 && kt == 2 && cw == 64 && !gauss) return RC_CARTPOLE32_64;
  if (uniform && hw == 64 && kt == 4 && cw == 32 && act_ok && a.D <= 16) return RC_64_D16;
  // (ReLU + Gaussian head only: the Tanh and categorical builds of this size need scratch)
  if (uniform && hw == 64 && kt == 4 && cw == 32 && a.hidden_act == 1 && a.D <= 32 && gauss) return RC_64_D32;
  return RC_GENERIC;
}

int device_cu_count() {
  const char* ev = getenv("IMITATION_AMD_PPO_CUS");
  if (ev && atoi(ev) > 0) return atoi(ev);
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

// Host planning: LDS images + parameter items + workgroup split. Returns false if the
// configuration is outside the fast path (falls back to ppo.hip).
// IMITATION_AMD_PPO_PLAN_DEBUG=1: which check rejected a plan (stderr)
static bool plan_reject(int site) {
  const char* ev = getenv("IMITATION_AMD_PPO_PLAN_DEBUG");
  if (ev && ev[0] == '1') fprintf(stderr, "ppo_rc_plan: rejected at check %d\n", site);
  return false;
}

bool ppo_rc_plan(const PPOArgs& a, PPORcGeo& g, size_t& lds_bytes) {
  g = PPORcGeo{};
  if (a.batch % 16 != 0 || a.batch <= 0 || a.rows % a.batch != 0 || a.D > 64 || a.A > 16) return plan_reject(1);
  if (a.n_pi < 1 || a.n_vf < 1 || a.n_pi > kL || a.n_vf > kL) return plan_reject(2);
  const int* dims[2] = {a.pi_dims, a.vf_dims};
  const int nls[2] = {a.n_pi, a.n_vf};
  int wmax = 0;
  for (int q = 0; q < 2; ++q)
    for (int l = 0; l + 1 < nls[q]; ++l) wmax = dims[q][l + 1] > wmax ? dims[q][l + 1] : wmax;
  if (wmax > 64) return plan_reject(3);
  g.kt = wmax <= 32 ? 2 : 4;
  const int KT = g.kt;
  g.nw = waves_for(KT);
  const char* nsev = getenv("IMITATION_AMD_PPO_NETSPLIT");
  // net split: each workgroup runs ONE net (actor or critic) over 64-row chunks -- its 4
  // row-tile waves at one wave per SIMD, with half of the dW / Adam items a both-nets
  // workgroup owns -- and the two nets meet once per minibatch for clip_grad_norm_
  const bool ns = !(nsev && nsev[0] == '0') && (a.rc_cw == 0 || a.rc_cw == 64) && a.batch % 64 == 0;
  // workgroup split: chunks of cw rows (64 for narrow nets, 32 for 64-wide ones: LDS, and
  // the 4-wave workgroup has 2 row-tile waves per net)
  int cw = KT == 2 || ns ? 64 : 32;
  if (a.rc_cw == 16 || a.rc_cw == 32 || (a.rc_cw == 64 && KT == 2)) cw = a.rc_cw;
  if (a.batch < cw) cw = a.batch;
  if (a.batch % cw != 0) {
    cw = 16;
  }
  bool narrow4 = false;  // generic both-nets build at one wave per SIMD (4 waves, <= 32-row chunks)
  if (!(ns && cw == 64) && rc_instance(a, KT, cw, false) == RC_GENERIC) {
    // the 8-wave generic build has 256 registers per wave and spills: run the 4-wave build
    // (2 row-tile waves per net, 512 registers each) for <= 32-wide nets; 64-wide nets outside
    // the [64, 64] family builds cannot hold their owned items without scratch -> the LDS kernel
    if (KT == 4) return plan_reject(4);
    narrow4 = true;
    if (cw > 32) cw = 32;
    if (a.batch % cw != 0) cw = 16;
  }
  const int chunks = a.batch / cw;
  int gmax = a.rc_gmax > 0 ? (a.rc_gmax < kMaxRcGroups ? a.rc_gmax : kMaxRcGroups) : kMaxRcGroups;
  {  // co-residency: every spinning workgroup must hold a CU of its own (> 80 KiB of LDS: one
     // per CU) while the rest of the chip stays free for concurrent streams (the discriminator
     // runs beside the update), so the working blocks are capped at half the device's CUs
    const int cus = a.rc_cus > 0 ? a.rc_cus : device_cu_count();
    const int per = (ns && cw == 64) ? 2 : 1;  // net split: two workgroups per row group
    const int cap = (cus / 2) / per;
    if (cap < 1) return plan_reject(5);
    if (gmax > cap) gmax = cap;
  }
  int G = 1;
  for (int c = gmax; c >= 1; --c)
    if (chunks % c == 0) {
      G = c;
      break;
    }
  g.cw = cw;
  g.G = G;
  g.nch = chunks / G;
  g.ns = ns && cw == 64 ? 1 : 0;
  if (g.ns || narrow4) g.nw = 4;
  // the generic 64-wide net-split build needs scratch (8 weight slots + 2 vectors at runtime
  // shapes): nets outside the specialised [64, 64] families take the LDS kernel
  if (g.ns && KT == 4 && rc_instance(a, KT, cw, true) == RC_GENERIC) return plan_reject(6);
  {  // the 32-wide specialised net-split builds run the split-bf16 forward / dX (kernel: BF3)
    const int inst = rc_instance(a, KT, cw, g.ns != 0);
    g.bf3 = rc_inst_is_bf3(inst) ? 1 : 0;
  }
  int off = 0;
  auto take = [&](int n) {
    const int o = off;
    off += (n + 3) & ~3;
    return o;
  };
  // parameter images first (zeroed at kernel start); net split: both nets' images start at
  // the same offset (a workgroup holds one net), the region is the larger of the two
  const int pbase = off;
  int pend = off;
  for (int q = 0; q < 2; ++q) {
    if (g.ns) off = pbase;
    for (int l = 0; l < nls[q]; ++l) {
      const int din = dims[q][l], dout = dims[q][l + 1];
      const bool last = l == nls[q] - 1;
      if (!last && dout > 16 * KT) return plan_reject(7);
      if (last && dout > 16) return plan_reject(8);
      if (l > 0 && din > 16 * KT) return plan_reject(9);
      g.din[q][l] = din;
      g.dout[q][l] = dout;
      const int ip = l == 0 ? ((din + 3) & ~3) : ((din + 15) & ~15);
      const int op = (dout + 15) & ~15;
      g.ldw[q][l] = (l == 0 ? ((din + 15) & ~15) : ip) + 4;
      // (BF3: the fp32 masters live in the Adam owners' registers -- no fp32 weight image)
      g.w_off[q][l] = take(g.bf3 ? 0 : op * g.ldw[q][l]);
      g.b_off[q][l] = take(op);
      if (g.bf3) {  // split-bf16 weight images (hi + lo): forward [op][pos(in)], transposed [din][pos(out)]
        const int kin = l == 0 ? 32 : 16 * KT, kout = last ? 32 : 16 * KT;
        g.wf_off[q][l] = take(op * bf3_ld(kin));
        g.wt_off[q][l] = l > 0 ? take(((din + 15) & ~15) * bf3_ld(kout)) : 0;
      }
    }
    pend = off > pend ? off : pend;
  }
  off = pend;
  g.ls_off = take(16);
  g.zero_off = take(64);
  g.param_lds = off;
  // activation / dZ images for the dW MFMAs, K-major split-bf16 (ppo_rc_kernel.h img_store):
  // per 16-padded column cs floats = hi rows [0, rows_pad) + lo rows [rows_pad, 2 rows_pad) in
  // bf16 (ppo_rc_kernel.h img_lo: 16-byte aligned halves, 68 / 36 dwords per column);
  // layer-0 input shared by both nets
  const int rows_pad = cw > 32 ? cw : 32;
  const int ldr = rows_pad + 4;
  g.ksteps = rows_pad / 32;
  const int h0 = take(((a.D + 15) & ~15) * ldr);
  const int abase = off;
  int aend = off;
  for (int q = 0; q < 2; ++q) {
    if (g.ns) off = abase;
    for (int l = 0; l < nls[q]; ++l) {
      if (l == 0) {
        g.h_off[q][0] = h0;
        g.ldh[q][0] = ldr;
      } else {
        g.ldh[q][l] = ldr;
        g.h_off[q][l] = take(((g.din[q][l] + 15) & ~15) * ldr);
      }
      g.ldz[q][l] = ldr;
      g.z_off[q][l] = take(((g.dout[q][l] + 15) & ~15) * ldr);
      g.db_off[q][l] = take(4 * 64);
    }
    aend = off > aend ? off : aend;
  }
  off = aend;
  // the G > 16 first-level stash reuses the activation images (G x 256 floats)
  g.xstash = G > 16 && aend - h0 >= G * 256 ? h0 : -1;
  g.lsp_off = take(4 * 16);
  g.nm_off = take(256);
  g.red_off = take(8 + 8 * 5 + 4);  // wave |g|^2, wave stats, [48] both nets' |g|^2
  g.trash_off = take(64);
  g.lds_floats = off;
  lds_bytes = (size_t)off * 4;
  if (getenv("IMITATION_AMD_PPO_PLAN_DEBUG")) fprintf(stderr, "ppo_rc_plan: %zu B of LDS\n", lds_bytes);
  if (lds_bytes > 160 * 1024) return plan_reject(10);
  // items: dW tiles first (ids [0, n_witems): a wave's weight items are its first slots),
  // actor's then critic's; then bias vectors: actor's, log_std (an actor item), critic's
  int n = 0;
  for (int q = 0; q < 2; ++q) {
    g.wbase[q] = n;
    for (int l = 0; l < nls[q]; ++l) {
      const int to = (g.dout[q][l] + 15) / 16, ti = (g.din[q][l] + 15) / 16;
      for (int ta = 0; ta < to; ++ta)
        for (int tb = 0; tb < ti; ++tb) {
          if (n >= kMaxRcItems) return plan_reject(11);
          g.items[n++] = q | (l << 1) | (0 << 3) | (ta << 5) | (tb << 9);
        }
    }
    g.nwit[q] = n - g.wbase[q];
  }
  g.n_witems = n;
  for (int q = 0; q < 2; ++q) {
    g.bbase[q] = n;
    for (int l = 0; l < nls[q]; ++l) {
      if (n >= kMaxRcItems) return plan_reject(12);
      g.items[n++] = q | (l << 1) | (1 << 3);
    }
    if (q == 0 && !a.discrete && a.log_std_off >= 0) {
      if (n >= kMaxRcItems) return plan_reject(13);
      g.items[n++] = 2 << 3;
    }
    g.nbit[q] = n - g.bbase[q];
  }
  g.n_items = n;
  int wmx = g.n_witems, bmx = n - g.n_witems;
  if (g.ns) {
    wmx = g.nwit[0] > g.nwit[1] ? g.nwit[0] : g.nwit[1];
    bmx = g.nbit[0] > g.nbit[1] ? g.nbit[0] : g.nbit[1];
  }
  int wcap = g.ns ? wslots_ns(KT) : wslots_for(KT), bcap = g.ns ? bslots_ns() : bslots_for(KT);
  if (narrow4) {
    wcap = kNarrow4W;
    bcap = kNarrow4B;
  }
  {  // the specialised instances size their slots to the shape they were built for
    const int inst = rc_instance(a, KT, cw, g.ns != 0);
    if (inst == RC_NS_64_D16) { wcap = 6; bcap = 1; }
    if (inst == RC_NS_64_D32) { wcap = 7; bcap = 1; }
    if (inst == RC_64_D16) { wcap = 12; bcap = 2; }
    if (inst == RC_64_D32) { wcap = 14; bcap = 2; }
  }
  if ((wmx + g.nw - 1) / g.nw > wcap || (bmx + g.nw - 1) / g.nw > bcap) return plan_reject(14);
  g.dp = (a.D + 3) & ~3;
  return true;
}

size_t ppo_rc_workspace_floats(const PPOArgs& a) {
  PPORcGeo g;
  size_t lds = 0;
  if (!ppo_rc_plan(a, g, lds)) return 0;
  const size_t K = (size_t)a.n_epochs * (a.rows / a.batch);
  const size_t slots = K * g.G * g.nch;
  return slots * 64 * (g.dp + 16 + 4) + K * 128 + 2 * (size_t)(g.G + 1) * g.n_items * 256 + 64;
}

hipError_t ppo_rc_launch(const PPOArgs& a, float* workspace, hipStream_t s) {
  PPORcGeo g;
  size_t lds = 0;
  if (!ppo_rc_plan(a, g, lds)) return hipErrorInvalidValue;
  const size_t K = (size_t)a.n_epochs * (a.rows / a.batch);
  const size_t slots = K * g.G * g.nch;
  g.xraw = workspace;
  g.acts = g.xraw + slots * 64 * g.dp;
  g.rowd = g.acts + slots * 64 * 16;
  g.mom = g.rowd + slots * 64 * 4;
  g.slab = g.mom + K * 128;
  g.red = g.slab + 2 * (size_t)g.G * g.n_items * 256;
  g.sync = reinterpret_cast<unsigned*>(g.red + 2 * (size_t)g.n_items * 256);
  {  // two-level exchange from 4 (64-wide nets) / 16 (<= 32-wide) cooperating workgroups
     // (IMITATION_AMD_PPO_XCHG2=0/1 forces it; measured: profiles/r3_ppo64_scale.md)
    const char* ev = getenv("IMITATION_AMD_PPO_XCHG2");
    g.xchg2 = ev ? (ev[0] == '1' && g.G > 1) : (g.G >= (g.kt == 4 ? 4 : 16));
  }
  if (K == 0) return hipSuccess;
  // > 80 KiB of LDS keeps the cooperating workgroups one per CU (the measured condition of
  // the sc1 hand-off); all G <= kMaxRcGroups (64) of them are co-resident (256 CUs)
  // (net split: the two workgroups must not share a CU's matrix cores either)
  size_t lds_launch = (g.G > 1 || g.ns) && lds < 96 * 1024 ? 96 * 1024 : lds;
  const int nblk = g.ns ? 2 * g.G : g.G;
  {  // cooperating workgroups on as few XCDs as possible (the "xcd" geometry field is the block
     // stride). GAIL emulated W = 2 / 4 / 8: 3.14 / 3.28 / 3.64 -> 2.99 / 2.96 / 3.36 ms per update,
     // headline round 3.63 -> 3.55 ms (profiles/r3_ppo_xcd.md)
    // At most 16 workgroups (half an XCD's 32 CUs) per XCD, so concurrent work on the other
    // stream (the discriminator) never holds a CU a spinning cooperating workgroup waits for:
    // stride 8 / 4 / 2 for <= 16 / 32 / 64 workgroups (blocks b % stride == 0 work: XCDs {0},
    // {0, 4}, {0, 2, 4, 6} of the deal). DRLHP emulated W = 8 (32 workgroups): one XCD 27.3 ms,
    // spread 25.6 ms (profiles/r3_ppo_xcd.md).
    g.xcd = 1;
    if (nblk > 1) g.xcd = nblk <= 16 ? 8 : nblk <= 32 ? 4 : nblk <= 64 ? 2 : 1;
    // never a wider stride than the device has XCDs (32 CUs each; a partitioned device has fewer)
    const int cus = a.rc_cus > 0 ? a.rc_cus : device_cu_count();
    const int xcds = cus / 32 > 1 ? cus / 32 : 1;
    while (g.xcd > xcds) g.xcd >>= 1;
  }
  const dim3 grid(nblk * g.xcd), block(64 * g.nw);
  int wmx = g.n_witems, bmx = g.n_items - g.n_witems;
  if (g.ns) {
    wmx = g.nwit[0] > g.nwit[1] ? g.nwit[0] : g.nwit[1];
    bmx = g.nbit[0] > g.nbit[1] ? g.nbit[0] : g.nbit[1];
  }
  const int nwslot = (wmx + g.nw - 1) / g.nw, nbslot = (bmx + g.nw - 1) / g.nw;
  typedef void (*RcKernel)(PPOArgs, PPORcGeo);
  RcKernel kern = nullptr;
#define IA_RC(KT, KW, KB, S0, NL, ACT, HW, CW, DT) kern = ppo_rc_kernel<KT, KW, KB, S0, NL, ACT, HW, CW, DT, waves_for(KT)>
#define IA_RC_NS(KT, KW, KB, S0, NL, ACT, HW, DT) kern = ppo_rc_kernel<KT, KW, KB, S0, NL, ACT, HW, 64, DT, 4>
  const auto fits = [&](int kw, int kb) { return nwslot <= kw && nbslot <= kb; };
  const bool cat = a.discrete != 0;
  const int hact = a.hidden_act;
  switch (rc_instance(a, g.kt, g.cw, g.ns != 0)) {
    case RC_NS_CHEETAH32: if (fits(3, 1)) IA_RC_NS(2, 3, 1, 5, 3, 2, 32, 0); break;
    case RC_NS_CARTPOLE32: if (fits(2, 1)) IA_RC_NS(2, 2, 1, 1, 3, 2, 32, 1); break;
    case RC_NS_HOPPER64R: if (fits(6, 1)) IA_RC_NS(4, 6, 1, 3, 3, 1, 64, 0); break;
    case RC_NS_WALKER64R: if (fits(7, 1)) IA_RC_NS(4, 7, 1, 5, 3, 1, 64, 0); break;
    case RC_NS_64_D16:
      if (hact == 1 && !cat) IA_RC_NS(4, 6, 1, -4, 3, 1, 64, 0);
      else if (hact == 1) IA_RC_NS(4, 6, 1, -4, 3, 1, 64, 1);
      else if (!cat) IA_RC_NS(4, 6, 1, -4, 3, 2, 64, 0);
      else IA_RC_NS(4, 6, 1, -4, 3, 2, 64, 1);
      break;
    case RC_NS_64_D32:
      if (hact == 1 && !cat) IA_RC_NS(4, 7, 1, -8, 3, 1, 64, 0);
      else if (hact == 1) IA_RC_NS(4, 7, 1, -8, 3, 1, 64, 1);
      else if (!cat) IA_RC_NS(4, 7, 1, -8, 3, 2, 64, 0);
      else IA_RC_NS(4, 7, 1, -8, 3, 2, 64, 1);
      break;
    case RC_CHEETAH32_64: if (fits(3, 1)) IA_RC(2, 3, 1, 5, 3, 2, 32, 64, 0); break;
    case RC_CHEETAH32_32: if (fits(3, 1)) IA_RC(2, 3, 1, 5, 3, 2, 32, 32, 0); break;
    case RC_HOPPER64R_32: if (fits(12, 2)) IA_RC(4, 12, 2, 3, 3, 1, 64, 32, 0); break;
    case RC_WALKER64R_32: if (fits(14, 2)) IA_RC(4, 14, 2, 5, 3, 1, 64, 32, 0); break;
    case RC_CARTPOLE32_64: if (fits(2, 1)) IA_RC(2, 2, 1, 1, 3, 2, 32, 64, 1); break;
    case RC_64_D16:
      if (hact == 1 && !cat) IA_RC(4, 12, 2, -4, 3, 1, 64, 32, 0);
      else if (hact == 1) IA_RC(4, 12, 2, -4, 3, 1, 64, 32, 1);
      else if (!cat) IA_RC(4, 12, 2, -4, 3, 2, 64, 32, 0);
      else IA_RC(4, 12, 2, -4, 3, 2, 64, 32, 1);
      break;
    case RC_64_D32:
      IA_RC(4, 14, 2, -8, 3, 1, 64, 32, 0);
      break;
    default: break;
  }
  if (kern == nullptr) {
    if (g.ns && g.kt == 2)
      IA_RC_NS(2, wslots_ns(2), bslots_ns(), 0, 0, -1, 0, -1);
    else if (g.kt == 2 && g.nw == 4)
      kern = ppo_rc_kernel<2, kNarrow4W, kNarrow4B, 0, 0, -1, 0, 0, -1, 4>;
    else
      return hipErrorInvalidValue;  // the plan never selects a spilling generic build
  }
#undef IA_RC
#undef IA_RC_NS
  if (nblk > 1) {
    // every working block must be resident at once: check the instance's occupancy at this
    // LDS size against the device (the plan capped the working blocks at half the CUs)
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), (int)block.x,
                                                     lds_launch) != hipSuccess)
      per_cu = 1;
    if (per_cu > 1 && lds_launch > 80 * 1024) per_cu = 1;  // LDS holds one block per CU (the API can read high)
    const int cus = a.rc_cus > 0 ? a.rc_cus : device_cu_count();
    if (per_cu < 1 || (long long)per_cu * cus < (long long)nblk) return hipErrorCooperativeLaunchTooLarge;
  }
  const int CH = g.G * g.nch;
  const int prep_waves = CH < kPrepWaves ? CH : kPrepWaves;
  hipLaunchKernelGGL(ppo_rc_prep_kernel, dim3((unsigned)K), dim3(64 * prep_waves), 0, s, a, g);
  hipLaunchKernelGGL(kern, grid, block, lds_launch, s, a, g);
  return hipGetLastError();
}

}  // namespace ia

// Register-chained PPO update (mode 0): the fast path of engine_ppo_update.
//
// This header holds the kernel template; its instances are compiled in parallel TUs
// (ppo_rc_inst*.hip, listed in ppo_rc_instances.h) and planned / launched by ppo_rc.hip.
//
// Same semantics as ppo.hip (SB3 PPO.train: RunningNorm train-mode update per
// minibatch, advantage normalisation, clipped surrogate + entropy + value loss,
// clip_grad_norm_, Adam; reference call chain common.py train_gen -> PPO.learn ->
// PPO.train) but laid out so that a minibatch needs three workgroup barriers instead
// of one per layer and stage:
//
// * The MLPs run in the TRANSPOSED formulation C[out][row] = W . H^T on
//   v_mfma_f32_16x16x4_f32 (exact fp32). A lane's accumulator then holds outputs
//   4*(lane>>4)+q of row lane&15, and with the K (input-feature) order permuted as
//   f(s, kk) = 16*(s>>2) + 4*kk + (s&3) those four registers ARE the B operand of the
//   next layer's MFMA steps -- activations never leave registers between layers, and
//   each wave (16 rows of one net) runs forward, loss and the dX backward chain with
//   no barrier. Weights are read from LDS as float4 (forward) / float (W^T backward).
// * Row-data preparation is hoisted out of the sequential loop: ppo_rc_prep_kernel
//   gathers every minibatch of every epoch in parallel (perm is known up front),
//   normalises advantages per minibatch and computes each minibatch's observation
//   moments; the kernel only Chan-merges those moments (one lane per feature) one
//   minibatch ahead.
// * dW (K = rows) needs rows along K, i.e. a transpose: layer inputs and dZ are
//   stored K-major in LDS once ([column][permuted row], row r at (r & 3) * cw/4 + r / 4,
//   so the rows 4s + kk that lane group kk feeds to MFMA step s are contiguous and one
//   ds_read_b128 serves four steps), then every wave computes whole dW tiles over all
//   rows for the parameter "items" it owns -- all of its weight tiles interleaved, so
//   their MFMA chains hide each other's latency. The owner keeps that tile's gradient and
//   Adam moments in registers, so after the grad-norm reduction Adam updates W in
//   LDS in place -- there is no gradient image at all.
//
// Large minibatches (AIRL-Hopper's 512 rows, or the data-parallel replicated update
// whose minibatch is world x the per-rank one) are split over G cooperating
// workgroups, each running nch chunks of cw rows and accumulating its dW partials in
// the owner registers. The G partials are exchanged through a double-buffered slab
// with the placement-independent sc1 hand-off (sc1 stores, every storing wave's
// vmcnt(0), a workgroup barrier, one agent-scope arrival per workgroup, sc1 poll,
// sc1 loads -- MI355X_MICROARCH "Workgroup dispatch ... & inter-workgroup
// visibility", row 1) and summed in workgroup order, so every workgroup applies the
// bit-identical update to its own LDS copy of the parameters; there is one grid-wide
// wait per minibatch and no parameter broadcast. The spin is bounded (timeout flag).
//
// barriers / minibatch: [fwd+loss+bwd chain] B1 [dW items] (exchange) [|g|^2] B2 [clip, Adam] B3
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "ia/engine.h"
#include "ia/wave.h"
#include "launchers.h"


namespace ia {
namespace rc {


typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) bf16 lbf;
typedef __attribute__((address_space(3))) bf16x8 lbf8;
typedef __attribute__((address_space(3))) float lf;
typedef __attribute__((address_space(3))) f4 lf4;

constexpr int kL = kWaveMaxLayers;

__device__ __forceinline__ f4 mfma(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }

// tanh as 1 - 2 / (exp(2x) + 1) on v_exp_f32 / v_rcp_f32 (abs error ~2e-7; saturates
// correctly at +-inf) instead of the branchy libm tanhf
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __expf(2.f * fminf(fmaxf(x, -15.f), 15.f));
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);  // v_rcp_f32 (1 ulp), not the IEEE divide sequence
}

__device__ __forceinline__ float act_fn(int act, float x) {
  switch (act) {
    case 1: return fmaxf(x, 0.f);
    case 2: return tanh_fast(x);
    case 3: return x > 0.f ? x : 0.01f * x;
    case 4: return 1.f / (1.f + expf(-x));
    default: return x;
  }
}
__device__ __forceinline__ float act_grad(int act, float y) {
  switch (act) {
    case 1: return y > 0.f ? 1.f : 0.f;
    case 2: return 1.f - y * y;
    case 3: return y > 0.f ? 1.f : 0.01f;
    case 4: return y * (1.f - y);
    default: return 1.f;
  }
}
// Row / lane-group reductions without LDS round trips (ia/wave.h): sum16 over the 16 rows
// of an MFMA tile (lanes with equal lane >> 4), sum_kk / max_kk over the 4 lane groups
// of one row (lanes r, r + 16, r + 32, r + 48).
__device__ __forceinline__ float sum16(float v) { return row_sum16(v); }
__device__ __forceinline__ float sum_kk(float v) { return add_halves(add_rows16(v)); }
__device__ __forceinline__ float max_kk(float v) { return max_halves(max_rows16(v)); }

// sc1 (L1-bypassing, agent-coherent) accesses for the cross-workgroup hand-off. The
// 16-B forms are inline asm so that a lane can issue all G partial loads back to back
// (relaxed atomic loads are 4-B and get serialised by the compiler); the results are
// tied to the explicit vmcnt(0) wait through "+v" operands so no use moves above it.
__device__ __forceinline__ void st_sc1_x4(float* p, f4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st_sc1_x1(float* p, float v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ f4 ld_sc1_x4(const float* p) {
  f4 v;
  asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void wait_vm4(f4& a, f4& b, f4& c, f4& d) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
}
__device__ __forceinline__ void wait_vm8(f4 (&v)[8]) {
  asm volatile("s_waitcnt vmcnt(0)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])::"memory");
}
template <int N>
__device__ __forceinline__ void wait_vm_n(f4 (&v)[N]) {
  if constexpr (N == 32) {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]),
                   "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])::"memory");
    asm volatile(""
                 : "+v"(v[16]), "+v"(v[17]), "+v"(v[18]), "+v"(v[19]), "+v"(v[20]), "+v"(v[21]), "+v"(v[22]), "+v"(v[23]),
                   "+v"(v[24]), "+v"(v[25]), "+v"(v[26]), "+v"(v[27]), "+v"(v[28]), "+v"(v[29]), "+v"(v[30]), "+v"(v[31])::"memory");
  } else if constexpr (N == 16) {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]),
                   "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])::"memory");
  } else if constexpr (N == 8) {
    wait_vm8(v);
  } else if constexpr (N == 4) {
    wait_vm4(v[0], v[1], v[2], v[3]);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i])::"memory");
  }
}
__device__ __forceinline__ unsigned ld_sc1u(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A bounded spin gave up (a partner workgroup never arrived: not co-resident, stalled, or the
// debug_stall test knob): raise the per-launch flag -- every other spin of this launch then
// stops at once -- and the persistent error word the host reads (EngineErrorFlag in Python),
// which turns the silently partial update into a RuntimeError.
__device__ __forceinline__ void spin_give_up(const PPOArgs& a, unsigned* tflag) {
  atomicOr(tflag, 1u);
  if (a.err) atomicOr(a.err, 1u);
}

// Geometry of one net layer in the LDS images (all offsets in floats, uniform).
struct LG {
  int din, dout, w, ldw, b, h, ldh, z, ldz, db;
};
__device__ __forceinline__ LG lg(const PPORcGeo& g, int q, int l) {
  LG r;
  r.din = rfl(g.din[q][l]);
  r.dout = rfl(g.dout[q][l]);
  r.w = rfl(g.w_off[q][l]);
  r.ldw = rfl(g.ldw[q][l]);
  r.b = rfl(g.b_off[q][l]);
  r.h = rfl(g.h_off[q][l]);
  r.ldh = rfl(g.ldh[q][l]);
  r.z = rfl(g.z_off[q][l]);
  r.ldz = rfl(g.ldz[q][l]);
  r.db = rfl(g.db_off[q][l]);
  return r;
}

// ---------------------------------------------------------------- main kernel
template <int S0M>
struct Rows {  // one chunk's rows for this lane, prefetched a chunk ahead
  float x[S0M];  // raw obs: feature 4s + kk of row lane&15 (s < S0)
  f4 act;       // actions 4kk..4kk+3 (Gaussian) / act index in .x (discrete)
  f4 rd;        // old_logp, adv_n, return
};

template <int S0M>
__device__ __forceinline__ void load_rows(const PPORcGeo& g, size_t slot, int row, int kk, int s0, Rows<S0M>& r) {
  const float* xr = g.xraw + (slot * 64 + row) * g.dp;
#pragma unroll
  for (int s = 0; s < S0M; ++s)
    if (s < s0) r.x[s] = xr[4 * s + kk];
  const float* ac = g.acts + (slot * 64 + row) * 16;
  r.act = *reinterpret_cast<const f4*>(ac + 4 * kk);
  r.rd = *reinterpret_cast<const f4*>(g.rowd + (slot * 64 + row) * 4);
}

// Sum of the G workgroups' partials of this wave's items, in group order, 8 sc1 loads in
// flight per lane and ONE wait per batch of IB = 8 / G items (a load round trip is ~1.2K
// cycles; a wait per item and 4 groups made the loads the exchange's dominant cost).
// ids[s]: item id of owned slot s (-1: empty slot).
template <int GT, int KI, int NF = 16>
__device__ __forceinline__ void exchange_sum(const float* slab, int n_items, const int (&ids)[KI], int lane, f4 (&xg)[KI]) {
  constexpr int IB0 = NF / GT;
  constexpr int IB = IB0 < KI ? IB0 : KI;
#pragma unroll
  for (int i0 = 0; i0 < KI; i0 += IB) {
    f4 v[NF];
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int it = i0 + i;
      const int id = it < KI && ids[it] >= 0 ? ids[it] : 0;
#pragma unroll
      for (int gi = 0; gi < GT; ++gi) v[i * GT + gi] = ld_sc1_x4(slab + ((size_t)gi * n_items + id) * 256 + lane * 4);
    }
#pragma unroll
    for (int e = IB * GT; e < NF; ++e) v[e] = v[0];
    wait_vm_n<NF>(v);
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int it = i0 + i;
      if (it >= KI || ids[it] < 0) continue;
      f4 sacc = v[i * GT];
#pragma unroll
      for (int gi = 1; gi < GT; ++gi) sacc += v[i * GT + gi];
      xg[it] = sacc;
    }
  }
}

// First level of the two-level exchange for G = GT workgroups: this wave sums the G
// partials of its slots sl = grp + r * GT (group order) and publishes them. All of those
// loads (<= KI + GT - 1) are issued back to back before ONE wait; slot ids are computed by
// slot_id (register arrays indexed by the run-time grp would go to scratch).
template <int GT, int KI, typename SlotId>
__device__ __forceinline__ void reduce_slots(const float* slab, float* red, size_t gs, int grp, int lane, const SlotId& slot_id) {
  constexpr int RM = (KI + GT - 1) / GT;
  f4 v[RM * GT];
  int rid[RM];
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    const int sl = grp + r * GT;
    rid[r] = sl < KI ? slot_id(sl) : -1;
    const int id = rid[r] >= 0 ? rid[r] : 0;
#pragma unroll
    for (int gi = 0; gi < GT; ++gi) v[r * GT + gi] = ld_sc1_x4(slab + (size_t)gi * gs + (size_t)id * 256 + lane * 4);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int e = 0; e < RM * GT; ++e) asm volatile("" : "+v"(v[e])::"memory");  // results tied to the wait
#pragma unroll
  for (int r = 0; r < RM; ++r) {
    if (rid[r] < 0) continue;
    f4 sacc = v[r * GT];
#pragma unroll
    for (int gi = 1; gi < GT; ++gi) sacc += v[r * GT + gi];
    st_sc1_x4(red + (size_t)rid[r] * 256 + lane * 4, sacc);
  }
}

// dW tiles of this wave's N weight items over one chunk (K = rows): acc[i] += dZ^T H for item i
// on v_mfma_f32_16x16x32_bf16 with the split-bf16 ("bf16x3") product: every image value is
// stored as hi = bf16(v) and lo = bf16(v - hi), and dZ^T H = hi.hi + hi.lo + lo.hi (the lo.lo term
// is ~2^-16 of the product: near-fp32 accuracy at 3 bf16 MFMAs per 32 rows instead of eight
// 16x16x4 fp32 ones). Images are K-major (rows contiguous): column c of an image has its hi rows
// at bf16 index 2 c cs + r and its lo rows at 2 c cs + img_lo(cs) + r (cs floats per column).
// Lane (r16, kk) reads rows
// 8 kk .. 8 kk + 7 (+ 32 per K-step) of column r16 of the item's dZ (A, M = out) and H (B,
// N = in) tiles; the accumulator layout is the fp32 kernel's (C[out 4 kk + j][in r16]), so the
// exchange and Adam code is unchanged. izo / iho: bf16 offsets of the lane's first element;
// lo: bf16 offset of the lo half (img_lo).
// A column of a K-major split-bf16 image is 2 cs bf16 (cs = rows_pad + 4 floats): hi rows at
// [0, rows_pad), lo rows at [rows_pad, 2 rows_pad), 8 bf16 of padding. The lo half starts at a
// 16-byte boundary (a ds_read_b128 off its natural alignment stalls ~60 cycles) and the column
// stride of rows_pad / 4 + 1 (odd) 16-byte slots spreads a read group's 16 columns over the banks.
__device__ __forceinline__ int img_lo(int cs) { return cs - 4; }

__device__ __forceinline__ f4 mfma_bf16(bf16x8 a, bf16x8 b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

template <int N>
__device__ __forceinline__ void dw_tiles(const lf* L, const int* izo, const int* iho, int lo, int ksteps, f4* acc) {
  const lbf* Lb = (const lbf*)L;
  // items in groups of GS: independent accumulation chains keep the MFMA pipe busy while only
  // the group's operands (4 x bf16x8 per item) are live (2 per group for the largest slot counts)
  constexpr int GS = N >= 12 ? 2 : 4;
#pragma unroll
  for (int i0 = 0; i0 < N; i0 += GS) {
    for (int ks = 0; ks < ksteps; ++ks) {
      bf16x8 zh[GS], zl[GS], hh[GS], hl[GS];
#pragma unroll
      for (int i = 0; i < GS; ++i) {
        if (i0 + i >= N) continue;
        const lbf* zp = Lb + izo[i0 + i] + 32 * ks;
        const lbf* hp = Lb + iho[i0 + i] + 32 * ks;
        zh[i] = *(const lbf8*)zp;
        zl[i] = *(const lbf8*)(zp + lo);
        hh[i] = *(const lbf8*)hp;
        hl[i] = *(const lbf8*)(hp + lo);
      }
#pragma unroll
      for (int i = 0; i < GS; ++i) {
        if (i0 + i >= N) continue;
        acc[i0 + i] = mfma_bf16(zh[i], hh[i], acc[i0 + i]);
        acc[i0 + i] = mfma_bf16(zh[i], hl[i], acc[i0 + i]);
        acc[i0 + i] = mfma_bf16(zl[i], hh[i], acc[i0 + i]);
      }
    }
  }
}

// one value into a split-bf16 K-major image: hi at [col][row], lo one half-column (cs bf16) on
__device__ __forceinline__ void img_store(lf* L, int off, int cs, int col, int row, float v) {
  lbf* p = (lbf*)(L + off) + (2 * col * cs + row);
  const bf16 h = (bf16)v;
  p[0] = h;
  p[img_lo(cs)] = (bf16)(v - (float)h);
}

// ---- split-bf16 forward / input-gradient path (BF3: 32- and 64-wide 3-layer nets, obs dim <= 32)
// The fp32 16x16x4 chains (8 MFMAs of 32 cycles per 32 of K) become v_mfma_f32_16x16x32_bf16
// triples (hi.hi + hi.lo + lo.hi: 3 x 16 cycles, ~2^-16 relative product error) over bf16 hi / lo
// weight images; the fp32 master weights live in the Adam owners' registers, which rewrite the
// images after every step. The B operand of a lane is its own 8 activations per 32 of K (C layout
// of the previous layer: features 16 t + 4 kk + j of tiles 2 s, 2 s + 1 in K-step s) in the K
// order pos_h(f); the weight images store column f at that position, so no data moves between
// lanes. Layer 0's input is lane kk's features 4 s + kk (s < 8) at position 8 kk + s (pos_in0).
// Image rows hold K + 8 bf16 (the 16 rows of a b128 group on distinct banks).
__host__ __device__ __forceinline__ int bf3_ld(int k) { return k + 8; }
__device__ __forceinline__ int bf3_pos_in0(int f) { return 8 * (f & 3) + (f >> 2); }
__device__ __forceinline__ int bf3_pos_h(int f) { return 32 * (f >> 5) + 8 * ((f >> 2) & 3) + 4 * ((f >> 4) & 1) + (f & 3); }

__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bf16 h = (bf16)v[j];
    hi[j] = h;
    lo[j] = (bf16)(v[j] - (float)h);
  }
}

// acc += A_tile(32 of K) . B with A's row of this lane at `a` (hi image; lo image `lo_off` bf16 on)
__device__ __forceinline__ f4 bf3_tile(const lbf* a, int lo_off, bf16x8 bh, bf16x8 bl, f4 acc) {
  const bf16x8 ah = *(const lbf8*)a;
  const bf16x8 al = *(const lbf8*)(a + lo_off);
  acc = mfma_bf16(ah, bh, acc);
  acc = mfma_bf16(ah, bl, acc);
  return mfma_bf16(al, bh, acc);
}

// Geometry of layer l's images: forward Wf [16-padded dout rows][pos(in)] (K = 32 for layer 0,
// 16 KT for hidden inputs), transposed Wt [16-padded din rows][pos_h(out)] (layers >= 1; K = 32 for
// the head's <= 16 outputs, 16 KT otherwise); lo image right after hi.
template <int KT>
__device__ __forceinline__ void bf3_store_w(lf* L, const PPORcGeo& g, int q, int l, int o, int i, float v, int nl) {
  const bf16 h = (bf16)v;
  const bf16 lo = (bf16)(v - (float)h);
  const int kin = l == 0 ? 32 : 16 * KT;
  const int rows = (g.dout[q][l] + 15) & ~15;
  lbf* wf = (lbf*)(L + g.wf_off[q][l]) + o * bf3_ld(kin) + (l == 0 ? bf3_pos_in0(i) : bf3_pos_h(i));
  wf[0] = h;
  wf[rows * bf3_ld(kin)] = lo;
  if (l > 0) {
    const int kout = l == nl - 1 ? 32 : 16 * KT;
    const int trows = (g.din[q][l] + 15) & ~15;
    lbf* wt = (lbf*)(L + g.wt_off[q][l]) + i * bf3_ld(kout) + bf3_pos_h(o);
    wt[0] = h;
    wt[trows * bf3_ld(kout)] = lo;
  }
}

// An Adam owner's 4 updated elements W[16 ta + 4 kk + j][16 tb + r16] (j < 4) into the images:
// forward image rows o = 16 ta + 4 kk + j at one column pos(in) (4 b16 stores per half), the
// transposed image row in at the 4 consecutive positions pos_h(16 ta + 4 kk + j) (one b64 store
// per half). kind (0 input layer, 1 hidden, 2 head), the image bases wf / wt (bf16, with the
// wave-uniform parts of pos) and lo-half offsets are the slot's hoisted uniforms; only the lane
// terms are formed here: pos_in0(16 tb + r16) = 4 tb + 8 (r16 & 3) + (r16 >> 2), pos_h(16 tb +
// r16) = 32 (tb >> 1) + 4 (tb & 1) + 8 (r16 >> 2) + (r16 & 3).
template <int KT>
__device__ __forceinline__ void bf3_store_tile(lf* L, int kind, int wf, int wfl, int wt, int wtl, int r16, int kk,
                                               const float (&v)[4]) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) bf16x4 lbf4;
  bf16x4 h4, l4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16 h = (bf16)v[j];
    h4[j] = h;
    l4[j] = (bf16)(v[j] - (float)h);
  }
  lbf* Lb = (lbf*)L;
  const int ldi = kind == 0 ? bf3_ld(32) : bf3_ld(16 * KT);
  lbf* pf = Lb + wf + 4 * kk * ldi + (kind == 0 ? 8 * (r16 & 3) + (r16 >> 2) : 8 * (r16 >> 2) + (r16 & 3));
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    pf[j * ldi] = h4[j];
    pf[j * ldi + wfl] = l4[j];
  }
  if (kind != 0) {
    const int ldo = kind == 2 ? bf3_ld(32) : bf3_ld(16 * KT);
    lbf* pt = Lb + wt + r16 * ldo + 8 * kk;
    *(lbf4*)pt = h4;
    *(lbf4*)(pt + wtl) = l4;
  }
}

// Shape specialisation: S0T (16-wide input k-steps / 4), NLT (layers per net), ACTT (hidden
// activation), HWT (hidden width) fold the per-layer loop bounds, tile counts and the
// activation switch at compile time; 0 / -1 = read them at run time (generic build).
// DT: action head (0 Gaussian, 1 categorical, -1 read at run time).
// NW: waves per workgroup. 8 (512 threads, 2 waves per SIMD) for the <= 32-wide nets; 4
// (256 threads, ONE wave per SIMD) for the 64-wide ones, whose owned gradient / Adam state
// (up to 16 items x 12 floats per lane) and 64-wide activation tiles need more than the 256
// registers a wave gets at 2 waves / SIMD: at 1 wave / SIMD the wave has the whole 512-entry
// VGPR + AGPR file, and nothing goes to scratch.
// KW / KB: weight-tile / bias-vector slots per wave. Wave w owns weight items w + it * NW
// (it < KW; a 16 x 16 tile, 4 elements per lane) and bias / log_std items n_witems + w + ib * NW
// (ib < KB; one element per lane), so the owned state is 12 KW + 3 KB floats per lane and
// every slot's kind is known at compile time.
template <int KT, int KW, int KB, int S0T, int NLT, int ACTT, int HWT, int CWT, int DT, int NW>
__global__ __launch_bounds__(64 * NW) void ppo_rc_kernel(PPOArgs a, PPORcGeo g) {
  constexpr int KI = KW + KB;
  constexpr int kThreads = 64 * NW;
  constexpr int kWaves = NW;
  constexpr int kHalf = NW / 2;  // row-tile waves per net
  extern __shared__ __attribute__((aligned(16))) float lds_raw[];
  lf* L = (lf*)lds_raw;
  const int tid = threadIdx.x;
  const int w = rfl(tid >> 6), lane = tid & 63;
  const int r16 = lane & 15, kk = lane >> 4;
  const bool ns = g.ns != 0;  // net split: workgroup 2 grp + q runs net q of row group grp
  int bid = (int)blockIdx.x;
  if (g.xcd > 1) {  // XCD-co-located plan: only every xcd-th block works
    if (bid % g.xcd) return;
    bid /= g.xcd;
  }
  const int q = ns ? (bid & 1) : w / kHalf;  // 0 actor, 1 critic
  const int gw = ns ? w : w % kHalf;         // row tile
  const int grp = ns ? (bid >> 1) : bid;     // row group
  const int G = g.G, nch = g.nch, cw = CWT > 0 ? CWT : g.cw;
  const int CH = G * nch;
  const int Bg = CH * cw;  // minibatch rows
  const int RT = cw / 16;
  const bool rows_wave = gw < RT;
  const int nl = NLT > 0 ? NLT : (q == 0 ? a.n_pi : a.n_vf);
  const int D = a.D, A = a.A;
  // S0T > 0: exact input k-steps; S0T < 0: at most -S0T (run-time count, register arrays sized
  // to the bound); 0: generic (<= 16)
  constexpr int S0M = S0T > 0 ? S0T : (S0T < 0 ? -S0T : 16);
  const int s0 = S0T > 0 ? S0T : (D + 3) / 4;
  // split-bf16 forward / dX (see bf3_tile): the specialised 3-layer builds with obs dim <= 32 and
  // 64-row chunks -- net split, and both 32-wide nets in one 8-wave workgroup (the plan sets g.bf3
  // for exactly these and allocates the bf16 weight images)
  constexpr bool BF3 = (HWT == 16 * KT) && NLT == 3 && S0T != 0 && S0M <= 8 && CWT == 64 && (NW == 4 || KT == 2);
  const bool gauss = DT >= 0 ? DT == 0 : !a.discrete;
  const bool has_ls = gauss && a.log_std_off >= 0;
  float am[4];  // action-slot masks of this lane group (Gaussian head)
#pragma unroll
  for (int j = 0; j < 4; ++j) am[j] = 4 * (lane >> 4) + j < a.A ? 1.f : 0.f;
  const int n_mb = a.rows / Bg;
  const int K = a.n_epochs * n_mb;
  const float invB = 1.f / (float)Bg;
  const float c_half_log2pi = 0.91893853320467274f;
  const int n_items = rfl(g.n_items);

  // ---- parameters -> LDS images (padding zero), Adam moments -> owner registers
  // Zero ALL of the LDS images once: padding entries (weight rows / columns past the layer
  // dims, unwritten input-image columns, normaliser entries of padding features) then stay
  // exactly 0, so padded dW / bias entries come out 0 without per-lane masks.
  for (int i = tid; i < g.lds_floats; i += kThreads) L[i] = 0.f;
  __syncthreads();
#pragma unroll
  for (int qq = 0; qq < 2; ++qq) {
#pragma unroll
    for (int l = 0; l < kL; ++l) {
      // (net split: the other net's images alias this one's -- only net q is loaded)
      if (l >= (qq == 0 ? a.n_pi : a.n_vf) || (ns && qq != q)) continue;
      const LG y = lg(g, qq, l);
      const int wo = qq == 0 ? a.pi_w_off[l] : a.vf_w_off[l];
      const int bo = qq == 0 ? a.pi_b_off[l] : a.vf_b_off[l];
      for (int i = tid; i < y.dout * y.din; i += kThreads) {
        const int o = i / y.din, c = i - o * y.din;
        if constexpr (BF3) bf3_store_w<KT>(L, g, qq, l, o, c, a.params[wo + i], qq == 0 ? a.n_pi : a.n_vf);
        else L[y.w + o * y.ldw + c] = a.params[wo + i];
      }
      for (int i = tid; i < y.dout; i += kThreads) L[y.b + i] = a.params[bo + i];
    }
  }
  if (tid < 16) L[g.ls_off + tid] = (has_ls && tid < A && !(ns && q != 0)) ? a.params[a.log_std_off + tid] : 0.f;
  // normaliser running state (double-buffered per-minibatch mean / rstd)
  // (owned by wave 7, one lane per feature)
  const int nc = tid - (kThreads - 64);
  const bool norm_lane = a.has_norm && nc >= 0 && nc < D;
  float run_m = 0.f, run_v = 1.f, run_c = 0.f;
  if (norm_lane) {
    run_m = a.norm_mean[nc];
    run_v = a.norm_var[nc];
    run_c = a.norm_count_i ? (float)a.norm_count_i[0] : a.norm_count[0];
  }
  // owned items: gradient / moments registers. Weight slot it of this wave is item
  // wb + w + it * NW (valid below nwq), bias slot ib is item bb + w + ib * NW (valid below nbq).
  const int n_witems = rfl(g.n_witems);
  const int wb = ns ? rfl(g.wbase[q]) : 0, nwq = ns ? rfl(g.nwit[q]) : n_witems;
  const int bb = ns ? rfl(g.bbase[q]) : n_witems, nbq = ns ? rfl(g.nbit[q]) : n_items - n_witems;
  float gm[KW][4], gv[KW][4];  // weight tiles: Adam moments
  f4 gg[KW];                   // and gradient (the dW MFMA chains accumulate into it)
  float wmst[BF3 ? KW : 1][4];  // BF3: the fp32 master weights of the owned tiles (no fp32 LDS image)
  float bm[KB], bv[KB], bg[KB];           // bias / log_std vectors
#pragma unroll
  for (int it = 0; it < KW; ++it) {
#pragma unroll
    for (int j = 0; j < 4; ++j) gm[it][j] = gv[it][j] = 0.f;
    gg[it] = {0.f, 0.f, 0.f, 0.f};
    if (w + it * kWaves < nwq) {
      const int desc = rfl(g.items[wb + w + it * kWaves]);
      const int iq = desc & 1, il = (desc >> 1) & 3, ta = (desc >> 5) & 15, tb = (desc >> 9) & 15;
      const int din = g.din[iq][il], dout = g.dout[iq][il];
      const int wo = iq == 0 ? a.pi_w_off[il] : a.vf_w_off[il];
      const int in = 16 * tb + r16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = 16 * ta + 4 * kk + j;
        if constexpr (BF3) wmst[it][j] = 0.f;
        if (o < dout && in < din) {
          gm[it][j] = a.exp_avg[wo + o * din + in];
          gv[it][j] = a.exp_avg_sq[wo + o * din + in];
          if constexpr (BF3) wmst[it][j] = a.params[wo + o * din + in];
        }
      }
    }
  }
#pragma unroll
  for (int ib = 0; ib < KB; ++ib) {
    bm[ib] = bv[ib] = bg[ib] = 0.f;
    if (w + ib * kWaves < nbq) {
      const int desc = rfl(g.items[bb + w + ib * kWaves]);
      const int iq = desc & 1, il = (desc >> 1) & 3, kind = (desc >> 3) & 3;
      if (kind == 1) {
        const int dout = g.dout[iq][il];
        const int bo = iq == 0 ? a.pi_b_off[il] : a.vf_b_off[il];
        if (lane < dout) {
          bm[ib] = a.exp_avg[bo + lane];
          bv[ib] = a.exp_avg_sq[bo + lane];
        }
      } else if (has_ls && lane < A) {
        bm[ib] = a.exp_avg[a.log_std_off + lane];
        bv[ib] = a.exp_avg_sq[a.log_std_off + lane];
      }
    }
  }
  // stats accumulators (per lane; one lane per row contributes)
  float st_ent = 0.f, st_pg = 0.f, st_vl = 0.f, st_cf = 0.f, st_kl = 0.f;
  float step = a.adam_step[0];
  float b1t = powf(a.beta1, step), b2t = powf(a.beta2, step);
  const int hid_act = ACTT >= 0 ? ACTT : a.hidden_act;
  // first minibatch norm stats
  if (norm_lane && K > 0) {
    const float m = g.mom[nc], v = g.mom[64 + nc], n = (float)Bg;
    const float tot = run_c + n, delta = m - run_m;
    run_m += delta * n / tot;
    run_v = (run_v * run_c + v * n + delta * delta * run_c * n / tot) / tot;
    run_c = tot;
    L[g.nm_off + nc] = run_m;
    L[g.nm_off + 64 + nc] = rsqrtf(run_v + a.norm_eps);
  }
  // dW item operands: this wave's valid weight slots are its first nwi (ids < n_witems);
  // the LDS offsets of a slot's dZ / H columns are a wave-uniform base (the descriptor) plus
  // ONE lane term shared by every slot (all K-major images have the row stride cw + 4)
  const int nwi = nwq > w ? min(KW, (nwq - w + kWaves - 1) / kWaves) : 0;
  // floats per column of the split-bf16 K-major images (ppo_rc_plan: max(cw, 32) + 4) and the
  // 32-row K-steps of a dW tile: compile-time under a fixed chunk width (offsets fold into the
  // ds_read immediates)
  constexpr int kRowsPad = CWT > 32 ? CWT : 32;
  const int cs = CWT > 0 ? kRowsPad + 4 : rfl(g.ldz[0][0]);
  const int ksteps = CWT > 0 ? kRowsPad / 32 : rfl(g.ksteps);
  const int lterm = r16 * 2 * cs + 8 * kk;  // bf16 offset of this lane's first dW operand
  // Per-slot wave-uniform LDS bases: the descriptor and layer tables are kernel-argument arrays,
  // so each dynamically indexed use is a dependent scalar-load chain. The 4-wave builds with at
  // most 8 weight slots resolve them once (HOIST); the 8-wave ones (256 VGPRs, no AGPRs) and the
  // 12 / 14-slot ones (full register file) re-resolve them per use.
  // slot_dw: the slot's dZ / H operand bases (bf16; + lterm per lane).
  // slot_img (BF3, Adam's image stores): forward image base (+ the lane term of the layer kind:
  // 0 input layer, 1 hidden, 2 head) and its lo-half offset; transposed image base / lo offset.
  constexpr bool HOIST = NW == 4 && KW <= 8;
  auto slot_dw = [&](int it, int& zu, int& hu) {
    const int desc = rfl(g.items[wb + w + it * kWaves]);
    const int iq = desc & 1, il = (desc >> 1) & 3, ta = (desc >> 5) & 15, tb = (desc >> 9) & 15;
    zu = 2 * rfl(g.z_off[iq][il]) + 16 * ta * 2 * cs;
    hu = 2 * rfl(g.h_off[iq][il]) + 16 * tb * 2 * cs;
  };
  auto slot_img = [&](int it, int& kd, int& wf, int& wl, int& wt, int& tl) {
    const int desc = rfl(g.items[wb + w + it * kWaves]);
    const int iq = desc & 1, il = (desc >> 1) & 3, ta = (desc >> 5) & 15, tb = (desc >> 9) & 15;
    const int nlq = iq == 0 ? a.n_pi : a.n_vf;
    const int ldi = bf3_ld(il == 0 ? 32 : 16 * KT);
    wf = rfl(2 * g.wf_off[iq][il] + 16 * ta * ldi + (il == 0 ? 4 * tb : 32 * (tb >> 1) + 4 * (tb & 1)));
    wl = rfl(((g.dout[iq][il] + 15) & ~15) * ldi);
    kd = il == 0 ? 0 : (il == nlq - 1 ? 2 : 1);
    wt = tl = 0;
    if (il > 0) {
      const int ldo = bf3_ld(il == nlq - 1 ? 32 : 16 * KT);
      wt = rfl(2 * g.wt_off[iq][il] + 16 * tb * ldo + 32 * (ta >> 1) + 4 * (ta & 1));
      tl = rfl(((g.din[iq][il] + 15) & ~15) * ldo);
    }
  };
  // this wave's net geometry per layer (fwd / bwd chains, loss), resolved once for the fully
  // specialised HOIST builds (GHOIST); the rest index the argument tables per use
  constexpr bool GHOIST = HOIST && NLT > 0;
  LG yq[GHOIST ? kL : 1];
  int wfq[GHOIST && BF3 ? kL : 1], wtq[GHOIST && BF3 ? kL : 1];
#pragma unroll
  for (int l = 0; l < kL; ++l) {
    if (!GHOIST || l >= nl) continue;
    yq[GHOIST ? l : 0] = lg(g, q, l);
    if constexpr (BF3) {
      wfq[GHOIST ? l : 0] = rfl(g.wf_off[q][l]);
      wtq[GHOIST ? l : 0] = rfl(g.wt_off[q][l]);
    }
  }
  auto LY = [&](int l) -> LG {
    if constexpr (GHOIST) return yq[GHOIST ? l : 0];
    else return lg(g, q, l);
  };
  auto WF = [&](int l) -> int {
    if constexpr (GHOIST && BF3) return wfq[GHOIST ? l : 0];
    else return rfl(g.wf_off[q][l]);
  };
  auto WT = [&](int l) -> int {
    if constexpr (GHOIST && BF3) return wtq[GHOIST ? l : 0];
    else return rfl(g.wt_off[q][l]);
  };
  constexpr int KH = HOIST ? KW : 1, KHB = HOIST && BF3 ? KW : 1;
  int izu[KH], ihu[KH];
  int bwf[KHB], bwt[KHB], bpk[KHB];  // bpk: kind | lo offsets << 2 / << 17 (each < 2^15)
#pragma unroll
  for (int it = 0; it < KH; ++it) {
    izu[it] = ihu[it] = 0;
    if (HOIST && it < nwi) slot_dw(it, izu[it], ihu[it]);
  }
#pragma unroll
  for (int it = 0; it < KHB; ++it) {
    bwf[it] = bwt[it] = bpk[it] = 0;
    if (HOIST && BF3 && it < nwi) {
      int kd, wl, tl;
      slot_img(it, kd, bwf[it], wl, bwt[it], tl);
      bpk[it] = kd | (wl << 2) | (tl << 17);
    }
  }
  // bias / log_std slots: kind (1 bias, 2 log_std, -1 empty), partial source, element mask
  int bkind[KB], b_off[KB], b_addr[KB];
  float b_okf[KB];  // 1 for lanes holding a real bias / log_std element
#pragma unroll
  for (int ib = 0; ib < KB; ++ib) {
    bkind[ib] = -1;
    b_off[ib] = 0;
    b_okf[ib] = 0.f;
    b_addr[ib] = g.trash_off + lane;
    if (w + ib * kWaves >= nbq) continue;
    const int desc = rfl(g.items[bb + w + ib * kWaves]);
    const int iq = desc & 1, il = (desc >> 1) & 3, kind = (desc >> 3) & 3;
    const LG y = lg(g, iq, il);
    bkind[ib] = kind;
    b_off[ib] = kind == 1 ? y.db : g.lsp_off;
    const bool ok = kind == 1 ? (lane < y.dout) : (has_ls && lane < A);
    b_okf[ib] = ok ? 1.f : 0.f;
    if (ok) b_addr[ib] = kind == 1 ? y.b + lane : g.ls_off + lane;
  }
  float pre_m = 0.f, pre_v = 0.f;  // moments of the next minibatch to merge
  if (norm_lane && K > 1) {
    pre_m = g.mom[128 + nc];
    pre_v = g.mom[128 + 64 + nc];
  }
  Rows<S0M> cur;
  const int row = 16 * gw + r16;
  // chunk unit u = k * nch + ch -> prep slot k * CH + grp * nch + ch
  auto slot_of = [&](int u) -> size_t { return (size_t)(u / nch) * CH + (size_t)grp * nch + (u % nch); };
  if (rows_wave && K > 0) load_rows(g, slot_of(0), row, kk, s0, cur);
  // cycle counters (a.prof): accumulated in LDS by one lane, so that they hold no registers
  // across the minibatch loop. [0..2] chunk, exchange + |g|^2, clip + Adam (wave 0);
  // [3..6] / [7..10] actor / critic row tile 0: rows/x, forward, loss, backward chain;
  // [11] wave 0 B1 wait, [12] dW items; [13..15] exchange: publish, arrival, loads;
  // [16] net-split |g|^2 hand-off, [17] Adam on the owned items (wave 0), [18] B3 wait
  __shared__ unsigned long long sprof[20];
  if (tid < 20) sprof[tid] = 0;
  // arrival counters per net under the net split ([0]/[2] actor, [4]/[6] critic)
  unsigned* arrive = g.sync + (ns ? 4 * q : 0);
  unsigned* tflag = g.sync + 1;
  unsigned* arrive2 = g.sync + (ns ? 4 * q + 2 : 2);
  const unsigned spin_lim = a.spin_limit ? a.spin_limit : (1u << 22);
  // test knob: the last working workgroup never publishes, so its partners' spins time out
  const bool stall = a.debug_stall != 0 && bid == (ns ? 2 * G : G) - 1;
  __syncthreads();

  // normalised input of this lane's row (cur) with normaliser buffer nbuf -> xo, and the
  // layer-0 input image for dW (padding features: raw value 0 from the prep kernel, normaliser
  // image entries 0)
  auto norm_rows = [&](int nbuf, float (&xo)[S0M]) {
    float nmv[S0M], nrv[S0M];
#pragma unroll
    for (int s = 0; s < S0M; ++s) {
      nmv[s] = 0.f;
      nrv[s] = 1.f;
      if (s < s0 && a.has_norm) {
        nmv[s] = L[g.nm_off + nbuf + 4 * s + kk];
        nrv[s] = L[g.nm_off + nbuf + 64 + 4 * s + kk];
      }
    }
#pragma unroll
    for (int s = 0; s < S0M; ++s) xo[s] = s < s0 ? (cur.x[s] - nmv[s]) * nrv[s] : 0.f;
    if (q == 0 || ns) {  // shared layer-0 input image (each workgroup its own under net split)
      const int h0 = rfl(g.h_off[0][0]);
#pragma unroll
      for (int s = 0; s < S0M; ++s)
        if (s < s0) img_store(L, h0, cs, 4 * s + kk, row, xo[s]);
    }
  };
  // pre_rows: under the exchange (G > 1) or the net split, chunk 0 of minibatch k+1 is
  // normalised while this workgroup waits for its partners (arrival / |g|^2 hand-off): its
  // rows are in cur since the last chunk, its normaliser buffer was merged after this
  // minibatch's B1, and every dW read of the layer-0 image is behind the barrier before it
  // (not the 12 / 14-slot builds: their register file is full; not with the G > 16 partial
  // stash, which borrows the activation images -- the layer-0 input image included -- during
  // the exchange)
  constexpr bool PREC = KW <= 8;
  const bool pre = PREC && (ns || G > 1) && g.xstash < 0;
  float xpre[PREC ? S0M : 1];
#pragma unroll
  for (int s = 0; s < (PREC ? S0M : 1); ++s) xpre[s] = 0.f;
  auto pre_rows = [&](int k) {
    if constexpr (PREC)
      if (pre && rows_wave && k + 1 < K) norm_rows(((k + 1) & 1) * 128, xpre);
  };

  for (int k = 0; k < K; ++k) {
    unsigned long long t0 = a.prof ? clock64() : 0;
    const int nb = (k & 1) * 128;  // norm buffer of minibatch k
#pragma unroll
    for (int it = 0; it < KW; ++it) gg[it] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ib = 0; ib < KB; ++ib) bg[ib] = 0.f;
    for (int ch = 0; ch < nch; ++ch) {
      const int u = k * nch + ch;
      Rows<S0M> nxt;
      if (rows_wave && u + 1 < K * nch) load_rows(g, slot_of(u + 1), row, kk, s0, nxt);
      // moments of minibatch k+1 (prefetched one minibatch earlier) -> registers; issue k+2
      float mom_m = 0.f, mom_v = 0.f;
      if (ch == 0 && norm_lane) {
        mom_m = pre_m;
        mom_v = pre_v;
        if (k + 2 < K) {
          pre_m = g.mom[(size_t)(k + 2) * 128 + nc];
          pre_v = g.mom[(size_t)(k + 2) * 128 + 64 + nc];
        }
      }
      unsigned long long c0 = a.prof ? clock64() : 0;
      if (rows_wave) {
        // ---------------- normalised input: B operand of layer 0 (natural K order 4s + kk)
        // (chunk 0 of minibatch k > 0 under the exchange / net split: done in minibatch k-1's
        // waiting window, see pre_rows)
        float xb[S0M];
        if constexpr (PREC) {
          if (pre && ch == 0 && k > 0) {
#pragma unroll
            for (int s = 0; s < S0M; ++s) xb[s] = xpre[s];
          } else {
            norm_rows(nb, xb);
          }
        } else {  // (the same as norm_rows, inline: the full-register-file builds stay spill-free)
          float nmv[S0M], nrv[S0M];
#pragma unroll
          for (int s = 0; s < S0M; ++s) {
            nmv[s] = 0.f;
            nrv[s] = 1.f;
            if (s < s0 && a.has_norm) {
              nmv[s] = L[g.nm_off + nb + 4 * s + kk];
              nrv[s] = L[g.nm_off + nb + 64 + 4 * s + kk];
            }
          }
#pragma unroll
          for (int s = 0; s < S0M; ++s) xb[s] = s < s0 ? (cur.x[s] - nmv[s]) * nrv[s] : 0.f;
          if (q == 0 || ns) {
            const int h0 = rfl(g.h_off[0][0]);
#pragma unroll
            for (int s = 0; s < S0M; ++s)
              if (s < s0) img_store(L, h0, cs, 4 * s + kk, row, xb[s]);
          }
        }
        unsigned long long c1 = a.prof ? clock64() : 0;
        // ---------------- forward (registers)
        f4 hreg[kL - 1][KT];  // outputs of hidden layers (C layout), kept for act'
        f4 head = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int l = 0; l < kL; ++l) {
          if (l >= nl) continue;
          const LG y = LY(l);
          const bool last = l == nl - 1;
          const int tout = last ? 1 : (HWT > 0 ? HWT / 16 : ((y.dout + 15) >> 4));  // head: dout <= 16
          // all of the layer's weight operands are read first, then the output tiles'
          // MFMA chains run interleaved (same accumulation order per tile as one chain)
          f4 acc[KT];
#pragma unroll
          for (int t = 0; t < KT; ++t) acc[t] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (BF3) {
            // B operand per 32 of K: this lane's 8 inputs (layer 0: features 4 s + kk; hidden: the
            // C layout of the previous layer's tiles 2 s, 2 s + 1), split into bf16 hi / lo
            constexpr int KS = KT / 2;
            const int ks_l = l == 0 ? 1 : KS;
            const int kin = l == 0 ? 32 : 16 * KT;
            const int rows = (y.dout + 15) & ~15;
            const lbf* wf = (const lbf*)(L + WF(l)) + r16 * bf3_ld(kin) + 8 * kk;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              if (ks >= ks_l) continue;
              float v[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                if (l == 0) v[j] = j < S0M ? xb[j < S0M ? j : 0] : 0.f;
                else v[j] = hreg[l > 0 ? l - 1 : 0][2 * ks + (j >> 2)][j & 3];
              }
              bf16x8 bh, bl;
              split8(v, bh, bl);
#pragma unroll
              for (int t = 0; t < KT; ++t)
                if (t < tout) acc[t] = bf3_tile(wf + 16 * t * bf3_ld(kin) + 32 * ks, rows * bf3_ld(kin), bh, bl, acc[t]);
            }
          } else if (l == 0 && KT > 2) {  // 64-wide: two tiles' operands at a time (register budget)
#pragma unroll
            for (int t0 = 0; t0 < KT; t0 += 2) {
              float w0[2][S0M];
#pragma unroll
              for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int s = 0; s < S0M; ++s)
                  if (t0 + t < tout && s < s0) w0[t][s] = L[y.w + (16 * (t0 + t) + r16) * y.ldw + 4 * s + kk];
#pragma unroll
              for (int s = 0; s < S0M; ++s)
#pragma unroll
                for (int t = 0; t < 2; ++t)
                  if (t0 + t < tout && s < s0) acc[t0 + t] = mfma(w0[t][s], xb[s], acc[t0 + t]);
            }
          } else if (l == 0) {
            float w0[KT][S0M];
#pragma unroll
            for (int t = 0; t < KT; ++t)
#pragma unroll
              for (int s = 0; s < S0M; ++s)
                if (t < tout && s < s0) w0[t][s] = L[y.w + (16 * t + r16) * y.ldw + 4 * s + kk];
#pragma unroll
            for (int s = 0; s < S0M; ++s)
#pragma unroll
              for (int t = 0; t < KT; ++t)
                if (t < tout && s < s0) acc[t] = mfma(w0[t][s], xb[s], acc[t]);
          } else if constexpr (KT > 2) {  // 64-wide: one tile at a time (register budget)
            const int tin = HWT > 0 ? HWT / 16 : ((y.din + 15) >> 4);
#pragma unroll
            for (int t = 0; t < KT; ++t) {
              if (t >= tout) continue;
              const lf* wr = L + y.w + (16 * t + r16) * y.ldw;
#pragma unroll
              for (int h = 0; h < KT; ++h) {
                if (h >= tin) continue;
                const f4 w4 = *(const lf4*)(wr + 16 * h + 4 * kk);
                acc[t] = mfma(w4.x, hreg[l - 1][h].x, acc[t]);
                acc[t] = mfma(w4.y, hreg[l - 1][h].y, acc[t]);
                acc[t] = mfma(w4.z, hreg[l - 1][h].z, acc[t]);
                acc[t] = mfma(w4.w, hreg[l - 1][h].w, acc[t]);
              }
            }
          } else {
            const int tin = HWT > 0 ? HWT / 16 : ((y.din + 15) >> 4);
            f4 w4[KT][KT];
#pragma unroll
            for (int t = 0; t < KT; ++t)
#pragma unroll
              for (int h = 0; h < KT; ++h)
                if (t < tout && h < tin) w4[t][h] = *(const lf4*)(L + y.w + (16 * t + r16) * y.ldw + 16 * h + 4 * kk);
#pragma unroll
            for (int h = 0; h < KT; ++h) {
#pragma unroll
              for (int t = 0; t < KT; ++t) {
                if (t >= tout || h >= tin) continue;
                acc[t] = mfma(w4[t][h].x, hreg[l - 1][h].x, acc[t]);
                acc[t] = mfma(w4[t][h].y, hreg[l - 1][h].y, acc[t]);
                acc[t] = mfma(w4[t][h].z, hreg[l - 1][h].z, acc[t]);
                acc[t] = mfma(w4[t][h].w, hreg[l - 1][h].w, acc[t]);
              }
            }
          }
#pragma unroll
          for (int t = 0; t < KT; ++t) {
            if (t >= tout) continue;
            const int o0 = 16 * t + 4 * kk;
            const f4 bb = *(const lf4*)(L + y.b + o0);
            f4 v;
            v.x = acc[t].x + bb.x;
            v.y = acc[t].y + bb.y;
            v.z = acc[t].z + bb.z;
            v.w = acc[t].w + bb.w;
            if (!last) {
              v.x = (HWT > 0 || o0 + 0 < y.dout) ? act_fn(hid_act, v.x) : 0.f;
              v.y = (HWT > 0 || o0 + 1 < y.dout) ? act_fn(hid_act, v.y) : 0.f;
              v.z = (HWT > 0 || o0 + 2 < y.dout) ? act_fn(hid_act, v.z) : 0.f;
              v.w = (HWT > 0 || o0 + 3 < y.dout) ? act_fn(hid_act, v.w) : 0.f;
              if (l < kL - 1) {
                hreg[l][t] = v;
                // input image of layer l + 1 (for its dW)
                const LG yn = LY(l + 1);
                img_store(L, yn.h, cs, o0, row, v.x);
                img_store(L, yn.h, cs, o0 + 1, row, v.y);
                img_store(L, yn.h, cs, o0 + 2, row, v.z);
                img_store(L, yn.h, cs, o0 + 3, row, v.w);
              }
            } else if (t == 0) {
              head = v;
            }
          }
        }
        unsigned long long c2 = a.prof ? clock64() : 0;
        // ---------------- loss -> dZ of the head (C layout, tile 0)
        f4 dz = {0.f, 0.f, 0.f, 0.f};
        const LG yh = LY(nl - 1);
        if (q == 0) {
          const float ao[4] = {cur.act.x, cur.act.y, cur.act.z, cur.act.w};
          const float hv[4] = {head.x, head.y, head.z, head.w};
          float dzv[4] = {0.f, 0.f, 0.f, 0.f};
          const float old_lp = cur.rd.x, adv = cur.rd.y;
          float logp, ent_row = 0.f;
          int act_row = 0;
          float pk[4] = {0.f, 0.f, 0.f, 0.f}, lpk[4] = {0.f, 0.f, 0.f, 0.f};
          float zs[4] = {0.f, 0.f, 0.f, 0.f}, isd[4] = {0.f, 0.f, 0.f, 0.f};
          if (gauss) {
            // branch-free over the 4 action slots of this lane group: padding slots have
            // log_std 0, action 0 and mean 0 (zero weight rows), so zs = 0 there and only the
            // constant term needs the slot mask am[j]
            float part = 0.f;
            const f4 ls4 = *(const lf4*)(L + g.ls_off + 4 * kk);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float lsv = ls4[j];
              isd[j] = __expf(-lsv);
              zs[j] = (ao[j] - hv[j]) * isd[j];
              part += am[j] * (-0.5f * zs[j] * zs[j] - lsv - c_half_log2pi);
            }
            logp = sum_kk(part);
          } else {
            const int n = yh.dout;
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (4 * kk + j < n) mx = fmaxf(mx, hv[j]);
            mx = max_kk(mx);
            float zsum = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (4 * kk + j < n) zsum += expf(hv[j] - mx);
            const float lz = logf(sum_kk(zsum));
            act_row = __shfl((int)cur.act.x, r16);  // lane group 0 holds the action index
            float sel = 0.f, ent = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int o = 4 * kk + j;
              if (o < n) {
                lpk[j] = hv[j] - mx - lz;
                pk[j] = expf(lpk[j]);
                ent -= pk[j] * lpk[j];
                if (o == act_row) sel = lpk[j];
              }
            }
            logp = sum_kk(sel);
            ent_row = sum_kk(ent);
          }
          const float lr_ = logp - old_lp;
          const float ratio = expf(lr_);
          const float lo = 1.f - a.clip_range, hi = 1.f + a.clip_range;
          const float pl1 = adv * ratio, pl2 = adv * fminf(fmaxf(ratio, lo), hi);
          float c1, c2;  // torch.min routes the gradient to the smaller operand, half each on ties
          if (pl1 < pl2) { c1 = 1.f; c2 = 0.f; } else if (pl2 < pl1) { c1 = 0.f; c2 = 1.f; } else { c1 = 0.5f; c2 = 0.5f; }
          const float inside = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
          const float dlogp = -invB * (c1 * adv + c2 * adv * inside) * ratio;
          if (gauss) {
            float lsp[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int o = 4 * kk + j;
              dzv[j] = dlogp * zs[j] * isd[j];
              lsp[j] = am[j] * dlogp * (zs[j] * zs[j] - 1.f);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float s = sum16(lsp[j]);
              if (r16 == 0) L[g.lsp_off + gw * 16 + 4 * kk + j] = s;
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int o = 4 * kk + j;
              dzv[j] = o < yh.dout ? dlogp * ((o == act_row ? 1.f : 0.f) - pk[j]) -
                                         a.ent_coef * invB * (-pk[j] * (lpk[j] + ent_row))
                                   : 0.f;
            }
          }
          dz = {dzv[0], dzv[1], dzv[2], dzv[3]};
          if (kk == 0) {
            st_pg += -fminf(pl1, pl2);
            st_cf += fabsf(ratio - 1.f) > a.clip_range ? 1.f : 0.f;
            st_kl += (ratio - 1.f) - lr_;
            if (!gauss) st_ent += -ent_row;
          }
        } else {
          float d = 0.f;
          if (kk == 0) {
            d = head.x - cur.rd.z;
            st_vl += d * d;
          }
          dz = {kk == 0 ? a.vf_coef * 2.f * d * invB : 0.f, 0.f, 0.f, 0.f};
        }
        unsigned long long c3 = a.prof ? clock64() : 0;
        // ---------------- backward chain: store dZ_l, bias partials, dZ_{l-1} = W_l^T dZ_l * act'
        f4 dzc[KT];
        dzc[0] = dz;
#pragma unroll
        for (int t = 1; t < KT; ++t) dzc[t] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int l = kL - 1; l >= 0; --l) {
          if (l >= nl) continue;
          const LG y = LY(l);
          const int tout = l == nl - 1 ? 1 : (HWT > 0 ? HWT / 16 : ((y.dout + 15) >> 4));
          const int tin = HWT > 0 ? HWT / 16 : ((y.din + 15) >> 4);
          // W_l^T operands (W[16 tt + 4 kk + j][16 u2 + r16]) read before this layer's
          // image stores, so the loads are not ordered behind them
          constexpr int KWT = KT > 2 ? 1 : KT;  // 64-wide: W^T read per tile below (register budget)
          float wt[KWT][KWT][4];
          if (!BF3 && KT <= 2 && l > 0) {
#pragma unroll
            for (int u2 = 0; u2 < KT; ++u2)
#pragma unroll
              for (int tt = 0; tt < KT; ++tt)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                  if (u2 < tin && tt < tout) wt[u2 % KWT][tt % KWT][j] = L[y.w + (16 * tt + 4 * kk + j) * y.ldw + 16 * u2 + r16];
          }
#pragma unroll
          for (int u2 = 0; u2 < KT; ++u2) {
            if (u2 >= tout) continue;
            const int zc = 16 * u2 + 4 * kk;
            img_store(L, y.z, cs, zc, row, dzc[u2].x);
            img_store(L, y.z, cs, zc + 1, row, dzc[u2].y);
            img_store(L, y.z, cs, zc + 2, row, dzc[u2].z);
            img_store(L, y.z, cs, zc + 3, row, dzc[u2].w);
            const float s0v = sum16(dzc[u2].x), s1v = sum16(dzc[u2].y), s2v = sum16(dzc[u2].z), s3v = sum16(dzc[u2].w);
            if (r16 == 0) {
              const f4 sv = {s0v, s1v, s2v, s3v};
              *(lf4*)(L + y.db + gw * 64 + 16 * u2 + 4 * kk) = sv;
            }
          }
          if (l == 0) break;
          // the input tiles' chains interleaved (per tile: tt, j ascending as one chain)
          f4 accb[KT];
#pragma unroll
          for (int u2 = 0; u2 < KT; ++u2) accb[u2] = {0.f, 0.f, 0.f, 0.f};
          if constexpr (BF3) {
            // B operand per 32 of K: this lane's dZ of output tiles 2 s, 2 s + 1 (head: tile 0 and
            // zeros); A: the transposed split-bf16 image [in][pos_h(out)]
            constexpr int KS = KT / 2;
            const bool head = l == nl - 1;
            const int ks_l = head ? 1 : KS;
            const int kout = head ? 32 : 16 * KT;
            const int trows = (y.din + 15) & ~15;
            const lbf* wt_img = (const lbf*)(L + WT(l)) + r16 * bf3_ld(kout) + 8 * kk;
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
              if (ks >= ks_l) continue;
              float v[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = (2 * ks + (j >> 2)) < tout ? dzc[2 * ks + (j >> 2)][j & 3] : 0.f;
              bf16x8 bh, bl;
              split8(v, bh, bl);
#pragma unroll
              for (int u2 = 0; u2 < KT; ++u2)
                if (u2 < tin) accb[u2] = bf3_tile(wt_img + 16 * u2 * bf3_ld(kout) + 32 * ks, trows * bf3_ld(kout), bh, bl, accb[u2]);
            }
          } else if constexpr (KT <= 2) {
#pragma unroll
            for (int tt = 0; tt < KT; ++tt)
#pragma unroll
              for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int u2 = 0; u2 < KT; ++u2)
                  if (u2 < tin && tt < tout) accb[u2] = mfma(wt[u2 % KWT][tt % KWT][j], dzc[tt][j], accb[u2]);
          } else {
#pragma unroll
            for (int u2 = 0; u2 < KT; ++u2) {
              if (u2 >= tin) continue;
#pragma unroll
              for (int tt = 0; tt < KT; ++tt) {
                if (tt >= tout) continue;
                const lf* wc = L + y.w + (16 * tt + 4 * kk) * y.ldw + 16 * u2 + r16;
                accb[u2] = mfma(wc[0], dzc[tt].x, accb[u2]);
                accb[u2] = mfma(wc[y.ldw], dzc[tt].y, accb[u2]);
                accb[u2] = mfma(wc[2 * y.ldw], dzc[tt].z, accb[u2]);
                accb[u2] = mfma(wc[3 * y.ldw], dzc[tt].w, accb[u2]);
              }
            }
          }
          f4 nd[KT];
#pragma unroll
          for (int u2 = 0; u2 < KT; ++u2) {
            nd[u2] = {0.f, 0.f, 0.f, 0.f};
            if (u2 >= tin) continue;
            const f4 acc = accb[u2];
            const f4 hv = hreg[l > 0 ? l - 1 : 0][u2];
            nd[u2].x = acc.x * act_grad(hid_act, hv.x);
            nd[u2].y = acc.y * act_grad(hid_act, hv.y);
            nd[u2].z = acc.z * act_grad(hid_act, hv.z);
            nd[u2].w = acc.w * act_grad(hid_act, hv.w);
          }
#pragma unroll
          for (int u2 = 0; u2 < KT; ++u2) dzc[u2] = nd[u2];
        }
        if (a.prof && lane == 0 && gw == 0) {
          const unsigned long long c4 = clock64();
          const int pb = q == 1 ? 7 : 3;
          sprof[pb + 0] += c1 - c0;
          sprof[pb + 1] += c2 - c1;
          sprof[pb + 2] += c3 - c2;
          sprof[pb + 3] += c4 - c3;
        }
      }
      const unsigned long long cb0 = a.prof ? clock64() : 0;
      __syncthreads();  // B1: H / dZ images, bias and log-std partials of this chunk complete
      const unsigned long long cb1 = a.prof ? clock64() : 0;
      // Chan merge for minibatch k+1 (one lane per feature, wave 7), off the chain's critical
      // path; minibatch k reads the other half of the double-buffered normaliser image
      if (ch == 0 && norm_lane && k + 1 < K) {
        const float n = (float)Bg;
        const float tot = run_c + n, delta = mom_m - run_m;
        run_m += delta * n / tot;
        run_v = (run_v * run_c + mom_v * n + delta * delta * run_c * n / tot) / tot;
        run_c = tot;
        L[g.nm_off + (128 - nb) + nc] = run_m;
        L[g.nm_off + (128 - nb) + 64 + nc] = rsqrtf(run_v + a.norm_eps);
      }

      // ---------------- dW / db / dlog_std partials of this chunk for the owned items
      {
        int izo[KW], iho[KW];
#pragma unroll
        for (int it = 0; it < KW; ++it) {
          izo[it] = iho[it] = 2 * g.zero_off;  // (bf16 units: the zero row)
          if (it < nwi) {
            int zu, hu;
            if constexpr (HOIST) {
              zu = izu[it];
              hu = ihu[it];
            } else {
              slot_dw(it, zu, hu);
            }
            izo[it] = zu + lterm;
            iho[it] = hu + lterm;
          }
        }
        // the chunk's dZ^T H continues each slot's MFMA chain from its running gradient
        // (padding entries are exactly 0: zeroed images)
        // (empty slots read the zero row: their MFMAs add zeros to gradients nobody reads,
        // so every wave runs the same straight-line body)
        dw_tiles<KW>(L, izo, iho, img_lo(cs), ksteps, gg);
      }
#pragma unroll
      for (int ib = 0; ib < KB; ++ib) {
        if (bkind[ib] <= 0) continue;
        {  // bias (row-tile partials of dZ) / log_std (partials of the Gaussian term)
          const int stride = bkind[ib] == 1 ? 64 : 16;
          float gval = 0.f;  // (lanes past the vector read finite neighbours, masked by b_okf)
          for (int r = 0; r < RT; ++r) gval += L[b_off[ib] + r * stride + lane];
          bg[ib] += gval * b_okf[ib];
        }
      }
      if (a.prof && tid == 0) {
        sprof[11] += cb1 - cb0;
        sprof[12] += clock64() - cb1;
      }
      if (rows_wave) cur = nxt;
      if (ch + 1 < nch) __syncthreads();  // images are rewritten by the next chunk
    }
    unsigned long long t1 = a.prof ? clock64() : 0;

    // ---------------- cross-workgroup exchange of the partials (G > 1)
    if (G > 1) {
      // owned slots as one list: weight tiles, then bias / log_std vectors ({g, 0, 0, 0})
      int ids[KI];
      f4 xg[KI];
#pragma unroll
      for (int it = 0; it < KW; ++it) {
        ids[it] = it < nwi ? wb + w + it * kWaves : -1;
        xg[it] = gg[it];
      }
#pragma unroll
      for (int ib = 0; ib < KB; ++ib) {
        ids[KW + ib] = bkind[ib] >= 0 ? bb + w + ib * kWaves : -1;
        xg[KW + ib] = {bg[ib], 0.f, 0.f, 0.f};
      }
      float* slab = g.slab + (size_t)(k & 1) * G * n_items * 256;
#pragma unroll
      for (int it = 0; it < KI; ++it) {
        if (ids[it] < 0) continue;
        st_sc1_x4(slab + ((size_t)grp * n_items + ids[it]) * 256 + lane * 4, xg[it]);
      }
      const unsigned long long e0 = a.prof ? clock64() : 0;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const unsigned long long e1 = a.prof ? clock64() : 0;
      if (tid == 0 && !stall) atomicAdd(arrive, 1u);
      pre_rows(k);
      if (tid == 0) {
        const unsigned target = (unsigned)G * (unsigned)(k + 1);
        unsigned spins = 0;
        while (ld_sc1u(arrive) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_lim || ld_sc1u(tflag) != 0u) {
            spin_give_up(a, tflag);
            break;
          }
        }
      }
      __syncthreads();
      const unsigned long long e2 = a.prof ? clock64() : 0;
      if (g.xchg2) {
        // Two-level exchange (large G): slot it of every wave is reduced by workgroup
        // it % G, so each wave of each workgroup sums ~KI / G of its slots over the G
        // partials -- group order, the same additions as the one-level sum -- and publishes
        // them; after a second arrival every workgroup reads the n_items reduced tiles once:
        // per-workgroup loads ~2 x n_items KB instead of G x n_items KB. The partial loads of
        // all the wave's reduced slots are issued back to back, 16 in flight per wait.
        float* red = g.red + (size_t)(k & 1) * n_items * 256;
        const size_t gs = (size_t)n_items * 256;
        const auto slot_id = [&](int sl) -> int {  // item id of owned slot sl (computed: no array lookup)
          if (sl < KW) return sl < nwi ? wb + w + sl * kWaves : -1;
          return w + (sl - KW) * kWaves < nbq ? bb + w + (sl - KW) * kWaves : -1;
        };
        if (G == 2) reduce_slots<2, KI>(slab, red, gs, grp, lane, slot_id);
        else if (G == 4) reduce_slots<4, KI>(slab, red, gs, grp, lane, slot_id);
        else if (G == 8) reduce_slots<8, KI>(slab, red, gs, grp, lane, slot_id);
        else if (G == 16) reduce_slots<16, KI>(slab, red, gs, grp, lane, slot_id);
        else if (g.xstash >= 0) {
          // G > 16: item j of this net's list (weight tiles, then vectors) is reduced by
          // workgroup j % G. Its G partials are split over the waves -- ONE load batch per
          // wave (<= 16 in flight) instead of G / 16 serial batches on one wave -- staged in
          // the activation images (idle between the last dW item and the next chunk; zeroed
          // again afterwards) and summed one element per lane in group order: the same additions as the one-level
          // sum, so the update stays bitwise plan-independent.
          lf* st = L + g.xstash;
          const int m = nwq + nbq;
          for (int j = grp; j < m; j += G) {
            const int id = j < nwq ? wb + j : bb + (j - nwq);
            const float* p = slab + (size_t)id * 256 + lane * 4;
            f4 v[16];
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int gi = w + e * kWaves;
              v[e] = {0.f, 0.f, 0.f, 0.f};
              if (gi < G) v[e] = ld_sc1_x4(p + (size_t)gi * gs);
            }
            wait_vm_n<16>(v);
#pragma unroll
            for (int e = 0; e < 16; ++e) {
              const int gi = w + e * kWaves;
              if (gi < G) *(lf4*)(st + gi * 256 + lane * 4) = v[e];
            }
            __syncthreads();
            for (int el = tid; el < 256; el += kThreads) {
              float sacc = st[el];
#pragma unroll 8
              for (int gi = 1; gi < G; ++gi) sacc += st[gi * 256 + el];
              st_sc1_x1(red + (size_t)id * 256 + el, sacc);
            }
            __syncthreads();  // the stash is rewritten by the next item
          }
          // the images' padding rows / columns are read as zeros (zeroed once at kernel
          // start, never rewritten): restore them
          if (grp < m)
            for (int i = tid; i < G * 64; i += kThreads) *(lf4*)(st + 4 * i) = f4{0.f, 0.f, 0.f, 0.f};
        } else {  // G > 16 without a stash: slot it is reduced by workgroup it % G, 16 loads in flight
#pragma unroll
          for (int it = 0; it < KI; ++it) {
            const int id = ids[it];
            if (id < 0 || it % G != grp) continue;
            const float* p = slab + (size_t)id * 256 + lane * 4;
            f4 sacc = {0.f, 0.f, 0.f, 0.f};
            for (int gi0 = 0; gi0 < G; gi0 += 16) {
              f4 v[16];
#pragma unroll
              for (int e = 0; e < 16; ++e) v[e] = ld_sc1_x4(p + (size_t)(gi0 + e < G ? gi0 + e : 0) * gs);
              wait_vm_n<16>(v);
              if (gi0 == 0) sacc = v[0];
              else sacc += v[0];
#pragma unroll
              for (int e = 1; e < 16; ++e)
                if (gi0 + e < G) sacc += v[e];
            }
            st_sc1_x4(red + (size_t)id * 256 + lane * 4, sacc);
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
          if (!stall) atomicAdd(arrive2, 1u);
          const unsigned target = (unsigned)G * (unsigned)(k + 1);
          unsigned spins = 0;
          while (ld_sc1u(arrive2) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > spin_lim || ld_sc1u(tflag) != 0u) {
              spin_give_up(a, tflag);
              break;
            }
          }
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < KI; ++it) xg[it] = ld_sc1_x4(red + (size_t)(ids[it] >= 0 ? ids[it] : 0) * 256 + lane * 4);
        wait_vm_n<KI>(xg);  // results tied to the wait (inline-asm loads are invisible to the compiler)
      } else if (G == 2) {
        exchange_sum<2, KI>(slab, n_items, ids, lane, xg);
      } else if (G == 4) {
        exchange_sum<4, KI>(slab, n_items, ids, lane, xg);
      } else if (G == 8) {
        exchange_sum<8, KI>(slab, n_items, ids, lane, xg);
      } else {
#pragma unroll
        for (int it = 0; it < KI; ++it) {
          if (ids[it] < 0) continue;
          f4 sacc = {0.f, 0.f, 0.f, 0.f};
          const float* p = slab + (size_t)ids[it] * 256 + lane * 4;
          const size_t gs = (size_t)n_items * 256;
          for (int gi = 0; gi < G; gi += 4) {  // any count: tail lanes read group 0
            f4 v0 = ld_sc1_x4(p + (size_t)gi * gs);
            f4 v1 = ld_sc1_x4(p + (size_t)(gi + 1 < G ? gi + 1 : 0) * gs);
            f4 v2 = ld_sc1_x4(p + (size_t)(gi + 2 < G ? gi + 2 : 0) * gs);
            f4 v3 = ld_sc1_x4(p + (size_t)(gi + 3 < G ? gi + 3 : 0) * gs);
            wait_vm4(v0, v1, v2, v3);
            sacc += v0;
            if (gi + 1 < G) sacc += v1;
            if (gi + 2 < G) sacc += v2;
            if (gi + 3 < G) sacc += v3;
          }
          xg[it] = sacc;
        }
      }
#pragma unroll
      for (int it = 0; it < KW; ++it) {
        if (ids[it] < 0) continue;
        gg[it] = xg[it];
      }
#pragma unroll
      for (int ib = 0; ib < KB; ++ib)
        if (ids[KW + ib] >= 0) bg[ib] = xg[KW + ib].x;
      if (a.prof && tid == 0) {
        sprof[13] += e1 - e0;
        sprof[14] += e2 - e1;
        sprof[15] += clock64() - e2;
      }
    }
    // entropy term of log_std (d(-ent_coef * H)/d log_std = -ent_coef), once per minibatch; |g|^2
    float ss = 0.f;
#pragma unroll
    for (int it = 0; it < KW; ++it) {
      if (it >= nwi) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) ss += gg[it][j] * gg[it][j];
    }
#pragma unroll
    for (int ib = 0; ib < KB; ++ib) {
      if (bkind[ib] < 0) continue;
      if (bkind[ib] == 2) bg[ib] -= a.ent_coef * b_okf[ib];
      ss += bg[ib] * bg[ib];
    }
    ss = wave_sum(ss);
    if (lane == 0) L[g.red_off + w] = ss;
    // Gaussian entropy loss uses log_std before this minibatch's update
    if (gauss && tid == 0 && grp == 0 && q == 0) {
      float sl = 0.f;
      for (int j = 0; j < A; ++j) sl += has_ls ? L[g.ls_off + j] : 0.f;
      st_ent += -(sl + A * (0.5f + c_half_log2pi));
    }
    __syncthreads();  // B2: all gradients formed
    unsigned long long t2 = a.prof ? clock64() : 0;

    // ---------------- clip_grad_norm_ + Adam on the owned items (W/b/log_std in LDS)
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < kWaves; ++i) tot += L[g.red_off + i];
    if (ns) {
      // the other net's |g|^2: ONE tagged 8-B agent-scope atomic each way (minibatch tag in
      // the high word; MI355X_MICROARCH inter-workgroup visibility: 8-B agent atomics both
      // sides), polled by the other workgroup; summed actor + critic in both workgroups so
      // that they apply the identical clip
      const unsigned long long x0 = a.prof ? clock64() : 0;
      unsigned long long* xs = reinterpret_cast<unsigned long long*>(g.sync + 8);
      const unsigned long long tag = (unsigned long long)(unsigned)(k + 1) << 32;
      if (tid == 0 && !stall) __hip_atomic_store(xs + q, tag | __float_as_uint(tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (G == 1) pre_rows(k);  // (G > 1: done in the arrival wait)
      if (tid == 0) {
        unsigned long long o = __hip_atomic_load(xs + (1 - q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while ((o >> 32) != (unsigned long long)(unsigned)(k + 1)) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > spin_lim || ld_sc1u(tflag) != 0u) {
            spin_give_up(a, tflag);
            break;
          }
          o = __hip_atomic_load(xs + (1 - q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const float other = __uint_as_float((unsigned)(o & 0xffffffffu));
        L[g.red_off + 48] = q == 0 ? tot + other : other + tot;
      }
      __syncthreads();
      tot = L[g.red_off + 48];
      if (a.prof && tid == 0) sprof[16] += clock64() - x0;  // (net split: the |g|^2 hand-off)
    }
    // (stamps straight into LDS: no live registers; not in the full-register-file builds)
    constexpr bool kProfAdam = KW <= 8;
    if (kProfAdam && a.prof && tid == 0) sprof[17] -= clock64();
    const float coef = fminf(1.f, a.max_grad_norm / (sqrtf(tot) + 1e-6f));
    step += 1.f;
    b1t *= a.beta1;
    b2t *= a.beta2;
    const float step_size = a.lr / (1.f - b1t);
    const float inv_bc2s = 1.f / sqrtf(1.f - b2t);
    const float b1 = a.beta1, b2 = a.beta2, eps = a.adam_eps;
    // torch Adam: p -= step_size * m / (sqrt(v) / sqrt(1 - b2^t) + eps), on v_sqrt / v_rcp
    // (~1 ulp each). All of this wave's parameter reads are issued before any write
    // (the items never alias), so the LDS read latency is paid once, not per element.
    // Weight element j of slot it lives at W[16 ta + 4 kk + j][16 tb + r16] of its layer
    // image; padding elements (rows / columns past the layer dims) have gradient and
    // moments exactly 0, so their update is exactly 0 and they are updated in place.
    int paddr[KW];
    int pstr[KW];
#pragma unroll
    for (int it = 0; it < KW; ++it) {
      paddr[it] = g.trash_off + lane;
      pstr[it] = 0;
      if (it < nwi) {
        const int desc = rfl(g.items[wb + w + it * kWaves]);
        const int iq = desc & 1, il = (desc >> 1) & 3, ta = (desc >> 5) & 15, tb = (desc >> 9) & 15;
        const int ldw = rfl(g.ldw[iq][il]);
        paddr[it] = rfl(g.w_off[iq][il]) + (16 * ta + 4 * kk) * ldw + 16 * tb + r16;
        pstr[it] = ldw;
      }
    }
    float pval[KW][4], bval[KB];
#pragma unroll
    for (int it = 0; it < KW; ++it)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (BF3) pval[it][j] = wmst[it][j];
        else pval[it][j] = L[paddr[it] + j * pstr[it]];
      }
#pragma unroll
    for (int ib = 0; ib < KB; ++ib) bval[ib] = L[b_addr[ib]];
#pragma unroll
    for (int it = 0; it < KW; ++it) {
      if (it >= nwi) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gval = gg[it][j] * coef;
        gm[it][j] = b1 * gm[it][j] + (1.f - b1) * gval;
        gv[it][j] = b2 * gv[it][j] + (1.f - b2) * gval * gval;
        const float denom = __builtin_amdgcn_sqrtf(gv[it][j]) * inv_bc2s + eps;
        const float nv = pval[it][j] - step_size * gm[it][j] * __builtin_amdgcn_rcpf(denom);
        if constexpr (BF3) wmst[it][j] = nv;
        else L[paddr[it] + j * pstr[it]] = nv;
      }
      if constexpr (BF3) {  // the split-bf16 images of the updated elements (padding stays 0)
        if constexpr (HOIST) {
          bf3_store_tile<KT>(L, bpk[it] & 3, bwf[it], (bpk[it] >> 2) & 0x7fff, bwt[it], bpk[it] >> 17, r16, kk, wmst[it]);
        } else {
          int kd, wf, wl, wt, tl;
          slot_img(it, kd, wf, wl, wt, tl);
          bf3_store_tile<KT>(L, kd, wf, wl, wt, tl, r16, kk, wmst[it]);
        }
      }
    }
#pragma unroll
    for (int ib = 0; ib < KB; ++ib) {
      if (bkind[ib] < 0) continue;
      const float gval = bg[ib] * coef;
      bm[ib] = b1 * bm[ib] + (1.f - b1) * gval;
      bv[ib] = b2 * bv[ib] + (1.f - b2) * gval * gval;
      const float denom = __builtin_amdgcn_sqrtf(bv[ib]) * inv_bc2s + eps;
      L[b_addr[ib]] = bval[ib] - step_size * bm[ib] * __builtin_amdgcn_rcpf(denom);
    }
    if (kProfAdam && a.prof && tid == 0) {
      const unsigned long long a1 = clock64();
      sprof[17] += a1;
      sprof[18] -= a1;
    }
    __syncthreads();  // B3: parameters updated
    if (a.prof && tid == 0) {
      const unsigned long long t3 = clock64();
      sprof[0] += t1 - t0;
      sprof[1] += t2 - t1;
      sprof[2] += t3 - t2;
      if (kProfAdam) sprof[18] += t3;
    }
  }

  // ---- stats (every workgroup: its rows); sums of minibatch means
  const float vals[5] = {st_ent, st_pg, st_vl, st_cf, st_kl};
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const float v = wave_sum(vals[i]);
    if (lane == 0) L[g.red_off + 8 + w * 5 + i] = v;
  }
  __syncthreads();
  if (tid < 5) {
    float s = 0.f;
    for (int i = 0; i < kWaves; ++i) s += L[g.red_off + 8 + i * 5 + tid];
    if (!(tid == 0 && gauss)) s *= invB;  // per-row sums -> sums of minibatch means
    if (G > 1 || ns) atomicAdd(a.stats + tid, s);
    else a.stats[tid] += s;
  }
  if (grp != 0) return;  // every workgroup holds the identical model: one writes it back
  // (net split: each workgroup writes its own net, the actor workgroup the shared state)
  const bool shared_wb = !ns || q == 0;

  // ---- write back: params (from LDS), moments (owners), log_std, normaliser
#pragma unroll
  for (int qq = 0; qq < 2; ++qq) {
#pragma unroll
    for (int l = 0; l < kL; ++l) {
      if (l >= (qq == 0 ? a.n_pi : a.n_vf) || (ns && qq != q)) continue;
      const LG y = lg(g, qq, l);
      const int wo = qq == 0 ? a.pi_w_off[l] : a.vf_w_off[l];
      const int bo = qq == 0 ? a.pi_b_off[l] : a.vf_b_off[l];
      if constexpr (!BF3)
        for (int i = tid; i < y.dout * y.din; i += kThreads) {
          const int o = i / y.din, c = i - o * y.din;
          a.params[wo + i] = L[y.w + o * y.ldw + c];
        }
      for (int i = tid; i < y.dout; i += kThreads) a.params[bo + i] = L[y.b + i];
    }
  }
  if (shared_wb && has_ls && tid < A) a.params[a.log_std_off + tid] = L[g.ls_off + tid];
#pragma unroll
  for (int it = 0; it < KW; ++it) {
    if (it >= nwi) continue;
    const int desc = rfl(g.items[wb + w + it * kWaves]);
    const int iq = desc & 1, il = (desc >> 1) & 3, ta = (desc >> 5) & 15, tb = (desc >> 9) & 15;
    const int din = g.din[iq][il], dout = g.dout[iq][il];
    const int wo = iq == 0 ? a.pi_w_off[il] : a.vf_w_off[il];
    const int in = 16 * tb + r16;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = 16 * ta + 4 * kk + j;
      if (o < dout && in < din) {
        a.exp_avg[wo + o * din + in] = gm[it][j];
        a.exp_avg_sq[wo + o * din + in] = gv[it][j];
        if constexpr (BF3) a.params[wo + o * din + in] = wmst[it][j];  // the owners hold the masters
      }
    }
  }
#pragma unroll
  for (int ib = 0; ib < KB; ++ib) {
    if (bkind[ib] < 0 || b_okf[ib] == 0.f) continue;
    const int desc = rfl(g.items[bb + w + ib * kWaves]);
    const int iq = desc & 1, il = (desc >> 1) & 3;
    const int off = bkind[ib] == 1 ? (iq == 0 ? a.pi_b_off[il] : a.vf_b_off[il]) : a.log_std_off;
    a.exp_avg[off + lane] = bm[ib];
    a.exp_avg_sq[off + lane] = bv[ib];
  }
  if (shared_wb && norm_lane && K > 0) {
    a.norm_mean[nc] = run_m;
    a.norm_var[nc] = run_v;
    if (nc == 0) {
      if (a.norm_count_i) a.norm_count_i[0] = (int)run_c;  // (an exact integer below 2^24)
      else a.norm_count[0] = run_c;
    }
  }
  if (shared_wb && tid == 0) a.adam_step[0] = step;
  // (stats barrier above orders the LDS). Net split: the critic workgroup owns the critic
  // row-tile counters [7..10] (the actor's are zero there), added atomically
  if (a.prof && tid < 20) {
    const bool critic_slot = tid >= 7 && tid <= 10;
    if (!ns) a.prof[tid] += sprof[tid];
    else if (q == 0 && !critic_slot) a.prof[tid] += sprof[tid];
    else if (q == 1 && critic_slot) atomicAdd(a.prof + tid, sprof[tid]);
  }
}

// waves per workgroup (NW) and owned weight / bias slots per wave of each tile width
// (generic builds; the shape-specialised ones size KW / KB to their exact item counts)
constexpr int waves_for(int kt) { return kt == 2 ? 8 : 4; }
constexpr int wslots_for(int kt) { return kt == 2 ? 5 : 16; }
constexpr int bslots_for(int kt) { return kt == 2 ? 2 : 3; }
// net split (4 waves, one net's items): up to 20 / 32 weight tiles and 8 vectors per net
constexpr int wslots_ns(int kt) { return kt == 2 ? 5 : 8; }
constexpr int bslots_ns() { return 2; }
// generic both-nets build at 4 waves (<= 32-wide nets): up to 20 weight tiles (3-layer nets with
// obs dim <= 32), 8 vectors
constexpr int kNarrow4W = 5;
constexpr int kNarrow4B = 2;


}  // namespace rc
}  // namespace ia

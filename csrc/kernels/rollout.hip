// Device rollout, serial part: T steps of actor sampling + env physics for N envs in
// ONE launch (replaces the reference's per-step host loop: SB3 collect_rollouts ->
// policy.forward -> VecEnv.step over pipes -> RewardVecEnvWrapper).
//
// Only what the NEXT step depends on stays on the serial chain: the actor mean /
// logits, the sampled action and the env step. Everything a step merely records --
// value estimate, log-prob, TimeLimit bootstrap, learned reward -- is recomputed for
// all T x N transitions at once by rollout_post_kernel (engine.hip), and the sampling
// noise of a whole chunk of steps is drawn up front by all 64 lanes into LDS.
//
// Mapping: one wave64 per env, one env per workgroup (no inter-wave sync at all).
// Actor layer l, "split" form (every width <= 32): lane (h, j) = (lane >> 5, lane & 31)
// owns unit j and half h of the K (input) range, its weights live in VGPRs, the layer
// input is broadcast from a 64-float LDS vector with ds_read_b128 (every lane of a
// half reads the same address), and the two half sums meet through
// v_permlane32_swap. Widths up to 64 use the "full" form (lane = unit, whole K).
// Split form with every hidden layer exactly 32 wide (the locomotion recipes): the "row" form
// -- no LDS at all, the layer input is a DPP row broadcast of the lane's own register (see
// nb_lane below).
// The locomotion model keeps its state in registers: joint j on lane j, the root
// coordinates uniform in every lane, cross-joint sums by DPP quad/row butterflies.
// No loop iteration waits on global memory: inputs are LDS, outputs are fire-and-
// forget stores.
#include <hip/hip_runtime.h>

#include "ia/engine.h"
#include "ia/envs.h"
#include "ia/wave.h"
#include "launchers.h"

namespace ia {
namespace {

constexpr int kNoiseFloats = 4096;  // per chunk of steps (16 KiB)

// Split form: weights in VGPRs, lane (h, j) holds W[j][k0 + i], i < 16.
// Full form:  weights in LDS, image [din/4][64 lanes][4 k] (one ds_read_b128 per 4 inputs).
template <bool SPLIT>
struct Actor {
  static constexpr int KH = SPLIT ? 16 : 1;
  float w[kWaveMaxLayers][KH];
  const lf* wt[kWaveMaxLayers];  // full form
  float bias[kWaveMaxLayers];
  int k0[kWaveMaxLayers];  // first input of this lane's slice (uniform per half)
  int ng[kWaveMaxLayers];  // groups of 4 inputs (uniform)
  int dout[kWaveMaxLayers];
  int n_layers, hidden_act;
};

__host__ __device__ __forceinline__ int split_kh(int din) { return ((din + 1) / 2 + 3) & ~3; }
// full form: every layer's image padded to 64 inputs (16 groups of 4), so the forward loop has
// a compile-time trip count and issues all its LDS loads back to back
constexpr int kFullGroups = 16;
__host__ __device__ __forceinline__ int full_lds_floats(const WaveMLP& m) { return m.n_layers * 4 * kFullGroups * 64; }

// Row form (split form, every hidden width 32): the 64 lanes are 4 DPP rows of 16; in layer l
// row r takes K-half `kh` and block `ub` of 16 units, (kh, ub) = (r & 1, r >> 1) in even layers
// and (r >> 1, r & 1) in odd ones, so the two K-halves of a unit meet through permlane16_swap
// (rows 0+1, 2+3) in even layers and permlane32_swap (rows 0+2, 1+3) in odd ones. Either swap
// leaves unit 16 * b + i in lane i of exactly the rows whose K-half is b in the next layer, so
// that layer reads input k0 + i as row_newbcast:i of the lane's own register. Same weights,
// products and summation order per unit as the LDS split form (bitwise the same outputs).
__device__ __forceinline__ void nb_lane(int l, int lane, int& kh, int& ub) {
  const int r = lane >> 4;
  kh = (l & 1) ? (r >> 1) : (r & 1);
  ub = (l & 1) ? (r & 1) : (r >> 1);
}

template <bool SPLIT, bool NB = false>
__device__ void load_actor(const WaveMLP& m, Actor<SPLIT>& r, lf* wlds) {
  const int lane = threadIdx.x;
  r.n_layers = m.n_layers;
  r.hidden_act = m.hidden_act;
#pragma unroll
  for (int l = 0; l < kWaveMaxLayers; ++l) {
    int h = SPLIT ? (lane >> 5) : 0;
    int j = SPLIT ? (lane & 31) : lane;
    if (NB) {
      int ub;
      nb_lane(l, lane, h, ub);
      j = 16 * ub + (lane & 15);
    }
    const bool on = l < m.n_layers;
    const int din = on ? m.dims[l] : 0, dout = on ? m.dims[l + 1] : 0;
    const int kh = SPLIT ? split_kh(din) : 4 * kFullGroups;
    const int k0 = h ? kh : 0;
    r.k0[l] = k0;
    r.ng[l] = kh >> 2;
    r.dout[l] = dout;
    if (SPLIT) {
      const int kend = h ? din : kh;
#pragma unroll
      for (int i = 0; i < Actor<SPLIT>::KH; ++i) {
        const int k = k0 + i;
        r.w[l][i] = (on && j < dout && k < kend && k < din) ? m.W[l][j * din + k] : 0.f;
      }
    } else {
      r.wt[l] = wlds;
      if (on) {
        for (int k = 0; k < kh; ++k) wlds[((k >> 2) * 64 + lane) * 4 + (k & 3)] = (j < dout && k < din) ? m.W[l][j * din + k] : 0.f;
        wlds += kh * 64;
      }
    }
    r.bias[l] = (on && j < dout && h == 0) ? m.b[l][j] : 0.f;
  }
}

// Hidden activation: compile-time for the common tanh / relu nets, runtime otherwise.
template <int HACT>
__device__ __forceinline__ float hidden_act(int act, float x) {
  if (HACT == ACT_TANH) return act_fast(ACT_TANH, x);
  if (HACT == ACT_RELU) return fmaxf(x, 0.f);
  return act_fast(act, x);
}

// Keep a loop-invariant value in a VGPR: one wave per SIMD has registers to spare, while
// the kernel's uniform values otherwise overflow the SGPR file and get spilled to VGPR
// lanes (one v_readlane per use inside the step loop).
template <typename T>
__device__ __forceinline__ T pin(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

// x (the normalised observation) is already in xb[0 .. 64) (zero padded). Returns, in
// lane j < dout of the last layer (both halves in split form), the actor output j.
// The split form always runs 4 groups of 4 inputs (zero weights pad the short layers):
// 4 extra FMAs on the 17-input layer instead of uniform branches around every group.
// NLT > 0: the layer count at compile time (the per-layer guards and the last-layer test fold
// away instead of costing exec-mask juggling on every layer of every step). HW > 0: every
// hidden layer is HW wide (32 split form, 64 full form), so no lane is past its layer's width
// and the activation runs unmasked.
template <bool SPLIT, int HACT, int NLT = -1, int HW = -1>
__device__ __forceinline__ float actor_forward(const Actor<SPLIT>& r, lf* xb) {
  const int lane = threadIdx.x;
  const int j = SPLIT ? (lane & 31) : lane;
  const lf4* x4 = (const lf4*)xb;
  float h = 0.f;
  const int nl = NLT > 0 ? NLT : r.n_layers;
#pragma unroll
  for (int l = 0; l < kWaveMaxLayers; ++l) {
    if (l < nl) {
      const lf4* src = x4 + (r.k0[l] >> 2);
      float acc0 = r.bias[l], acc1 = 0.f;
      if (SPLIT) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32v4 v = src[g];
          acc0 = fmaf(r.w[l][4 * g + 0], v.x, acc0);
          acc1 = fmaf(r.w[l][4 * g + 1], v.y, acc1);
          acc0 = fmaf(r.w[l][4 * g + 2], v.z, acc0);
          acc1 = fmaf(r.w[l][4 * g + 3], v.w, acc1);
        }
      } else {
        const lf4* w4 = (const lf4*)r.wt[l] + lane;
        float acc2 = 0.f, acc3 = 0.f;
#pragma unroll
        for (int g = 0; g < kFullGroups; ++g) {  // zero-padded past din (weights and inputs)
          const f32v4 v = src[g], w = w4[g * 64];
          acc0 = fmaf(w.x, v.x, acc0);
          acc1 = fmaf(w.y, v.y, acc1);
          acc2 = fmaf(w.z, v.z, acc2);
          acc3 = fmaf(w.w, v.w, acc3);
        }
        acc0 += acc2;
        acc1 += acc3;
      }
      float acc = acc0 + acc1;
      if (SPLIT) acc = add_halves(acc);
      const bool last = l == nl - 1;
      const bool full = HW > 0 && !last;  // (HW == 32 split / 64 full: every lane is a unit)
      h = (full || j < r.dout[l]) ? (last ? acc : hidden_act<HACT>(r.hidden_act, acc)) : 0.f;
      if (!last) {
        wave_sync();  // every lane has read this layer's input
        // split form: lanes 32..63 hold copies of 0..31, and the next layer reads xb[0 .. 32)
        // only (its last 16 weights are zero), so the write needs no mask
        if (SPLIT && HW <= 0) {
          if (lane < 32) xb[lane] = h;
        } else {
          xb[lane] = h;
        }
        wave_sync();
      }
    }
  }
  return h;
}

// Row form of actor_forward (NLT layers, hidden widths 32): x = this lane's layer-0 input,
// input k0 + (lane & 15) of its row's K-half (actor_obs_index). Returns the actor output j in
// lane j < dout of the last layer.
// acc += x[row lane I] * w as ONE v_fmac_f32_dpp (the compiler keeps a separate v_mov_b32_dpp
// per broadcast, twice the VALU issue). I == 0 is the layer's first read of x, just written by a
// VALU op: the DPP read needs two wait states after it.
template <int I>
__device__ __forceinline__ float fmac_row_bcast(float acc, float x, float w) {
  if constexpr (I == 0)
    asm("s_nop 1\n\tv_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc) : "v"(x), "v"(w), "i"(I));
  else
    asm("v_fmac_f32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(x), "v"(w), "i"(I));
  return acc;
}

template <int I>
__device__ __forceinline__ void nb_dot(const float* w, float x, float& a0, float& a1) {
  if constexpr (I < 16) {
    a0 = fmac_row_bcast<I>(a0, x, w[I]);  // == fmaf(w[I], x_I, a0)
    a1 = fmac_row_bcast<I + 1>(a1, x, w[I + 1]);
    nb_dot<I + 2>(w, x, a0, a1);
  }
}

template <int HACT, int NLT>
__device__ __forceinline__ float actor_forward_nb(const Actor<true>& r, float x) {
  static_assert(NLT > 0, "the row form needs the layer count at compile time");
#pragma unroll
  for (int l = 0; l < NLT; ++l) {
    float acc0 = r.bias[l], acc1 = 0.f;
    nb_dot<0>(r.w[l], x, acc0, acc1);
    const float acc = (l & 1) ? add_halves(acc0 + acc1) : add_rows16(acc0 + acc1);
    x = l == NLT - 1 ? acc : hidden_act<HACT>(r.hidden_act, acc);
  }
  return x;
}

// The observation index whose (normalised) value is lane `lane`'s row-form layer-0 input.
__device__ __forceinline__ int actor_obs_index(int lane, int obs_dim) {
  return ((lane >> 4) & 1 ? split_kh(obs_dim) : 0) + (lane & 15);
}

// Generic (non-locomotion) envs step on lane 0, inlined: an out-of-line call needs a stack
// frame (544 B/lane of scratch in the generic instances), while the inlined switch fits the
// loop's register budget (<= 222 VGPRs at two waves per SIMD, 0 scratch: tools/kernel_resources.py).
__device__ __forceinline__ float env_step_lane0(const EnvParams& P, float* s, const float* action, int* term, uint64_t* rng) {
  return env_step(P, s, action, term, *rng);
}
__device__ __forceinline__ void env_reset_lane0(const EnvParams& P, float* s, float* o, uint64_t* rng) {
  env_reset(P, s, *rng);
  env_obs(P, s, o);
}

// ---------------------------------------------------------------- locomotion, state in registers
// ENV template values of the chain kernel.
enum ChainEnv : int { CE_GENERIC = 0, CE_LOCO = 1, CE_LOCO3 = 2 /* planar root: nq_root == nv_root == 3 */ };

struct LocoRegs {
  float q, qd;          // joint lane state (lane < nj)
  float rq[8], rv[8];   // root coordinates (uniform)
  float gear, stiff, damp, thrust, pcoup;  // per-joint-lane constants
  float dt, drag, fwd_weight, healthy, ctrl_cost, inv_nj, inv_dt_total;
};

__device__ void loco_load(const LocoParams& p, const lf* s, LocoRegs& L) {
  const int lane = threadIdx.x, nq = loco_nq(p);
  const bool jl = lane < p.nj;
  L.q = jl ? s[p.nq_root + lane] : 0.f;
  L.qd = jl ? s[nq + p.nv_root + lane] : 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    L.rq[i] = i < p.nq_root ? s[i] : 0.f;
    L.rv[i] = i < p.nv_root ? s[nq + i] : 0.f;
  }
}

__device__ void loco_store(const LocoParams& p, const LocoRegs& L, lf* s) {
  const int lane = threadIdx.x, nq = loco_nq(p);
  if (lane < p.nj) {
    s[p.nq_root + lane] = L.q;
    s[nq + p.nv_root + lane] = L.qd;
  }
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i < p.nq_root) s[i] = L.rq[i];
      if (i < p.nv_root) s[nq + i] = L.rv[i];
    }
  }
}

// Observation [qpos[obs_skip:], qvel] in lane layout, through the LDS scratch sb.
template <int ENV>
__device__ float loco_obs(const LocoParams& p, const LocoRegs& L, lf* sb, int oxi, float& ox) {
  const int lane = threadIdx.x;
  const int nr = ENV == CE_LOCO3 ? 3 : 8;
  const int nqr = ENV == CE_LOCO3 ? 3 : p.nq_root, nvr = ENV == CE_LOCO3 ? 3 : p.nv_root;
  const int npr = nqr - p.obs_skip, nj = p.nj;
  float rqi = 0.f, rvi = 0.f;
#pragma unroll
  for (int i = 0; i < nr; ++i) {
    rqi = (lane + p.obs_skip) == i ? L.rq[i] : rqi;
    rvi = lane == i ? L.rv[i] : rvi;
  }
  wave_sync();
  if (lane < npr) sb[lane] = rqi;
  if (lane < nj) {
    sb[npr + lane] = L.q;
    sb[npr + nj + nvr + lane] = L.qd;
  }
  if (lane < nvr) sb[npr + nj + lane] = rvi;
  wave_sync();
  const int D = npr + nj + nvr + nj;
  ox = sb[oxi];  // (the row-form actor's input layout; past D a zero word of xb, oxi < 0)
  return lane < D ? sb[lane] : 0.f;
}

// ia::loco_step (envs.h) with the joint loops spread over lanes; a_in = action of joint
// lane j. Returns the step reward (uniform).
// FS > 0: frame_skip at compile time. The substeps are then unrolled, so the root-state
// chain (stance -> thrust / lift lane sums -> root velocities) of one substep overlaps the
// joint chain (sin -> qdd -> qd -> q) of the next instead of each substep ending at the loop
// back-edge.
template <int ENV, int FS = -1>
__device__ float loco_step_regs(const LocoParams& p, LocoRegs& L, float a_in) {
  const int lane = threadIdx.x;
  const bool jl = lane < p.nj;
  const float a = jl ? fminf(fmaxf(a_in, -1.f), 1.f) : 0.f;
  const float ctrl = sum_lanes8(a * a);
  const float pitch = sum_lanes8(L.pcoup * a);
  const float x_before = L.rq[0];
  const float dt = L.dt;
  float q = L.q, qd = L.qd;
  const auto substep = [&]() {
    const float qdd = L.gear * a - L.stiff * q - L.damp * qd - 2.0f * __sinf(q);
    const float st_all = stance(q);  // every lane (no exec-masked branch around the exp / rcp)
    const float st = jl ? st_all : 0.f;
    const float th_j = L.thrust * st * fmaxf(-qd, 0.f);
    qd = qd + dt * qdd;
    const float thrust = sum_lanes8(th_j);
    const float lift = sum_lanes8(st);
    const float vx = L.rv[0];
    L.rv[0] = vx + dt * (thrust - L.drag * vx * (1.0f + fabsf(vx)));
    if (ENV == CE_LOCO3) {
      L.rv[1] = L.rv[1] + dt * (-20.f * L.rq[1] - 4.f * L.rv[1] + 0.5f * (lift * L.inv_nj - 0.5f));
      L.rv[2] = L.rv[2] + dt * (-15.f * __sinf(L.rq[2]) - 3.f * L.rv[2] + pitch);
      L.rq[0] += dt * L.rv[0];
      L.rq[1] += dt * L.rv[1] * 1.f;
      L.rq[2] += dt * L.rv[2] * 1.f;
    } else {
      if (p.nv_root > 1) L.rv[1] = L.rv[1] + dt * (-20.f * L.rq[1] - 4.f * L.rv[1] + 0.5f * (lift * L.inv_nj - 0.5f));
      if (p.nv_root > 2) L.rv[2] = L.rv[2] + dt * (-15.f * __sinf(L.rq[2]) - 3.f * L.rv[2] + pitch);
#pragma unroll
      for (int i = 3; i < 8; ++i)
        if (i < p.nv_root) L.rv[i] = L.rv[i] * (1.f - 2.f * dt) + dt * 0.1f * pitch;
      L.rq[0] += dt * L.rv[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) {
        if (i < p.nq_root) {
          if (i < p.nv_root) {
            L.rq[i] += dt * L.rv[i] * 1.f;
          } else {  // free-joint quaternion slots (3D bodies only)
            const int vi = i % p.nv_root;
            float v = 0.f;
#pragma unroll
            for (int u = 0; u < 8; ++u) v = u == vi ? L.rv[u] : v;
            L.rq[i] += dt * v * 0.1f;
          }
        }
      }
    }
    // joint limit: clamp q and kill the velocity into the stop, as selects (no branches)
    const float qn = q + dt * qd;
    const bool hi = qn > 1.2f, lo = qn < -1.2f;
    qd = (hi && qd > 0.f) || (lo && qd < 0.f) ? 0.f : qd;
    q = fminf(fmaxf(qn, -1.2f), 1.2f);
  };
  if constexpr (FS > 0) {
#pragma unroll
    for (int sub = 0; sub < FS; ++sub) substep();
  } else {
    for (int sub = 0; sub < p.frame_skip; ++sub) substep();
  }
  L.q = jl ? q : 0.f;
  L.qd = jl ? qd : 0.f;
  return L.fwd_weight * (L.rq[0] - x_before) * L.inv_dt_total + L.healthy - L.ctrl_cost * ctrl;
}

// Per-lane output cursors (VGPRs, advanced by one step per iteration): the per-step
// stores need no scalar base registers, and the five per-env scalars of a step go out
// as ONE store (lane 0 env reward, 1 done, 2 truncation, 3 finished-episode return,
// 4 episode start).
// Typed global (address_space 1): pin()'s asm would otherwise erase the address space and
// the stores would be FLAT, which count in lgkmcnt too -- every LDS wait of the next actor
// layer then also waited for the previous step's stores to retire.
typedef __attribute__((address_space(1))) float gfl;
struct Cursors {
  gfl* obs;
  gfl* next_obs;
  gfl* act_raw;
  gfl* act_env;
  gfl* sc;
  int vec_step, act_step, sc_step;
};

// Phase clock of the breakdown probe: the core clock, read after `dep` is in a register (the
// volatile asm keeps the stamps in program order and the input ties each to its phase's result).
__device__ __forceinline__ long long stamp(float dep) {
  long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(dep));
  return t;
}

template <bool SPLIT, int ENV, int HACT, int NLT = -1, int HW = -1, int FS = -1, bool PROF = false, bool ROW = true>
__global__ __launch_bounds__(64) void rollout_chain_kernel(RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_raw[];
  lf* xb = (lf*)lds_raw;       // [64] layer input broadcast
  lf* sb = xb + 64;            // [64] observation scratch
  lf* st = sb + 64;            // [kMaxState] env state (generic envs, resets)
  lf* act = st + kMaxState;    // [64]
  lf* noise = act + 64;        // [kNoiseFloats]
  li* explore = (li*)(noise + kNoiseFloats);  // [T]
  lf* wlds = (lf*)(explore + ((a.T + 3) & ~3)); // full-form actor weights (16-B aligned)
  const int n = blockIdx.x;
  const int lane = threadIdx.x;
  const EnvParams& P = a.P;
  const int D = P.obs_dim;
  constexpr bool loco = ENV != CE_GENERIC;
  const bool discrete = !loco && a.n_actions > 0;  // locomotion envs are continuous (host check)
  const int A = discrete ? 1 : P.act_dim;
  const int AW = discrete ? a.n_actions : P.act_dim;  // noise values per step
  const int S = state_size(P);

  // row form: the split form with every hidden layer 32 wide (HW == 32, depth NLT known)
  constexpr bool NB = ROW && SPLIT && HW == 32 && NLT > 0;
  Actor<SPLIT> ar;
  load_actor<SPLIT, NB>(a.pi, ar, wlds);
  // lane layout of the observation (stores) and, for the row form, the layer-0 input layout
  const int oxi = NB ? actor_obs_index(lane, D) : lane;
  const bool ox_on = oxi < D;
  // LDS word (relative to sb) of this lane's layer-0 input: past D, a word of xb, which the row
  // form never writes (0 from the prologue) -- so (ox - 0) * 1 = +0 exactly as the LDS form's 0.f
  const int oxr = ox_on ? oxi : lane - 64;
  const float nmean = pin((a.pi.norm_mean && ox_on) ? a.pi.norm_mean[oxi] : 0.f);
  const float nrstd = pin((a.pi.norm_mean && ox_on) ? rsqrtf(a.pi.norm_var[oxi] + a.pi.norm_eps) : 1.f);
  const float lstd = (!discrete && a.log_std && lane < A) ? a.log_std[lane] : 0.f;
  const float sd = pin(expf(lstd));
  const float lo = pin((!discrete && a.act_low && lane < A) ? a.act_low[lane] : 0.f);
  const float hi = pin((!discrete && a.act_high && lane < A) ? a.act_high[lane] : 0.f);

  for (int i = lane; i < S; i += 64) st[i] = a.state[(size_t)n * S + i];
  xb[lane] = 0.f;
  LocoRegs L{};
  if (loco) {
    const LocoParams& p = P.loco;
    const bool jl = lane < p.nj;
    L.gear = pin(jl ? p.gear[lane] : 0.f);
    L.stiff = pin(jl ? p.stiff[lane] : 0.f);
    L.damp = pin(jl ? p.damp[lane] : 0.f);
    L.thrust = pin(jl ? p.thrust[lane] : 0.f);
    L.pcoup = pin(jl ? p.pitch_coupling[lane] : 0.f);
    L.dt = pin(p.dt);
    L.drag = pin(p.drag);
    L.fwd_weight = pin(p.fwd_weight);
    L.healthy = pin(p.healthy_reward);
    L.ctrl_cost = pin(p.ctrl_cost);
    L.inv_nj = pin(1.f / (float)p.nj);
    L.inv_dt_total = pin(1.f / (p.dt * (float)p.frame_skip));
  }
  wave_sync();
  if (loco) loco_load(P.loco, st, L);

  Cursors c;
  c.vec_step = a.N * D;
  c.act_step = a.N * A;
  c.sc_step = a.N;
  c.obs = pin((gfl*)(a.obs_buf + (size_t)n * D + (lane < D ? lane : 0)));
  c.next_obs = pin((gfl*)(a.next_obs + (size_t)n * D + (lane < D ? lane : 0)));
  c.act_raw = pin((gfl*)(a.act_raw + (size_t)n * A + (lane < A ? lane : 0)));
  c.act_env = pin((gfl*)(a.act_env + (size_t)n * A + (lane < A ? lane : 0)));
  {
    float* b = lane == 0 ? a.env_rew : lane == 1 ? a.dones : lane == 2 ? a.trunc : lane == 3 ? a.ep_ret_out : a.starts;
    c.sc = pin((gfl*)(b + n));
  }

  float o = lane < D ? a.cur_obs[(size_t)n * D + lane] : 0.f;
  float ox = ox_on ? a.cur_obs[(size_t)n * D + oxi] : 0.f;  // (row form: == o otherwise)
  float start = a.cur_start[n];
  uint64_t rng = a.rng[n];
  int elapsed = a.elapsed[n];
  float ep_ret = a.ep_ret[n];
  const int chunk = AW > 0 ? max(1, min(a.T, kNoiseFloats / AW)) : a.T;
  const bool has_explore = a.explore_mode != nullptr;
  const int max_steps = a.max_steps;
  long long ph[4] = {0, 0, 0, 0}, n_prof = 0;

  for (int t0 = 0; t0 < a.T; t0 += chunk) {
    const int tc = min(chunk, a.T - t0);
    // ---- this chunk's sampling noise, all lanes in parallel (off the step chain)
    wave_sync();
    for (int e = lane; e < tc * AW; e += 64) {
      const int tr = e / AW, k = e - tr * AW;
      const uint64_t key = hash3(a.seed, (uint64_t)n, (uint64_t)(a.step0 + t0 + tr));
      uint64_t s = key ^ (kLaneTweak * (uint64_t)(k + 1));
      float v;
      if (a.deterministic) {  // mean / argmax(logits)
        v = 0.f;
      } else if (discrete) {  // Gumbel-max: argmax(logits + G) ~ Categorical(softmax(logits))
        const float u = fmaxf(uniform01(s), 1e-12f);
        v = -logf(-logf(u));
      } else {
        v = normal01(s);
      }
      noise[e] = v;
    }
    if (has_explore)
      for (int e = lane; e < tc; e += 64) explore[e] = a.explore_mode[t0 + e];
    wave_sync();

    const lf* nz = noise + (lane < AW ? lane : 0);
    for (int tr = 0; tr < tc; ++tr, nz += AW) {
      long long t0 = 0, t1 = 0, t2 = 0, t3 = 0;
      if constexpr (PROF) t0 = stamp(o);
      if (lane < D) *c.obs = o;
      // ---- actor
      float head;
      if constexpr (NB) {
        head = actor_forward_nb<HACT, NLT>(ar, (ox - nmean) * nrstd);
      } else {
        xb[lane] = lane < D ? (o - nmean) * nrstd : 0.f;
        wave_sync();
        head = actor_forward<SPLIT, HACT, NLT, HW>(ar, xb);
      }
      float a_raw, a_env;
      if (discrete) {
        const float g = lane < a.n_actions ? head + *nz : -INFINITY;
        const float mx = wave_max(g);
        const unsigned long long m = __ballot(g == mx && lane < a.n_actions);
        const int k = m ? __builtin_ctzll(m) : a.n_actions - 1;
        a_raw = a_env = (float)k;
      } else {
        a_raw = head + sd * *nz;
        a_env = fminf(fmaxf(a_raw, lo), hi);
      }
      if (has_explore && explore[tr]) {  // ExplorationWrapper's random policy (uniform branch)
        const uint64_t key = hash3(a.seed, (uint64_t)n, (uint64_t)(a.step0 + t0 + tr));
        uint64_t s = key ^ kExploreTweak;
        if (discrete) {
          s ^= kExploreDiscreteTweak;
          const float u = uniform01(s);
          int k = (int)(u * (float)a.n_actions);
          k = k < a.n_actions ? k : a.n_actions - 1;
          a_raw = a_env = (float)k;
        } else {
          s ^= kLaneTweak * (uint64_t)(lane + 1);
          const float u = uniform01(s);
          a_env = lo + u * (hi - lo);
          a_raw = a_env;
        }
      }
      if (lane < A) {
        *c.act_raw = a_raw;
        *c.act_env = a_env;
      }
      // ---- env step + SB3 auto-reset, TimeLimit, Monitor
      int term = 0;
      float r_env;
      float o_next, ox_next;
      if constexpr (PROF) t1 = stamp(a_env);
      if (loco) {
        r_env = loco_step_regs<ENV, FS>(P.loco, L, a_env);
        if constexpr (PROF) t2 = stamp(r_env);
        o_next = loco_obs<ENV>(P.loco, L, sb, oxr, ox_next);
        if constexpr (PROF) t3 = stamp(o_next);
      } else {
        if (lane < A) act[lane] = a_env;
        wave_sync();
        if (lane == 0) {
          r_env = env_step_lane0(P, (float*)st, (const float*)act, &term, &rng);
          env_obs(P, (const float*)st, (float*)sb);
        }
        wave_sync();
        term = __builtin_amdgcn_readfirstlane(term);
        r_env = bcast(r_env, 0);
        o_next = lane < D ? sb[lane] : 0.f;
        ox_next = sb[oxr];
      }
      elapsed += 1;
      ep_ret += r_env;
      const bool trunc = !term && elapsed >= max_steps;
      const bool done = term || trunc;
      if (lane < D) *c.next_obs = o_next;
      {  // selects, not a nest of exec-masked branches
        float v = start;
        v = lane == 3 ? (done ? ep_ret : 0.f) : v;
        v = lane == 2 ? (trunc ? 1.f : 0.f) : v;
        v = lane == 1 ? (done ? 1.f : 0.f) : v;
        v = lane == 0 ? r_env : v;
        if (lane < 5) *c.sc = v;
      }
      c.obs += c.vec_step;
      c.next_obs += c.vec_step;
      c.act_raw += c.act_step;
      c.act_env += c.act_step;
      c.sc += c.sc_step;
      if (done) {
        wave_sync();
        if (lane == 0) {
          if (loco) loco_reset(P.loco, (float*)st, rng);
          else env_reset_lane0(P, (float*)st, (float*)sb, &rng);
        }
        wave_sync();
        if (loco) {
          loco_load(P.loco, st, L);
          o = loco_obs<ENV>(P.loco, L, sb, oxr, ox);
        } else {
          o = lane < D ? sb[lane] : 0.f;
          ox = sb[oxr];
        }
        elapsed = 0;
        ep_ret = 0.f;
      } else {
        o = o_next;
        ox = ox_next;
      }
      start = done ? 1.f : 0.f;
      if constexpr (PROF) {
        const long long t4 = stamp(o);
        ph[0] += t1 - t0;
        ph[1] += t2 - t1;
        ph[2] += t3 - t2;
        ph[3] += t4 - t3;
        ++n_prof;
      }
    }
  }
  if constexpr (PROF) {
    if (lane < 5) a.prof[n * 5 + lane] = lane == 4 ? n_prof : lane == 0 ? ph[0] : lane == 1 ? ph[1] : lane == 2 ? ph[2] : ph[3];
  }
  if (loco) loco_store(P.loco, L, st);
  wave_sync();
  for (int i = lane; i < S; i += 64) a.state[(size_t)n * S + i] = st[i];
  if (lane < D) a.cur_obs[(size_t)n * D + lane] = o;
  if (lane == 0) {
    a.cur_start[n] = start;
    a.elapsed[n] = elapsed;
    a.ep_ret[n] = ep_ret;
  }
  // lane 0's rng advanced inside env_step / env_reset; persist it
  rng = (uint64_t)__builtin_amdgcn_readfirstlane((int)(rng & 0xffffffffu)) |
        ((uint64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(rng >> 32)) << 32);
  if (lane == 0) a.rng[n] = rng;
}

}  // namespace

bool rollout_split_form(const WaveMLP& m) {
  for (int l = 0; l <= m.n_layers; ++l)
    if (m.dims[l] > 32) return false;
  return true;
}

size_t rollout_lds_bytes(const RolloutArgs& a) {
  const size_t full = rollout_split_form(a.pi) ? 0 : (size_t)full_lds_floats(a.pi);
  return (size_t)(64 + 64 + kMaxState + 64 + kNoiseFloats + full) * sizeof(float) + (size_t)((a.T + 3) & ~3) * sizeof(int);
}

hipError_t rollout_launch(const RolloutArgs& a, hipStream_t s) {
  if (a.T <= 0 || a.N <= 0) return hipSuccess;
  if (a.P.obs_dim > 64 || a.pi.n_layers < 1 || a.pi.n_layers > kWaveMaxLayers) return hipErrorInvalidValue;
  for (int l = 0; l <= a.pi.n_layers; ++l)
    if (a.pi.dims[l] > 64 || a.pi.dims[l] < 1) return hipErrorInvalidValue;
  if (a.pi.dims[0] != a.P.obs_dim) return hipErrorInvalidValue;
  if (a.n_actions > 64 || (a.P.kind == ENV_LOCO && (a.P.loco.nj > 8 || a.n_actions > 0))) return hipErrorInvalidValue;
  const size_t lds = rollout_lds_bytes(a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const bool split = rollout_split_form(a.pi);
  const LocoParams& p = a.P.loco;
  const int env = a.P.kind != ENV_LOCO ? CE_GENERIC : (p.nq_root == 3 && p.nv_root == 3) ? CE_LOCO3 : CE_LOCO;
  const int act = a.pi.n_layers > 1 ? a.pi.hidden_act : ACT_IDENTITY;
  const dim3 g(a.N), b(64);
  // (planar locomotion with the usual two uniform hidden layers -- [32, 32] split form, [64, 64]
  // full form -- + head: depth and width are compile-time too)
  const bool nl3 = a.pi.n_layers == 3;
  const int hw = nl3 && a.pi.dims[1] == a.pi.dims[2] ? a.pi.dims[1] : 0;
  // (+ the frame skip of the benchmark recipes: HalfCheetah 5 with the [32, 32] tanh actor,
  // Hopper / Walker 4 with the [64, 64] ReLU one)
  const int fs = env == CE_LOCO3 ? p.frame_skip : 0;
  if (a.prof || a.lds_actor) {  // the probe / test instances: the HalfCheetah bench configuration only
    if (!(split && env == CE_LOCO3 && act == ACT_TANH && hw == 32 && fs == 5)) return hipErrorInvalidValue;
    if (a.prof && a.lds_actor)
      hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_TANH, 3, 32, 5, true, false>), g, b, lds, s, a);
    else if (a.prof)
      hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_TANH, 3, 32, 5, true>), g, b, lds, s, a);
    else
      hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_TANH, 3, 32, 5, false, false>), g, b, lds, s, a);
  } else if (split && env == CE_LOCO3 && act == ACT_TANH && hw == 32 && fs == 5)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_TANH, 3, 32, 5>), g, b, lds, s, a);
  else if (split && env == CE_LOCO3 && act == ACT_TANH && hw == 32 && fs == 4)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_TANH, 3, 32, 4>), g, b, lds, s, a);
  else if (!split && env == CE_LOCO3 && act == ACT_RELU && hw == 64 && fs == 4)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO3, ACT_RELU, 3, 64, 4>), g, b, lds, s, a);
  else if (!split && env == CE_LOCO3 && act == ACT_RELU && hw == 64 && fs == 5)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO3, ACT_RELU, 3, 64, 5>), g, b, lds, s, a);
  else if (split && env == CE_LOCO3 && act == ACT_TANH && hw == 32)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_TANH, 3, 32>), g, b, lds, s, a);
  else if (split && env == CE_LOCO3 && act == ACT_RELU && hw == 32)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_RELU, 3, 32>), g, b, lds, s, a);
  else if (!split && env == CE_LOCO3 && act == ACT_TANH && hw == 64)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO3, ACT_TANH, 3, 64>), g, b, lds, s, a);
  else if (!split && env == CE_LOCO3 && act == ACT_RELU && hw == 64)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO3, ACT_RELU, 3, 64>), g, b, lds, s, a);
  else if (split && env == CE_LOCO3 && act == ACT_TANH && nl3)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_TANH, 3>), g, b, lds, s, a);
  else if (split && env == CE_LOCO3 && act == ACT_RELU && nl3)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_RELU, 3>), g, b, lds, s, a);
  else if (!split && env == CE_LOCO3 && act == ACT_TANH && nl3)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO3, ACT_TANH, 3>), g, b, lds, s, a);
  else if (!split && env == CE_LOCO3 && act == ACT_RELU && nl3)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO3, ACT_RELU, 3>), g, b, lds, s, a);
  else if (split && env == CE_LOCO3 && act == ACT_TANH)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_TANH>), g, b, lds, s, a);
  else if (split && env == CE_LOCO3 && act == ACT_RELU)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO3, ACT_RELU>), g, b, lds, s, a);
  else if (!split && env == CE_LOCO3 && act == ACT_TANH)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO3, ACT_TANH>), g, b, lds, s, a);
  else if (!split && env == CE_LOCO3 && act == ACT_RELU)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO3, ACT_RELU>), g, b, lds, s, a);
  else if (split && env == CE_GENERIC)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_GENERIC, -1>), g, b, lds, s, a);
  else if (!split && env == CE_GENERIC)
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_GENERIC, -1>), g, b, lds, s, a);
  else if (split)
    hipLaunchKernelGGL((rollout_chain_kernel<true, CE_LOCO, -1>), g, b, lds, s, a);
  else
    hipLaunchKernelGGL((rollout_chain_kernel<false, CE_LOCO, -1>), g, b, lds, s, a);
  return hipGetLastError();
}

}  // namespace ia

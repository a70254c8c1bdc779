// Device-resident training engine: argument blocks shared by the HIP kernels
// (csrc/kernels/engine.hip, ppo.hip) and their host launchers / bindings.
//
// The engine keeps a whole adversarial-imitation round on the GPU (SURVEY §7.4
// items 2-3): env state, policy / value / reward nets, rollout buffer, GAE, the
// PPO update and the generator replay buffer never leave HBM.
#pragma once
#include <stdint.h>

#include "ia/common.h"
#include "ia/envs.h"

namespace ia {

constexpr int kWaveMaxLayers = 4;
constexpr int kWaveMaxDim = 64;  // one lane per unit
constexpr int kEngineMaxObs = 64;

// An MLP evaluated by ONE wave (lane j = unit j), used per env inside the rollout kernel.
struct WaveMLP {
  int n_layers;
  int dims[kWaveMaxLayers + 1];
  int hidden_act;
  int out_act;
  const float* W[kWaveMaxLayers];  // [dout][din] row-major (nn.Linear layout)
  const float* b[kWaveMaxLayers];
  const float* norm_mean;  // optional input RunningNorm (eval mode)
  const float* norm_var;
  float norm_eps;
};

enum RewardTransform : int { REW_RAW = 0, REW_SOFTPLUS = 1 };

// Serial part of a device rollout (rollout.hip): actor sampling + env physics.
struct RolloutArgs {
  EnvParams P;
  int max_steps;  // TimeLimit horizon
  int T;          // steps per env this call
  int N;          // envs
  uint64_t seed;  // action-sampling stream
  long long step0;  // global step counter (decorrelates calls)
  // persistent env state (device)
  float* state;      // [N][state_dim]
  uint64_t* rng;     // [N]
  int* elapsed;      // [N]
  float* ep_ret;     // [N] running env return (Monitor)
  float* cur_obs;    // [N][D]  (policy's _last_obs)
  float* cur_start;  // [N]     (_last_episode_starts)
  // actor: trunk + action head, input RunningNorm (eval mode) in pi.norm_*
  WaveMLP pi;
  const float* log_std;  // [A] (Gaussian) or nullptr (Categorical)
  const float* act_low;  // [A] Box bounds for clipping
  const float* act_high;
  int n_actions;  // >0: Categorical over n_actions
  // optional ExplorationWrapper schedule: explore_mode[t] != 0 -> every env takes a uniform
  // random action at step t (Box.sample / Discrete.sample) instead of the policy's
  const int* explore_mode;  // [T] or nullptr
  // deterministic actions (evaluation, SB3 predict(deterministic=True)): the Gaussian mean /
  // the categorical argmax -- the sampling noise is zero
  int deterministic;
  // outputs, [T][N] (+ trailing feature dim)
  float* obs_buf;
  float* act_raw;   // sampled (unclipped) action, PPO buffer
  float* act_env;   // action given to the env (clipped), replay buffer / reward
  float* env_rew;
  float* starts;
  float* dones;
  float* trunc;     // 1 where the episode was cut by the TimeLimit (not terminated)
  float* next_obs;  // terminal obs on done
  float* ep_ret_out;  // episode return where done
  // optional phase-clock probe (tools/rollout_breakdown.py): [N][5] int64 = core-clock cycles spent
  // in actor+sampling, env physics, observation, step tail, and the step count; the HalfCheetah
  // bench configuration only
  long long* prof;
  // test hook (tests/engine/test_rollout_probe.py): the HalfCheetah configuration with the LDS
  // split-form actor instead of the row form, to check the two are bitwise equal
  int lds_actor;
};

// Parallel part (engine.hip): per transition V(s), log pi(a|s), the TimeLimit bootstrap
// boot = gamma V(s') on truncation, and the reward
// rewards = (rew_enabled ? R(s, a, s', d) [+ shaping] : env_rew) + boot; rows T*N .. T*N+N
// give last_values = V(cur_obs). rew_raw (optional) keeps R before output normalisation.
struct RolloutPostArgs {
  int T, N;
  int D;          // obs dim
  int A;          // act buffer width (1 for Categorical)
  int n_actions;  // >0: Categorical (acts hold the index)
  float gamma;
  const float* obs;
  const float* act_raw;
  const float* act_env;
  const float* next_obs;
  const float* dones;
  const float* trunc;
  const float* env_rew;
  const float* cur_obs;
  WaveMLP pi, vf;
  const float* log_std;
  int rew_enabled;
  WaveMLP rew;
  int use_state, use_action, use_next_state, use_done;
  int rew_transform;
  int shaped;
  WaveMLP pot;
  float shaping_gamma;
  float* values;
  float* logp;  // nullptr: skip the actor (sampling-only rollouts)
  float* boot;
  float* rewards;
  float* rew_raw;
  float* last_values;
};

// NormalizedRewardNet output normalisation over a rollout, step by step in env order:
// rewards[t][n] = (rew_raw[t][n] - mean) / sqrt(var + eps) + boot[t][n], then the running
// (mean, var, count) are Chan-merged with step t's batch moments (over the N envs, or the
// global ones given in step_stats[t] = (count, mean, biased var) under data parallelism).
struct OutNormArgs {
  int T, N;
  const float* rew_raw;
  const float* boot;
  float* rewards;
  float* mean;   // [1] running state, updated in place
  float* var;    // [1]
  float* count;  // [1] (float)
  int* count_i;  // optional: the module's int32 count, read / written instead of count
  float eps;
  const float* step_stats;  // [T][3] or nullptr
};

// One PPO update (all epochs x minibatches) in one persistent workgroup.
struct PPOArgs {
  int D, A;             // obs dim, action dim (Gaussian) / n_actions (Categorical)
  int discrete;
  int n_pi, n_vf;       // layer counts (incl. head)
  int pi_dims[kWaveMaxLayers + 1];
  int vf_dims[kWaveMaxLayers + 1];
  int hidden_act;
  // flat parameter / grad / Adam state vectors; layout = torch module order
  float* params;
  float* grads;
  float* exp_avg;
  float* exp_avg_sq;
  int n_params;
  int pi_w_off[kWaveMaxLayers], pi_b_off[kWaveMaxLayers];
  int vf_w_off[kWaveMaxLayers], vf_b_off[kWaveMaxLayers];
  int log_std_off;  // -1 if none
  // features RunningNorm (train mode: stats updated from each minibatch)
  float* norm_mean;
  float* norm_var;
  float* norm_count;  // float counter (exact up to 2^24)
  int* norm_count_i;  // optional: the module's int32 counter, read / written instead of norm_count
  float norm_eps;
  int has_norm;
  // data: flat rollout [rows]
  const float* obs;
  const float* acts;
  const float* old_logp;
  const float* adv;
  const float* returns;
  const int* perm;  // [n_epochs][rows]
  int rows, batch, n_epochs;
  // hyper-parameters
  float clip_range, ent_coef, vf_coef, max_grad_norm;
  float lr, beta1, beta2, adam_eps;
  int normalize_advantage;
  float* adam_step;  // running step count (float)
  // diagnostics [5]: entropy_loss, pg_loss, value_loss, clip_fraction, approx_kl (sums over minibatches)
  float* stats;
  int zero_stats;  // mode 0 fast path: the prep launch zeroes stats (no separate memset)
  int mode;  // 0: full persistent update; 1: one minibatch -> grads only; 2: apply clip+Adam from grads
  int mb_index;  // minibatch index for mode 1 (epoch * n_mb + mb)
  unsigned long long* prof;  // optional [10] cycle counters per phase
  int rc_gmax;   // mode 0 fast path: max cooperating workgroups per minibatch (0 = default kMaxRcGroups)
  int rc_cw;     // mode 0 fast path: rows per chunk override (0 = 64 for <= 32-wide nets, 32 otherwise)
  // fail-fast for the cooperating workgroups (mode 0 fast path): a bounded spin that gives up
  // ORs 1 into *err (persistent, host-checked; may be null) besides the per-launch flag
  unsigned* err;
  unsigned spin_limit;  // sleeps before a spin gives up (0 = default 2^22)
  int debug_stall;      // test knob: the last working workgroup never publishes (forces a timeout)
  int rc_cus;           // CU count to plan against (0 = query the current device)
};

// CUs of the current device (cached per device; IMITATION_AMD_PPO_CUS overrides, e.g. tests).
int device_cu_count();

// Geometry + workspace of the register-chained PPO kernel (ppo_rc.hip), planned on the host.
constexpr int kMaxRcItems = 64;
constexpr int kMaxRcGroups = 64;  // cooperating workgroups per minibatch (one per CU, co-resident)
struct PPORcGeo {
  int din[2][kWaveMaxLayers], dout[2][kWaveMaxLayers];
  int w_off[2][kWaveMaxLayers], ldw[2][kWaveMaxLayers], b_off[2][kWaveMaxLayers];
  int h_off[2][kWaveMaxLayers], ldh[2][kWaveMaxLayers];  // ldh / ldz: floats per image column
  int z_off[2][kWaveMaxLayers], ldz[2][kWaveMaxLayers], db_off[2][kWaveMaxLayers];
  int ls_off, lsp_off, nm_off, red_off, param_lds;
  int zero_off;  // 64 floats of zeros (never written): operand of the padding dW items
  int trash_off;   // 64 floats: Adam target of padding elements
  int lds_floats;  // whole image size (zeroed at kernel start)
  int n_items;
  int n_witems;            // items [0, n_witems) are dW tiles
  int items[kMaxRcItems];  // q | layer << 1 | kind << 3 (0 W tile, 1 bias, 2 log_std) | out tile << 5 | in tile << 9
  int dp;                  // padded obs row stride of xraw
  int kt;                  // 16-wide tiles per hidden layer (2: width <= 32, 4: width <= 64)
  int cw;                  // rows per chunk (one fwd/bwd pass of a workgroup)
  int ksteps;              // 32-row K-steps of a dW tile (split-bf16 images padded to >= 32 rows)
  int bf3;                 // split-bf16 forward / dX weight images (ppo_rc_kernel.h bf3_tile)
  int wf_off[2][kWaveMaxLayers], wt_off[2][kWaveMaxLayers];  // their offsets (floats; hi then lo)
  int nch;                 // chunks per workgroup per minibatch
  int G;                   // cooperating workgroups per minibatch (minibatch = G * nch * cw rows)
  int nw;                  // waves per workgroup (8: <= 32-wide nets, 4: 64-wide nets at 1 wave / SIMD)
  float* xraw;             // [K][G*nch][64][dp] gathered raw observations (one 64-row slot per chunk)
  float* acts;             // [K][G*nch][64][16]
  float* rowd;             // [K][G*nch][64][4] old_logp, normalised advantage, return
  float* mom;              // [K][128] per-minibatch obs mean / var
  float* slab;             // [2][G][n_items][256] per-workgroup gradient partials (G > 1)
  float* red;              // [2][n_items][256] reduced gradients (two-level exchange)
  int xchg2;               // two-level exchange: item id reduced by workgroup id % G, then shared
  unsigned* sync;          // [0] arrival counter, [1] timeout flag, [2] second-level arrivals (zeroed per launch)
  // net split (G == 1): workgroup q runs net q only (actor 0 / critic 1) on its own CU; the
  // two meet once per minibatch to sum |g|^2 for clip_grad_norm_. Items of net q: weight tiles
  // [wbase[q], wbase[q] + nwit[q]), bias / log_std vectors [bbase[q], bbase[q] + nbit[q]).
  int ns;
  int wbase[2], nwit[2], bbase[2], nbit[2];
  int xstash;  // LDS offset of the G x 256-float partial stash (item-split first level, G > 16; -1: none)
  // XCD placement (speed only, never correctness): > 1 launches xcd x the workgroups and only
  // blocks b % xcd == 0 work (logical id b / xcd), so under the observed round-robin dealing of
  // blocks over the 8 XCDs every cooperating workgroup shares one XCD's L2
  int xcd;
};

}  // namespace ia

// Host launch entry points of every HIP kernel (raw pointers + stream only, so
// that the torch-facing binding TUs never include device code and the kernel
// TUs never include torch headers).  All launchers are graph-capture safe: no
// allocation, no synchronisation.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "ia/engine.h"
#include "ia/tmlp.h"

namespace ia {

// ---- tmlp.hip: fused tiny-MLP
int tmlp_waves_for(const MLPDesc& d);
size_t tmlp_slab_floats(const MLPDesc& d, int B);
hipError_t tmlp_forward(const MLPDesc& d, const float* X, int B, float* Y, hipStream_t s);
hipError_t tmlp_backward(const MLPDesc& d, const float* X, const float* dY, int B, float* dX, const MLPGrads& g,
                         float* slab, hipStream_t s);

// Fused discriminator loss on top of the backward kernel (kDisc): writes the gradient
// slab [nblk][n_params] (flat order W0, b0, W1, b1, ...) and stats slab [nblk][kDiscStats].
int tmlp_disc_blocks(const MLPDesc& d, int B);
hipError_t tmlp_disc_fwd_bwd(const MLPDesc& d, const float* X, int B, const DiscLoss& dl, float* slab, hipStream_t s);

// ---- disc.hip: fused discriminator update
struct DiscGatherArgs {
  int mb;  // rows per side: X holds 2*mb rows, expert first
  int din, obs_dim, act_width;
  int use_state, use_action, use_next_state, use_done;
  int act_discrete;
  const int64_t* e_idx;
  const int64_t* g_idx;
  const float *e_obs, *e_next_obs, *e_acts;
  const int64_t* e_acts_i;
  const bool* e_dones;
  const float *g_obs, *g_next_obs, *g_acts;
  const int64_t* g_acts_i;
  const bool* g_dones;
  const float* shift;  // per-column shift for the moment sums (running mean) or null
  float* X;            // [2*mb][din]
  float* partials;     // [nblk][2][din]
};
struct DiscNormArgs {
  int mode;  // 0: reduce partials + merge; 1: reduce partials -> sums only; 2: merge from sums
  int mb, din, nblk;
  double* sums;  // [2][din] (modes 1, 2)
  int n_total;   // rows behind sums (mode 2: all DP ranks)
  const float* partials;
  const float* shift;
  float *rew_mean, *rew_var;
  int* rew_count;
  int pol_cols;
  float *pol_mean, *pol_var;
  int* pol_count;
  // non-null: record this batch's (mean[pol_cols], var[pol_cols], n) here instead of
  // merging into pol_mean / pol_var (applied later, in order, by pol_norm_merge)
  float* pol_defer;
};
struct DiscAdamArgs {
  int n_params, nblk, stats_nblk;
  int reduce, adam;  // reduce slab -> grad; apply Adam (from reduced or from grads[])
  const float* slab;
  const float* stats_slab;
  float* stats_out;  // [kDiscStats] or null
  float* grads;
  float *params, *exp_avg, *exp_avg_sq;
  float beta1, beta2, eps, weight_decay, step_size, bc2_sqrt;
  // device step counter (already incremented for this step) or null: with it the bias
  // corrections come from the device (graph-capturable) with learning rate lr
  const float* step;
  float lr;
  int decoupled;      // AdamW: p *= 1 - lr * weight_decay (else L2: g += weight_decay * p)
  float stats_scale;  // stats_out = scale * sums (0: 1)
};
int disc_gather_blocks(int mb);
hipError_t disc_gather(const DiscGatherArgs& a, hipStream_t s);
hipError_t disc_norm(const DiscNormArgs& a, hipStream_t s);
hipError_t disc_adam(const DiscAdamArgs& a, hipStream_t s);
// Chan-merge n_slots deferred batch records ([slot][2 * cols + 1]) into a RunningNorm, in
// slot order (bitwise the merges disc_norm would have done in place).
hipError_t pol_norm_merge(float* mean, float* var, int* count, const float* defer, int n_slots, int cols,
                          hipStream_t s);

// ---- airl_disc.hip: fused AIRL discriminator update (gather, norms, fwd/loss/bwd; Adam = disc_adam)
constexpr int kAirlMaxLayers = 4;
struct AirlNet {
  int n_layers;
  int dims[kAirlMaxLayers + 1];
  int hidden_act;  // output layer is identity
  const float* W[kAirlMaxLayers];  // [dout][din] fp32 (nn.Linear layout)
  const float* b[kAirlMaxLayers];
  int param_off;                   // offset of this net in a gradient slab row (reward nets)
  int w_off[kAirlMaxLayers], b_off[kAirlMaxLayers];  // offsets within the net
};
struct AirlDiscArgs {
  int mb;         // rows per side (2 * mb per minibatch, expert first)
  int D, A;       // obs dim, action dim (Box) / n_actions (Discrete)
  int aw;         // action width in the base input (A, or n_actions one-hot)
  int aw_pi;      // stored action width for log pi (A, or 1: the index)
  int act_discrete;
  int use_state, use_action, use_next_state, use_done, din_b;
  const int64_t* e_idx;  // [B] (minibatch k uses [k * mb, (k + 1) * mb))
  const int64_t* g_idx;
  const float *e_obs, *e_next_obs, *e_acts;
  const int64_t* e_acts_i;
  const bool* e_dones;
  const float *g_obs, *g_next_obs, *g_acts;
  const int64_t* g_acts_i;
  const bool* g_dones;
  // gathered minibatch
  float *Xb, *S, *S2, *Act, *Done;
  float* partials;  // [gather blocks][2][din_b + 2 D]
  int gather_blocks;
  double* sums;     // [2][din_b + 2 D] (DP modes)
  // RunningNorms: b base input, p potential, q policy features (null = none)
  float *b_mean, *b_var, *p_mean, *p_var, *q_mean, *q_var;
  int *b_count, *p_count, *q_count;
  float eps_b, eps_p, eps_q;
  int merge_b, merge_p, merge_q;  // train mode (update stats)
  float* nrm;  // [4][256]: (mean[128], rstd[128]) for policy, base, potential(s'), potential(s)
  float* q_defer;  // merge_q deferred: the s moments (mean[128], var[128]) for airl_q_merge, else null
  AirlNet pol, base, pot;
  const float* log_std;  // [A] (Gaussian) or null
  float gamma;           // shaping discount
  float scale;           // dBCE/dlogit scale (mean over 2 mb rows * mb / B)
  int n_params;          // base + potential parameters (slab row)
  float* slab;           // [n_mb * fwd blocks][n_params]
  float* stats_slab;     // [n_mb * fwd blocks][kDiscStats]
  unsigned long long* prof;  // optional phase cycle counters (block 0) [8]
};
struct AirlPlan {
  int ldp, ldr, ld_ht, dmax_pad;
  int pimg_bytes, rimg_bytes, ht_bytes;
  int wf_off[3][kAirlMaxLayers];  // pre-staged weight images: 0 policy, 1 base, 2 potential
  int wt_off[3][kAirlMaxLayers];  // transposed images (reward nets, layers >= 1)
  int rimg_off, scratch_off, lds_bytes;
};
int airl_gather_blocks(int mb);
int airl_fwd_blocks(int mb);
bool airl_plan(const AirlDiscArgs& a, AirlPlan& p);
hipError_t airl_gather(const AirlDiscArgs& a, int k, hipStream_t s);
hipError_t airl_norm(const AirlDiscArgs& a, int mode, int n_total, hipStream_t s);
// policy-norm merges deferred by airl_norm (q_defer) for `count` staged minibatches whose nrm /
// q_defer rows are `stride` floats apart, in staging order; n rows per minibatch
hipError_t airl_q_merge(const AirlDiscArgs& a, int count, long long stride, int n, hipStream_t s);
hipError_t airl_fwd_bwd(const AirlDiscArgs& a, const AirlPlan& p, int k, hipStream_t s);

// ---- pref_rm.hip: fused preference reward-model minibatch (gather, fwd, bwd; Adam = disc_adam)
struct PrefRmArgs {
  int n, L, din;          // pairs in the minibatch, fragment length, reward-net input width
  int ds, da, dns;        // state / action / next-state column widths of the input (0: unused)
  const float *s_all, *a_all, *ns_all, *d_all;  // dataset rows [pair * 2L + t][*] (fragment 1, then 2)
  const int64_t* idx;     // [n] pair ids of this minibatch
  const float* prefs_all;  // [P]
  const float* gt_all;     // [P][2][L] ground-truth rewards or null
  AirlNet net;             // reward MLP, scalar identity head; offsets into the flat parameters
  float *rmean, *rvar;     // input RunningNorm (null: none)
  int* rcount;
  float eps;
  int merge;               // train mode: merge the minibatch moments
  float* X;                // [2nL][din]
  float* partials;         // [blocks][2 * din] shifted column sums
  double* sums;            // [2 * din] their block-order sum (data parallel: then all-reduced)
  unsigned* cnt;           // [1] zero-initialised gather-block counter (self-resetting)
  float* old_mv;           // [256] running mean / var before this minibatch
  int* old_cnt;            // [1]
  float* nrm;              // [256] mean / rstd the forward normalised with
  float* r;                // [2nL] rewards
  float* slab;             // [blocks][n_params]
  float* pstats;           // [n][8] per pair: loss, correct, ground-truth loss
  float discount, threshold, noise, gscale;  // gscale: the trainer's loss factor 1 / batch_size
  float* step;             // Adam step counter (device), bumped by the gather
  int n_params;
  const int* cursor;       // device epoch cursor or null: pair ids at idx + *cursor * idx_stride
  int idx_stride;
};
struct PrefPlan {
  int ldr, ld_ht, dmax_pad, rimg_bytes, ht_bytes;
  int wf_off[kAirlMaxLayers], wt_off[kAirlMaxLayers];
  int rimg_off, scratch_off, lds_bytes;
};
int pref_rm_blocks(int n_pairs, int L);
bool pref_rm_plan(const PrefRmArgs& a, PrefPlan& p);
hipError_t pref_rm_gather(const PrefRmArgs& a, hipStream_t s);
hipError_t pref_rm_fwd(const PrefRmArgs& a, const PrefPlan& p, int n_total, hipStream_t s);
hipError_t pref_rm_bwd(const PrefRmArgs& a, const PrefPlan& p, hipStream_t s);
// epoch end: metrics of the epoch's minibatches [n * 8] -> all[*cursor * n * 8 ...], ++*cursor
hipError_t pref_rm_epoch_end(const float* metrics, float* all, int n, int* cursor, hipStream_t s);

// ---- wlin.hip: wide MLP layers (129..1024) on MFMA, bias / activation fused
struct WideLinArgs {
  int M, N, K;           // rows, layer outputs, layer inputs
  const float* X;        // [M][K] layer input (fwd, dW)
  const float* W;        // [N][K] nn.Linear weight
  const float* b;        // [N] or null (fwd)
  float* Y;              // [M][N] (fwd)
  int act;               // fwd: activation of Y; dx: activation that produced H
  const float* dZ;       // [M][N] gradient at this layer's pre-activation output (dx, dW)
  float* G;              // [M][K] (dx)
  const float* H;        // [M][K] activation output whose derivative multiplies G, or null
  const float* scale;    // [K] per-column factor of G (input normaliser rstd) or null
  float* dW;             // [N][K] (dW)
  float* db;             // [N] or null (dW)
  int accumulate;        // dW / db: add into existing values
  float* ws;             // dW split-M partials: wlin_dw_ws_floats(M, N, K) floats (null if 0)
  int* cnt;              // dW: wlin_dw_tiles(N, K) zero-initialised tile counters (self-resetting)
};
int wlin_dw_tiles(int N, int K);
int wlin_dw_splits(int M, int N, int K);
size_t wlin_dw_ws_floats(int M, int N, int K);
hipError_t wlin_forward(const WideLinArgs& a, hipStream_t s);
hipError_t wlin_backward_x(const WideLinArgs& a, hipStream_t s);
hipError_t wlin_backward_w(const WideLinArgs& a, hipStream_t s);

// ---- dagger.hip: device env step of the DAgger collector (one workgroup per env)
struct DaggerEnvArgs {
  EnvParams P;
  int N, max_steps, sdim;
  int mode;  // 0: step with the given actions; 1: reset every env
  float* state;
  uint64_t* rng;
  int* elapsed;
  float* ep_ret;            // running episode return
  const int64_t* act_i;     // discrete actions [N] (or null)
  const float* act_f;       // continuous actions [N, act_dim] (or null)
  uint8_t* obs_u8;          // image envs: current frame stack [N, 84, 84, 4], updated in place
  float* obs_f;             // vector envs: current observation [N, obs_dim], updated in place
  float* rew;               // [N] this step
  uint8_t *term, *trunc;    // [N] this step
  uint8_t* term_obs_u8;     // [N, 84, 84, 4] terminal frames (written for done envs)
  float* term_obs_f;        // [N, obs_dim] terminal observations (written for done envs)
  float* ep_ret_out;        // [N] episode return at episode end (else 0)
  int* ep_len_out;          // [N] episode length at episode end (else 0)
  void* obs_rec;            // optional: the pre-step observation is copied here ([N, obs...])
};
hipError_t dagger_env_step(const DaggerEnvArgs& a, hipStream_t s);

// ---- cnn_infer.hip: NatureCNN actor tail for the DAgger collector
// h[B][NH] = relu(X[B][K] . W[NH][K]^T + bias), X / W bf16 (K % 32 == 0, NH % 16 == 0)
hipError_t cnn_fc(const void* X, const void* W, const float* bias, float* H, int B, int K, int NH, hipStream_t s);
// NatureCNN feature-layer backward (cnn_fc.hip): X bf16 [M][K] (NHWC-flattened conv output,
// K = C * HW), dH / Hout fp32 [M][NH], Wt bf16 [K][NH]; dW fp32 [NH][K] in torch's (c, h, w)
// column order, db fp32 [NH], dX bf16 [M][K] (nullptr: not needed)
bool fc_train_ok(int M, int K, int NH, int C, int HW);
// dZb: bf16 [M][NH] scratch; mask_dx: dX = 0 where X <= 0 (X is the post-ReLU conv output, so the conv
// trunk's top-layer ReLU mask is applied once here instead of in every dZ load downstream)
hipError_t fc_backward(const void* X, const float* dH, const float* Hout, const void* Wt, float* dW, float* db, void* dX,
                       void* dZb, int M, int K, int NH, int C, int HW, hipStream_t s, bool mask_dx = false);
struct CnnFcPair {
  const void* X[2];
  const void* W[2];
  const float* bias[2];
  float* H[2];
};
hipError_t cnn_fc_pair(const CnnFcPair& p, int B, int K, int NH, hipStream_t s);
struct CnnHeadArgs {
  const float *h, *W2, *b2;  // h [B, NH], W2 [A, NH], b2 [A]
  int B, NH, A;
  int mode;                  // 0: argmax; 1: Gumbel-max sample
  uint64_t seed;
  uint64_t* counter;         // device call counter (advanced by one per launch), or null
  int64_t* out;              // [B] chosen action
  int64_t* rec_out;          // optional second copy of the action (record slot)
  const int64_t* mix_expert; // optional: expert actions for the beta-mix
  const float* beta;         // device scalar (with mix_expert)
  int64_t* exec_out;         // optional: executed action (u > beta ? own : expert)
};
hipError_t cnn_head(const CnnHeadArgs& a, hipStream_t s);
// expert head (e) + learner head (r, its exec_out mixed with e's action of the same row), one launch
hipError_t cnn_head_pair(const CnnHeadArgs& e, const CnnHeadArgs& r, hipStream_t s);

// ---- bc_head.hip: categorical BC head (logits, loss metrics, dW / db / dh) + ||theta||^2 in
// one launch (B <= 64, NH 256 or 512, A <= 8)
struct BcHeadArgs {
  const float *h, *W, *b;   // features [B, NH] (16-B aligned), head weight [A, NH] (16-B aligned), bias [A]
  const int64_t* acts;      // [B]
  int B, NH, A;
  float ent_w, l2_w;
  const float* params;      // flat parameter bucket (16-B aligned), n_params floats
  long n_params;
  float *dW, *db, *dh;      // gradient slots (written, not accumulated), dh [B, NH]
  float* metrics;           // [7]: neglogp, entropy, ent_loss, prob_true_act, l2_norm, l2_loss, loss
  float* partials;          // [bc_head_sumsq_blocks(n_params)]
  unsigned* cnt;            // zero-initialised hand-off counter (left zero)
  long long* prof;          // optional phase clocks of block 0 (tools/bc_head_probe.py)
};
bool bc_head_ok(int B, int NH, int A);
int bc_head_sumsq_blocks(long n_params);
hipError_t bc_head_train(const BcHeadArgs& a, hipStream_t s);

// ---- optim.hip: fused Adam / AdamW over a flat fp32 buffer
struct AdamArgs {
  float *params, *grads, *exp_avg, *exp_avg_sq;
  float* step;        // device step counter: already incremented for this step, or (cnt != null)
                      // incremented by the kernel (every block uses *step + 1, the last block to
                      // finish stores it)
  unsigned* cnt;      // zeroed hand-off counter for the in-kernel increment (left zero), or null
  int64_t n;
  float lr, beta1, beta2, eps, weight_decay;
  int decoupled;  // AdamW: p *= 1 - lr * wd
  int maximize;
  int zero_grad;  // clear the gradient after reading it
  // optional, block 0 after its update: app_all[*app_cursor][0 .. app_n) = app_src, ++*app_cursor
  // (a graphed BC epoch's per-step metrics row; saves the append launch)
  const float* app_src;
  float* app_all;
  int* app_cursor;
  int app_n;
};
struct ConvReduceMulti;
// red (optional): conv layers' deferred weight-gradient reductions whose dW / db slots lie in
// grads (16-B aligned ranges); their elements are summed from the slabs and updated by blocks of
// this launch (the BC step's conv_reduce_multi folded into Adam: bitwise the two launches)
hipError_t adam_flat(const AdamArgs& a, hipStream_t s, const ConvReduceMulti* red = nullptr);

// ---- rl.hip: GAE scan over [T, N]
hipError_t gae_launch(const float* rew, const float* val, const float* starts, const float* last_val, const float* dones,
                      int T, int N, float gamma, float lam, float* adv, float* ret, hipStream_t s,
                      float* mom = nullptr);  // optional [N][4] return / advantage moments
// E keyed pseudo-random permutations of [0, n) (Feistel + cycle walking), out [E, n] int32
hipError_t perm_feistel(int E, int n, uint64_t seed, int* out, hipStream_t s);
// categorical head: log-prob of the taken action + entropy from raw logits [B][A], and the
// logit gradient for upstream gradients g_lp / g_ent (either may be nullptr = 0)
hipError_t cat_eval_fwd(const float* z, const int64_t* act, int B, int A, float* logp, float* ent, hipStream_t s);
hipError_t cat_eval_bwd(const float* z, const int64_t* act, int B, int A, const float* g_lp, const float* g_ent, float* dz,
                        hipStream_t s);
// BC loss on a categorical head: metrics [neglogp, entropy, ent_loss, prob_true_act, l2_norm,
// l2_loss, loss] (flat/n: parameter buffer for l2_norm, part: sumsq_nparts(n) floats), and the
// logit gradient for an upstream gradient g[7] of the metric vector
int sumsq_nparts(long n);
hipError_t bc_cat_loss_fwd(const float* z, const int64_t* act, int B, int A, const float* flat, long n, float* part,
                           float ent_w, float l2_w, float* out, float* loss_out, hipStream_t s);
hipError_t bc_cat_loss_bwd(const float* z, const int64_t* act, int B, int A, const float* g, const float* g_loss,
                           float ent_w, float* dz, hipStream_t s);

// ---- norm.hip: RunningNorm update (batch moments + Chan merge + count) and normalise, one
// workgroup (B * D <= 2^20, D <= 256); y == nullptr: statistics only
bool running_norm_ok(int B, int D);
// ws: running_norm_ws_floats(B, D) floats (multi-workgroup path for large B; nullptr -> one workgroup)
size_t running_norm_ws_floats(int B, int D);
// ema_inv_lr / ema_num_batches (both or neither): EMANorm's merge with decay ema_decay
hipError_t running_norm(const float* x, int B, int D, float* mean, float* var, int* count, float eps, int update, float* y,
                        float* ws, hipStream_t s, float* ema_inv_lr = nullptr, int* ema_num_batches = nullptr,
                        float ema_decay = 0.f);

// ---- gather.hip: one-launch multi-field row gather (row r <- source row b[r] * n_envs + e[r],
// or b[r] when e == nullptr)
constexpr int kGatherMax = 8;
struct GatherField {
  const void* src;
  void* dst;
  int64_t row_bytes;
  int64_t rows;  // source rows: out-of-range indices produce zero rows, never a stray read
};
struct GatherArgs {
  GatherField f[kGatherMax];
  int k;
};
hipError_t gather_rows(const GatherArgs& a, const int64_t* b, const int64_t* e, int n_envs, int n, hipStream_t s);
// rows perm[*cursor * n .. + n) (int32 ids) of every source (graph-captured epochs)
hipError_t gather_rows_cursor(const GatherArgs& a, const int* perm, const int* cursor, int n, hipStream_t s,
                              float* inc = nullptr);  // inc: ++*inc by one thread (an optimizer's step counter)
// all[*cursor * n ..] = src[0 .. n), ++*cursor
hipError_t append_at_cursor(const float* src, float* all, int n, int* cursor, hipStream_t s);

// ---- tabular.hip: MCE-IRL soft value iteration / occupancy (fp64, one workgroup, LDS-resident
// vectors: S * (A + 1) doubles <= 150 KB) and KDE log-density scoring (fp64, d <= kKdeMaxDim)
bool soft_vi_fits(int S, int A);
hipError_t soft_value_iteration(const double* T, const double* R, int S, int A, int H, double gamma, double* V, double* Q,
                                double* P, hipStream_t s);
hipError_t occupancy_measures(const double* T, const double* P, const double* D0, int S, int A, int H, double* D,
                              hipStream_t s);
constexpr int kKdeMaxDim = 32;
int kde_splits(int NQ, int N);
// kind: 0 gaussian, 1 exponential, 2 tophat, 3 epanechnikov, 4 linear, 5 cosine;
// pmax / psum: kde_splits(NQ, N) * NQ doubles of scratch; out[i] = logsumexp_j log k + offset
hipError_t kde_score(const double* q, const double* x, int NQ, int N, int d, double inv_h, int kind, double offset,
                     double* pmax, double* psum, double* out, hipStream_t s);

// ---- pref.hip: Bradley-Terry preference loss over fragment pairs
hipError_t pref_loss_fwd(const float* r1, const float* r2, const float* prefs, int P, int L, float discount,
                         float threshold, float noise, float* probs, float* losses, float* coef, hipStream_t s);
hipError_t pref_loss_bwd(const float* coef, const float* gout, int P, int L, float discount, float* d1, float* d2,
                         hipStream_t s);

// ---- rollout.hip / engine.hip: device-resident rollout (serial actor + env chain, then the
// parallel value / log-prob / bootstrap / learned-reward pass)
bool rollout_split_form(const WaveMLP& m);
size_t rollout_lds_bytes(const RolloutArgs& a);
hipError_t rollout_launch(const RolloutArgs& a, hipStream_t s);
size_t rollout_post_lds_bytes(const RolloutPostArgs& a);
hipError_t rollout_post_launch(const RolloutPostArgs& a, hipStream_t s);
hipError_t reward_outnorm_launch(const OutNormArgs& a, hipStream_t s);

// ---- ppo_rc.hip: register-chained single-rank PPO update (falls back to ppo.hip)
bool ppo_rc_plan(const PPOArgs& a, PPORcGeo& g, size_t& lds_bytes);
size_t ppo_rc_workspace_floats(const PPOArgs& a);
hipError_t ppo_rc_launch(const PPOArgs& a, float* workspace, hipStream_t s);

// ---- ppo.hip: persistent PPO update
size_t ppo_lds_bytes(const PPOArgs& a);
hipError_t ppo_launch(const PPOArgs& a, hipStream_t s);

// ---- conv.hip: NHWC implicit-GEMM convolutions (NatureCNN / reward CNN), bf16 MFMA
struct ConvGeo {
  int B, H, W, C;  // input NHWC
  int KH, KW, S;   // kernel, stride
  int OH, OW, N;   // output NHWC
  int P;           // zero padding (symmetric; > 0 only for stride 1 with C % 8 == 0)
  int Kp;          // GEMM K = KH*KW*C rounded up to 32; weights [N][Kp] zero-padded
};
bool conv_geo_ok(const ConvGeo& g);
// one-launch weight packing for a conv stack (ops/conv.py): fp32 [N][C][KH][KW] -> bf16
// [N][KH][KW][C] and optionally bf16 [C][KH][KW][N]
constexpr int kMaxPack = 8;
struct ConvPackLayer {
  const float* w;
  void* wb;  // bf16
  void* wt;  // bf16, nullptr: not needed
  int N, C, KH, KW;
  int t_hwc;  // wt layout: 0 [C][KH][KW][N] (conv dgrad), 1 [KH][KW][C][N] (NHWC-flattened FC)
};
struct ConvPackArgs {
  ConvPackLayer layer[kMaxPack];
  int n;
};
struct GatherArgs;
// ga (optional): a cursor-indexed row gather (gather_rows_cursor) run in the same launch
hipError_t conv_pack_weights(const ConvPackArgs& a, hipStream_t s, const GatherArgs* ga = nullptr, const int* perm = nullptr,
                             const int* cursor = nullptr, int gn = 0, float* inc = nullptr);
// two same-geometry unpadded convs (+ bias + ReLU) in one launch: X/W/bias/Y of set z
struct ConvPair {
  const void* X[2];
  const void* W[2];
  const float* bias[2];
  void* Y[2];
};
hipError_t conv_fwd_pair(int in_kind, const ConvPair& p, const ConvGeo& g, float in_scale, int relu, hipStream_t s);
void conv_wgrad_blocks(const ConvGeo& g, int* nblk, int* m_per_block);
size_t conv_wgrad_slab_floats(const ConvGeo& g);
// deferred wgrad reductions (conv_wgrad with dW == nullptr leaves its block partials in slab):
// every layer's slab -> dW (torch layout) / db in one launch
struct ConvReduceMulti {
  int n;
  ConvGeo g[kMaxPack];
  const float* slab[kMaxPack];
  float* dW[kMaxPack];
  float* db[kMaxPack];
  int nblk[kMaxPack];  // filled by conv_reduce_multi
};
hipError_t conv_reduce_multi(const ConvReduceMulti& r, hipStream_t s);
// in_kind: 0 fp32, 1 bf16, 2 uint8 input; weights bf16 [N][KH][KW][C]; Y bf16 [B*OH*OW][N]
hipError_t conv_forward(int in_kind, const void* X, const void* Wb, const float* bias, void* Y, const ConvGeo& g,
                        float in_scale, int relu, hipStream_t s);
// split-K form (BC-size batches; other summation order than conv_forward): 16 x 16 tiles of 2 or 4
// waves, each wave's k-steps' loads at once, LDS sum in wave order
bool conv_forward_sk_ok(const ConvGeo& g);
hipError_t conv_forward_sk(int in_kind, const void* X, const void* Wb, const float* bias, void* Y, const ConvGeo& g,
                           float in_scale, int relu, hipStream_t s);
// dW fp32 [N][KH][KW][C], db fp32 [N] (may be null); slab of conv_wgrad_slab_floats
hipError_t conv_wgrad(int in_kind, const void* X, const void* dY, const void* Y, float* slab, float* dW, float* db,
                      const ConvGeo& g, float in_scale, int relu_out, hipStream_t s);
// one layer's weight-gradient partials (slab, as conv_wgrad with dW == nullptr; bf16 X) and its data
// gradient (as conv_dgrad with Xp = X) in ONE launch; small unpadded batches (conv_back_pair_ok)
bool conv_back_pair_ok(const ConvGeo& g);
hipError_t conv_back_pair(const void* X, const void* dY, const void* Y, float* slab, const void* Wt, void* dZp,
                          const ConvGeo& g, int relu_out, int relu_in, hipStream_t s);
// dZp bf16 [B*H*W][C] = [Xp > 0] * conv^T(dY * [Y > 0]); Wt bf16 [C][KH][KW][N]
// form: kDgradAuto picks by batch; the others force one kernel of the small-batch family (tests)
enum DgradForm : int { kDgradAuto = -1, kDgradPlain = 0, kDgradPrefetch = 1, kDgradSplit = 2 };
hipError_t conv_dgrad(const void* dY, const void* Y, const void* Wt, const void* Xp, void* dZp, const ConvGeo& g,
                      int relu_out, int relu_in, hipStream_t s, int form = kDgradAuto);

// ---- comm.hip: one-shot all-reduce over IPC-mapped peer staging regions (small DP buckets)
constexpr int kOneShotMaxRanks = 8;
constexpr int kOneShotMaxBlocks = 64;
struct OneShotArgs {
  char* base[kOneShotMaxRanks];  // every rank's region as mapped in this process (base[rank] local)
  const void* in;                // 16-B aligned, float (f64 == 0) or double elements
  void* out;                     // 16-B aligned, may alias in
  int n, rank, world;            // n: elements
  int f64;                       // elements are double (normaliser sums) instead of float
  double scale;                  // applied to this rank's contribution before the sum
  size_t stage_bytes;
  long long timeout_ticks;       // wall-clock ticks before a block gives up (NaN output + error word)
};
size_t oneshot_region_bytes(size_t stage_bytes);
size_t oneshot_handle_bytes();
int oneshot_blocks(int n, size_t stage_bytes, int elem_bytes = 4);
hipError_t oneshot_alloc(size_t stage_bytes, void** ptr, void* handle);  // zeroed uncached region + IPC handle
hipError_t oneshot_open(const void* handle, void** ptr);
hipError_t oneshot_close(void* ptr);
hipError_t oneshot_free(void* ptr);
hipError_t oneshot_read_error(void* local, int* err);
// stream-ordered copy of the error word into pinned host memory (no device-wide sync)
hipError_t oneshot_read_error_async(void* local, int* host_pinned, hipStream_t s);
hipError_t oneshot_clear_error(void* local);
long long oneshot_ticks_per_second();
hipError_t oneshot_allreduce(const OneShotArgs& a, hipStream_t s);

}  // namespace ia

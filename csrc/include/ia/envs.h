// Batched environment dynamics shared by the host (C++ vec-env runtime,
// csrc/runtime/vec_env.cpp) and the device (fused rollout kernel,
// csrc/kernels/rollout.hip).  One env instance = one row of SoA state.
//
// The reference gets these environments from gymnasium / seals / MuJoCo / ALE
// (setup.py:198-213; created in src/imitation/util/util.py:80-166).  None of
// those exist on this machine, so:
//   * classic control (CartPole, Pendulum, MountainCar, Acrobot) follows the
//     published gymnasium equations exactly (same constants, same integrator);
//   * seals fixed-horizon CartPole keeps the pole dynamics but never terminates;
//   * MuJoCo tasks (HalfCheetah, Hopper, Walker2d, Swimmer, Ant) are replaced by a
//     *synthetic planar locomotion model* with the identical observation/action
//     spaces and horizon (obs 17/11/17/8/27, act 6/3/6/2/8, horizon 1000). It is a
//     stiff articulated chain whose feet generate thrust only while in stance, so a
//     coordinated gait is required to move forward. Returns are NOT comparable to
//     MuJoCo numbers; shapes and costs of the learning pipeline are.
//   * Pong is a synthetic Atari-shaped game (84x84x4 uint8 frames, Discrete(6)).
#pragma once
#include <math.h>
#include <stdint.h>

#include "ia/rng.h"

// Transcendentals of the env models: full-precision libm on the host runtime, the
// hardware fast paths (v_exp_f32 / v_sin_f32 based) inside the device rollout,
// where the serial per-env chain is the latency bottleneck. Results agree to
// ~1e-6 relative per call; tests compare host vs device trajectories with a tolerance.
#if defined(__HIP_DEVICE_COMPILE__)
#define IA_EXPF(x) __expf(x)
#define IA_SINF(x) __sinf(x)
#define IA_COSF(x) __cosf(x)
#define IA_RCPF(x) __builtin_amdgcn_rcpf(x)  // v_rcp_f32 (1 ulp), not the div_scale/fixup sequence
#else
#define IA_RCPF(x) (1.0f / (x))
#define IA_EXPF(x) expf(x)
#define IA_SINF(x) sinf(x)
#define IA_COSF(x) cosf(x)
#endif

namespace ia {

enum EnvKind : int {
  ENV_CARTPOLE = 0,      // gymnasium CartPole (v0: 200 steps, v1: 500 steps)
  ENV_SEALS_CARTPOLE = 1,  // seals/CartPole-v0: fixed horizon 500, no termination
  ENV_PENDULUM = 2,
  ENV_MOUNTAINCAR = 3,
  ENV_ACROBOT = 4,
  ENV_LOCO = 5,          // synthetic MuJoCo-shaped locomotion
  ENV_PONG = 6,          // synthetic Atari-shaped pong
};

constexpr int kMaxJoints = 8;
constexpr int kMaxState = 40;  // floats of physical state per env
constexpr int kPongH = 84, kPongW = 84, kPongStack = 4;

struct LocoParams {
  int nq_root;     // root position coordinates (x first)
  int nv_root;     // root velocity coordinates (vx first)
  int nj;          // actuated joints
  int obs_skip;    // leading qpos entries excluded from the observation
  int frame_skip;
  float dt;
  float ctrl_cost;
  float fwd_weight;
  float healthy_reward;
  float drag;
  float gear[kMaxJoints];
  float stiff[kMaxJoints];
  float damp[kMaxJoints];
  float thrust[kMaxJoints];
  float pitch_coupling[kMaxJoints];
};

struct EnvParams {
  int kind;
  int obs_dim;
  int act_dim;       // continuous action dim, or 1 for discrete
  int n_actions;     // discrete cardinality (0 = continuous)
  int terminates;    // 1 if the env has a termination condition
  LocoParams loco;
};

// ----------------------------------------------------------------------------- CartPole
// gymnasium/envs/classic_control/cartpole.py (Euler integrator, tau=0.02).
IA_HD void cartpole_reset(float* s, uint64_t& rng) {
  for (int i = 0; i < 4; ++i) s[i] = uniform(rng, -0.05f, 0.05f);
}
IA_HD void cartpole_obs(const float* s, float* o) {
  for (int i = 0; i < 4; ++i) o[i] = s[i];
}
// returns reward; sets *term
IA_HD float cartpole_step(float* s, int action, int* term, bool seals) {
  const float gravity = 9.8f, masscart = 1.0f, masspole = 0.1f;
  const float total_mass = masspole + masscart, length = 0.5f;
  const float polemass_length = masspole * length, force_mag = 10.0f, tau = 0.02f;
  const float theta_threshold = 12.0f * 2.0f * 3.14159265358979f / 360.0f, x_threshold = 2.4f;
  float x = s[0], x_dot = s[1], theta = s[2], theta_dot = s[3];
  float force = action == 1 ? force_mag : -force_mag;
  float costheta = cosf(theta), sintheta = sinf(theta);
  float temp = (force + polemass_length * theta_dot * theta_dot * sintheta) / total_mass;
  float thetaacc = (gravity * sintheta - costheta * temp) /
                   (length * (4.0f / 3.0f - masspole * costheta * costheta / total_mass));
  float xacc = temp - polemass_length * thetaacc * costheta / total_mass;
  x = x + tau * x_dot;
  x_dot = x_dot + tau * xacc;
  theta = theta + tau * theta_dot;
  theta_dot = theta_dot + tau * thetaacc;
  s[0] = x; s[1] = x_dot; s[2] = theta; s[3] = theta_dot;
  bool failed = x < -x_threshold || x > x_threshold || theta < -theta_threshold || theta > theta_threshold;
  if (seals) {  // seals FixedHorizonCartPole: reward 1 while upright, never terminates
    *term = 0;
    return failed ? 0.0f : 1.0f;
  }
  *term = failed ? 1 : 0;
  return 1.0f;
}

// ----------------------------------------------------------------------------- Pendulum
IA_HD float angle_normalize(float x) {
  const float pi = 3.14159265358979f;
  float y = fmodf(x + pi, 2.0f * pi);
  if (y < 0) y += 2.0f * pi;
  return y - pi;
}
IA_HD void pendulum_reset(float* s, uint64_t& rng) {
  s[0] = uniform(rng, -3.14159265358979f, 3.14159265358979f);
  s[1] = uniform(rng, -1.0f, 1.0f);
}
IA_HD void pendulum_obs(const float* s, float* o) {
  o[0] = cosf(s[0]); o[1] = sinf(s[0]); o[2] = s[1];
}
IA_HD float pendulum_step(float* s, float u) {
  const float max_speed = 8.f, max_torque = 2.f, dt = .05f, g = 10.f, m = 1.f, l = 1.f;
  u = fminf(fmaxf(u, -max_torque), max_torque);
  float th = s[0], thdot = s[1];
  float an = angle_normalize(th);
  float cost = an * an + .1f * thdot * thdot + .001f * (u * u);
  float newthdot = thdot + (3.f * g / (2.f * l) * sinf(th) + 3.f / (m * l * l) * u) * dt;
  newthdot = fminf(fmaxf(newthdot, -max_speed), max_speed);
  s[0] = th + newthdot * dt;
  s[1] = newthdot;
  return -cost;
}

// ----------------------------------------------------------------------------- MountainCar
IA_HD void mountaincar_reset(float* s, uint64_t& rng) {
  s[0] = uniform(rng, -0.6f, -0.4f);
  s[1] = 0.f;
}
IA_HD float mountaincar_step(float* s, int action, int* term) {
  const float min_pos = -1.2f, max_pos = 0.6f, max_speed = 0.07f, goal = 0.5f;
  const float force = 0.001f, gravity = 0.0025f;
  float p = s[0], v = s[1];
  v += (action - 1) * force + cosf(3.f * p) * (-gravity);
  v = fminf(fmaxf(v, -max_speed), max_speed);
  p += v;
  p = fminf(fmaxf(p, min_pos), max_pos);
  if (p == min_pos && v < 0) v = 0;
  s[0] = p; s[1] = v;
  *term = (p >= goal && v >= 0.f) ? 1 : 0;
  return -1.0f;
}

// ----------------------------------------------------------------------------- Acrobot
// gymnasium acrobot.py "book" dynamics, RK4 with dt=0.2.
IA_HD void acrobot_dsdt(const float* s, float a, float* d) {
  const float m1 = 1.f, m2 = 1.f, l1 = 1.f, lc1 = .5f, lc2 = .5f, I1 = 1.f, I2 = 1.f, g = 9.8f;
  const float pi = 3.14159265358979f;
  float theta1 = s[0], theta2 = s[1], dtheta1 = s[2], dtheta2 = s[3];
  float d1 = m1 * lc1 * lc1 + m2 * (l1 * l1 + lc2 * lc2 + 2 * l1 * lc2 * cosf(theta2)) + I1 + I2;
  float d2 = m2 * (lc2 * lc2 + l1 * lc2 * cosf(theta2)) + I2;
  float phi2 = m2 * lc2 * g * cosf(theta1 + theta2 - pi / 2.f);
  float phi1 = -m2 * l1 * lc2 * dtheta2 * dtheta2 * sinf(theta2) - 2 * m2 * l1 * lc2 * dtheta2 * dtheta1 * sinf(theta2) +
               (m1 * lc1 + m2 * l1) * g * cosf(theta1 - pi / 2) + phi2;
  float ddtheta2 = (a + d2 / d1 * phi1 - m2 * l1 * lc2 * dtheta1 * dtheta1 * sinf(theta2) - phi2) /
                   (m2 * lc2 * lc2 + I2 - d2 * d2 / d1);
  float ddtheta1 = -(d2 * ddtheta2 + phi1) / d1;
  d[0] = dtheta1; d[1] = dtheta2; d[2] = ddtheta1; d[3] = ddtheta2;
}
IA_HD void acrobot_reset(float* s, uint64_t& rng) {
  for (int i = 0; i < 4; ++i) s[i] = uniform(rng, -0.1f, 0.1f);
}
IA_HD void acrobot_obs(const float* s, float* o) {
  o[0] = cosf(s[0]); o[1] = sinf(s[0]); o[2] = cosf(s[1]); o[3] = sinf(s[1]); o[4] = s[2]; o[5] = s[3];
}
IA_HD float wrapf(float x, float m, float M) {
  float diff = M - m;
  while (x > M) x -= diff;
  while (x < m) x += diff;
  return x;
}
IA_HD float acrobot_step(float* s, int action, int* term) {
  const float pi = 3.14159265358979f, dt = 0.2f;
  float torque = (float)(action - 1);
  float k1[4], k2[4], k3[4], k4[4], tmp[4];
  acrobot_dsdt(s, torque, k1);
  for (int i = 0; i < 4; ++i) tmp[i] = s[i] + dt / 2 * k1[i];
  acrobot_dsdt(tmp, torque, k2);
  for (int i = 0; i < 4; ++i) tmp[i] = s[i] + dt / 2 * k2[i];
  acrobot_dsdt(tmp, torque, k3);
  for (int i = 0; i < 4; ++i) tmp[i] = s[i] + dt * k3[i];
  acrobot_dsdt(tmp, torque, k4);
  for (int i = 0; i < 4; ++i) s[i] = s[i] + dt / 6.f * (k1[i] + 2 * k2[i] + 2 * k3[i] + k4[i]);
  s[0] = wrapf(s[0], -pi, pi);
  s[1] = wrapf(s[1], -pi, pi);
  s[2] = fminf(fmaxf(s[2], -4 * pi), 4 * pi);
  s[3] = fminf(fmaxf(s[3], -9 * pi), 9 * pi);
  bool done = -cosf(s[0]) - cosf(s[1] + s[0]) > 1.f;
  *term = done ? 1 : 0;
  return done ? 0.f : -1.f;
}

// ----------------------------------------------------------------------------- Locomotion
// State layout: qpos[0 .. nq) followed by qvel[0 .. nv).  qpos = root (x, z,
// pitch, ...) then joints; qvel = root velocities (vx, vz, vpitch, ...) then joints.
IA_HD int loco_nq(const LocoParams& p) { return p.nq_root + p.nj; }
IA_HD int loco_nv(const LocoParams& p) { return p.nv_root + p.nj; }

IA_HD void loco_reset(const LocoParams& p, float* s, uint64_t& rng) {
  const int nq = loco_nq(p), nv = loco_nv(p);
  for (int i = 0; i < nq; ++i) s[i] = uniform(rng, -0.1f, 0.1f);
  s[0] = 0.f;                      // x starts at the origin
  if (p.nq_root > 1) s[1] += 0.0f;  // height offset handled as deviation from nominal
  for (int i = 0; i < nv; ++i) s[nq + i] = 0.1f * normal01(rng);
}

IA_HD void loco_obs(const LocoParams& p, const float* s, float* o) {
  const int nq = loco_nq(p), nv = loco_nv(p);
  int k = 0;
  for (int i = p.obs_skip; i < nq; ++i) o[k++] = s[i];
  for (int i = 0; i < nv; ++i) o[k++] = s[nq + i];
}

IA_HD float stance(float q) {  // smooth contact indicator: foot on ground when q < 0
  return IA_RCPF(1.0f + IA_EXPF(8.0f * q));
}

IA_HD float loco_step(const LocoParams& p, float* s, const float* a_in) {
  const int nq = loco_nq(p);
  float* qpos = s;
  float* qvel = s + nq;
  float a[kMaxJoints];
  float ctrl = 0.f;
  for (int j = 0; j < p.nj; ++j) {
    a[j] = fminf(fmaxf(a_in[j], -1.f), 1.f);
    ctrl += a[j] * a[j];
  }
  const float x_before = qpos[0];
  const int jq = p.nq_root, jv = p.nv_root;
  for (int sub = 0; sub < p.frame_skip; ++sub) {
    float thrust = 0.f, lift = 0.f, pitch_torque = 0.f;
    for (int j = 0; j < p.nj; ++j) {
      float q = qpos[jq + j], qd = qvel[jv + j];
      // actuated, damped, spring-loaded hinge with a gravity-like nonlinearity
      float qdd = p.gear[j] * a[j] - p.stiff[j] * q - p.damp[j] * qd - 2.0f * IA_SINF(q);
      qvel[jv + j] = qd + p.dt * qdd;
      float st = stance(q);
      // a stance foot sweeping backwards (qd < 0) pushes the body forward
      thrust += p.thrust[j] * st * fmaxf(-qd, 0.f);
      lift += st;
      pitch_torque += p.pitch_coupling[j] * a[j];
    }
    float vx = qvel[0];
    float vx_dd = thrust - p.drag * vx * (1.0f + fabsf(vx));
    qvel[0] = vx + p.dt * vx_dd;
    if (p.nv_root > 1) {  // height: spring towards nominal, lifted by stance legs
      float z = qpos[1], vz = qvel[1];
      float vz_dd = -20.f * z - 4.f * vz + 0.5f * (lift / (float)p.nj - 0.5f);
      qvel[1] = vz + p.dt * vz_dd;
    }
    if (p.nv_root > 2) {  // pitch: torsional spring driven by joint torques
      float th = qpos[2], vth = qvel[2];
      float th_dd = -15.f * IA_SINF(th) - 3.f * vth + pitch_torque;
      qvel[2] = vth + p.dt * th_dd;
    }
    for (int i = 3; i < p.nv_root; ++i) {  // extra root dofs: damped, weakly driven
      qvel[i] = qvel[i] * (1.f - 2.f * p.dt) + p.dt * 0.1f * pitch_torque;
    }
    // semi-implicit Euler on positions; root quaternion-ish extras share velocities cyclically
    qpos[0] += p.dt * qvel[0];
    for (int i = 1; i < p.nq_root; ++i) qpos[i] += p.dt * qvel[i < p.nv_root ? i : (i % p.nv_root)] * (i < p.nv_root ? 1.f : 0.1f);
    for (int j = 0; j < p.nj; ++j) {
      float q = qpos[jq + j] + p.dt * qvel[jv + j];
      // joint range [-1.2, 1.2] rad with inelastic limit
      if (q > 1.2f) { q = 1.2f; if (qvel[jv + j] > 0) qvel[jv + j] = 0.f; }
      if (q < -1.2f) { q = -1.2f; if (qvel[jv + j] < 0) qvel[jv + j] = 0.f; }
      qpos[jq + j] = q;
    }
  }
  const float dt_total = p.dt * p.frame_skip;
  const float x_vel = (qpos[0] - x_before) / dt_total;
  return p.fwd_weight * x_vel + p.healthy_reward - p.ctrl_cost * ctrl;
}

// ----------------------------------------------------------------------------- Pong
// State: ball x,y,vx,vy; agent paddle y; opponent paddle y; scores; frame counter.
// Rendering writes an 84x84 grayscale frame; the observation is the last 4
// frames stacked on the channel axis (HWC, like SB3 VecFrameStack on Atari).
enum { PG_BX = 0, PG_BY, PG_VX, PG_VY, PG_PA, PG_PO, PG_SA, PG_SO, PG_N };

IA_HD void pong_serve(float* s, uint64_t& rng, float dir) {
  s[PG_BX] = 42.f; s[PG_BY] = uniform(rng, 30.f, 54.f);
  s[PG_VX] = dir * 1.5f; s[PG_VY] = uniform(rng, -1.2f, 1.2f);
}
IA_HD void pong_reset(float* s, uint64_t& rng) {
  pong_serve(s, rng, uniform01(rng) < 0.5f ? -1.f : 1.f);
  s[PG_PA] = 42.f; s[PG_PO] = 42.f; s[PG_SA] = 0.f; s[PG_SO] = 0.f;
}
IA_HD float pong_step(float* s, int action, int* term, uint64_t& rng) {
  // ALE Pong minimal action set: NOOP, FIRE, RIGHT(up), LEFT(down), RIGHTFIRE, LEFTFIRE
  float move = 0.f;
  if (action == 2 || action == 4) move = -2.5f;
  if (action == 3 || action == 5) move = 2.5f;
  float reward = 0.f;
  for (int f = 0; f < 4; ++f) {  // frameskip 4
    s[PG_PA] = fminf(fmaxf(s[PG_PA] + move, 8.f), 76.f);
    float target = s[PG_BY];
    float dpo = fminf(fmaxf(target - s[PG_PO], -1.6f), 1.6f);
    s[PG_PO] = fminf(fmaxf(s[PG_PO] + dpo, 8.f), 76.f);
    s[PG_BX] += s[PG_VX]; s[PG_BY] += s[PG_VY];
    if (s[PG_BY] < 2.f) { s[PG_BY] = 2.f; s[PG_VY] = -s[PG_VY]; }
    if (s[PG_BY] > 82.f) { s[PG_BY] = 82.f; s[PG_VY] = -s[PG_VY]; }
    // agent paddle at x = 76, opponent at x = 8
    if (s[PG_BX] >= 75.f && s[PG_VX] > 0) {
      if (fabsf(s[PG_BY] - s[PG_PA]) <= 7.f) {
        s[PG_VX] = -s[PG_VX] * 1.03f; s[PG_VY] += 0.15f * (s[PG_BY] - s[PG_PA]);
      } else if (s[PG_BX] > 83.f) {
        s[PG_SO] += 1.f; reward -= 1.f; pong_serve(s, rng, 1.f);
      }
    }
    if (s[PG_BX] <= 9.f && s[PG_VX] < 0) {
      if (fabsf(s[PG_BY] - s[PG_PO]) <= 7.f) {
        s[PG_VX] = -s[PG_VX] * 1.03f; s[PG_VY] += 0.15f * (s[PG_BY] - s[PG_PO]);
      } else if (s[PG_BX] < 1.f) {
        s[PG_SA] += 1.f; reward += 1.f; pong_serve(s, rng, -1.f);
      }
    }
    s[PG_VX] = fminf(fmaxf(s[PG_VX], -4.f), 4.f);
    s[PG_VY] = fminf(fmaxf(s[PG_VY], -3.f), 3.f);
  }
  *term = (s[PG_SA] >= 21.f || s[PG_SO] >= 21.f) ? 1 : 0;
  return reward;
}
// Pixel (r, c) of the current frame.
IA_HD uint8_t pong_pixel(const float* s, int r, int c) {
  if (r < 1 || r > 82) return 236;  // walls
  float fr = (float)r, fc = (float)c;
  if (fabsf(fc - s[PG_BX]) <= 1.f && fabsf(fr - s[PG_BY]) <= 1.f) return 236;
  if (c >= 75 && c <= 76 && fabsf(fr - s[PG_PA]) <= 7.f) return 147;
  if (c >= 7 && c <= 8 && fabsf(fr - s[PG_PO]) <= 7.f) return 108;
  return 87;
}

// ----------------------------------------------------------------------------- dispatch
IA_HD int state_size(const EnvParams& P) {
  switch (P.kind) {
    case ENV_CARTPOLE: case ENV_SEALS_CARTPOLE: case ENV_ACROBOT: return 4;
    case ENV_PENDULUM: case ENV_MOUNTAINCAR: return 2;
    case ENV_LOCO: return loco_nq(P.loco) + loco_nv(P.loco);
    case ENV_PONG: return PG_N;
  }
  return 0;
}

IA_HD void env_reset(const EnvParams& P, float* s, uint64_t& rng) {
  switch (P.kind) {
    case ENV_CARTPOLE: case ENV_SEALS_CARTPOLE: cartpole_reset(s, rng); break;
    case ENV_PENDULUM: pendulum_reset(s, rng); break;
    case ENV_MOUNTAINCAR: mountaincar_reset(s, rng); break;
    case ENV_ACROBOT: acrobot_reset(s, rng); break;
    case ENV_LOCO: loco_reset(P.loco, s, rng); break;
    case ENV_PONG: pong_reset(s, rng); break;
  }
}

// Vector observation (all kinds except Pong, whose frames are rendered separately).
IA_HD void env_obs(const EnvParams& P, const float* s, float* o) {
  switch (P.kind) {
    case ENV_CARTPOLE: case ENV_SEALS_CARTPOLE: cartpole_obs(s, o); break;
    case ENV_PENDULUM: pendulum_obs(s, o); break;
    case ENV_MOUNTAINCAR: o[0] = s[0]; o[1] = s[1]; break;
    case ENV_ACROBOT: acrobot_obs(s, o); break;
    case ENV_LOCO: loco_obs(P.loco, s, o); break;
    default: break;
  }
}

// action: pointer to act_dim floats (discrete actions are passed as a float index)
IA_HD float env_step(const EnvParams& P, float* s, const float* action, int* term, uint64_t& rng) {
  *term = 0;
  switch (P.kind) {
    case ENV_CARTPOLE: return cartpole_step(s, (int)action[0], term, false);
    case ENV_SEALS_CARTPOLE: return cartpole_step(s, (int)action[0], term, true);
    case ENV_PENDULUM: return pendulum_step(s, action[0]);
    case ENV_MOUNTAINCAR: return mountaincar_step(s, (int)action[0], term);
    case ENV_ACROBOT: return acrobot_step(s, (int)action[0], term);
    case ENV_LOCO: return loco_step(P.loco, s, action);
    case ENV_PONG: return pong_step(s, (int)action[0], term, rng);
  }
  return 0.f;
}

}  // namespace ia

"""Device-resident adversarial imitation (GAIL / AIRL-ready) -- the MI355X fast path.

Same algorithm, hyper-parameters and public surface as
:class:`imitation_amd.algorithms.adversarial.gail.GAIL` (reference
``src/imitation/algorithms/adversarial/{common,gail}.py``), but a training round
never leaves the GPU:

=====================  ==========================================================
reference (host loop)  this engine
=====================  ==========================================================
SB3 collect_rollouts:  ``engine_rollout`` -- ONE kernel runs n_steps x n_envs of
policy fwd, VecEnv     policy sampling, env physics (native model) and the
pipes, reward wrapper  TimeLimit bootstrap; buffers are written straight into
numpy<->device copies  HBM. The learned reward ``softplus(D(s,a))`` does not feed
                       back into the dynamics: ``engine_reward_batch`` computes it
                       for all T x N transitions in one parallel pass afterwards
RolloutBuffer GAE      ``gae`` kernel (one lane per env)
(python loop)
PPO.train              ``engine_ppo_update`` -- ONE persistent workgroup runs all
(~10 launches / mb)    epochs x minibatches (fp32 MFMA, params in LDS, Adam in L2)
BufferingWrapper +     device replay ring, same FIFO content as the reference's
ReplayBuffer (numpy)   flatten-then-store order
train_disc             fused MLP fwd/bwd kernels + device demo sampler
=====================  ==========================================================

Data parallel: each rank runs its own envs; the PPO update switches to the
per-minibatch kernel pair with an RCCL all-reduce of the normaliser moments and
of the flat gradient between them (synchronous DP == large-batch SGD), and the
discriminator averages its gradient bucket once per update.

Eligibility (checked in :func:`supports`): native vector env (non-image), an
on-policy :class:`~imitation_amd.rl.ppo.PPO` with an MLP actor-critic (widths ≤ 64,
≤ 4 layers, minibatch ≤ 128 and a multiple of 16), and an MLP
``BasicRewardNet`` (optionally inside ``NormalizedRewardNet``). Anything else
should use the host-loop trainers.
"""

from __future__ import annotations

import contextlib

import os
import time
from typing import Any, Dict, List, Mapping, Optional, Sequence, Tuple

import numpy as np
import torch as th
from torch import nn

from imitation_amd.utils.streams import shared_stream
from imitation_amd import ops
from imitation_amd.algorithms.adversarial import common
from imitation_amd.algorithms.adversarial.gail import GAIL
from imitation_amd.data import buffer as buffer_mod
from imitation_amd.data import types
from imitation_amd.envs import spaces
from imitation_amd.envs.vec_env import NativeVecEnv, VecEnvWrapper
from imitation_amd.ops import rl as rl_ops
from imitation_amd.ops.mlp import act_code
from imitation_amd.parallel import dist as pdist
from imitation_amd.rewards import reward_nets
from imitation_amd.rl.policies import ActorCriticPolicy
from imitation_amd.rl.ppo import PPO
from imitation_amd.util import networks
from imitation_amd.utils import gcfreeze, profiling


def _unwrap_native(venv) -> Optional[NativeVecEnv]:
    e = venv
    while e is not None:
        if isinstance(e, NativeVecEnv):
            return e
        e = getattr(e, "venv", None)
    return None


def _mlp_layers(seq: nn.Sequential) -> Tuple[Optional[networks.BaseNorm], List[nn.Linear], int, int]:
    """(input norm, linears, hidden act code, out act code) of a build_mlp / trunk Sequential."""
    norm = None
    lins: List[nn.Linear] = []
    acts: List[int] = []
    for m in seq:
        if isinstance(m, networks.BaseNorm):
            norm = m
        elif isinstance(m, nn.Linear):
            lins.append(m)
            acts.append(0)
        elif isinstance(m, (nn.Flatten, networks.SqueezeLayer, nn.Dropout)):
            continue
        else:
            c = act_code(m)
            if c is None:
                raise ValueError(f"engine cannot fuse activation {m}")
            acts[-1] = c
    hidden = acts[0] if len(acts) > 1 else 0
    return norm, lins, hidden, acts[-1] if acts else 0


def _policy_nets(policy: ActorCriticPolicy):
    fe = policy.features_extractor
    norm = getattr(fe, "normalize", None)
    pi_trunk = list(policy.mlp_extractor.policy_net)
    vf_trunk = list(policy.mlp_extractor.value_net)

    def trunk(mods):
        lins, act = [], 0
        for m in mods:
            if isinstance(m, nn.Linear):
                lins.append(m)
            else:
                c = act_code(m)
                if c is None:
                    raise ValueError(f"engine cannot fuse activation {m}")
                act = c
        return lins, act

    pl, pa = trunk(pi_trunk)
    vl, va = trunk(vf_trunk)
    if pl and vl and pa != va:
        raise ValueError("actor and critic trunks must share the activation")
    return norm, pl + [policy.action_net], vl + [policy.value_net], pa or va


def supports(venv, gen_algo, reward_net) -> Tuple[bool, str]:
    """Whether :class:`DeviceGAIL` can run this configuration (reason when not)."""
    ok, why = supports_generator(venv, gen_algo)
    if not ok:
        return ok, why
    base = reward_net.base if isinstance(reward_net, reward_nets.NormalizedRewardNet) else reward_net
    if not isinstance(base, reward_nets.BasicRewardNet):
        return False, "reward net is not a BasicRewardNet"
    return True, ""


def supports_generator(venv, gen_algo) -> Tuple[bool, str]:
    """Env + PPO generator eligibility shared by the device GAIL / AIRL engines."""
    if not th.cuda.is_available():
        return False, "no GPU"
    nat = _unwrap_native(venv)
    if nat is None:
        return False, "env is not a native vector env"
    if nat._is_image:
        return False, "image observations"
    if not isinstance(gen_algo, PPO):
        return False, "generator is not PPO"
    pol = gen_algo.policy
    if type(pol).__name__.startswith("Homogenous") or not isinstance(pol, ActorCriticPolicy):
        return False, "policy is not a plain ActorCriticPolicy"
    if not pol.share_features_extractor:
        return False, "separate features extractors"
    try:
        norm, pl, vl, act = _policy_nets(pol)
    except ValueError as e:
        return False, str(e)
    dims = [pol.features_dim] + [l.out_features for l in pl]
    if max(dims) > 64 or len(pl) > 4 or len(vl) > 4:
        return False, "policy too wide / deep for the engine"
    if gen_algo.batch_size % 16 != 0:
        return False, "minibatch must be a multiple of 16"
    if (gen_algo.n_steps * gen_algo.n_envs) % gen_algo.batch_size != 0:
        return False, "rollout size not a multiple of the minibatch"
    if gen_algo.batch_size > 64 and not ppo_path(pol, nat, gen_algo.batch_size,
                                                 gen_algo.n_steps * gen_algo.n_envs).startswith("rc"):
        return False, "minibatch > 64 needs the register-chained PPO kernel, which rejects this policy"
    if gen_algo.clip_range_vf is not None or gen_algo.target_kl is not None:
        return False, "clip_range_vf / target_kl not supported by the engine"
    return True, ""


def ppo_path(pol: ActorCriticPolicy, nat, batch: int, rows: int, rc_gmax: int = 0) -> str:
    """Which PPO kernel the engine would run (``"rc:g<G>x<nch>x<cw>:kt<KT>"`` or ``"lds"``)."""
    norm, pl, vl, act = _policy_nets(pol)
    discrete = isinstance(nat.action_space, spaces.Discrete)
    D = int(np.prod(nat.observation_space.shape))
    A = int(nat.action_space.n) if discrete else int(np.prod(nat.action_space.shape))
    d = dict(D=D, A=A, discrete=int(discrete), pi_dims=[D] + [l.out_features for l in pl],
             vf_dims=[D] + [l.out_features for l in vl], batch=int(batch), rows=int(rows),
             log_std_off=0 if (hasattr(pol, "log_std") and not discrete) else -1, rc_gmax=int(rc_gmax),
             hidden_act=int(act))
    return ops.native().engine_ppo_path(d)


class _FlatParams:
    """Re-point a list of parameters at views of one flat fp32 device buffer."""

    def __init__(self, params: Sequence[nn.Parameter]):
        self.params = list(params)
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        self.flat = th.zeros(n, device=dev, dtype=th.float32)
        self.offsets = []
        off = 0
        for p in self.params:
            self.flat[off : off + p.numel()].copy_(p.detach().reshape(-1))
            self.offsets.append(off)
            p.data = self.flat[off : off + p.numel()].view_as(p)
            off += p.numel()
        self.n = n

    def offset(self, p: nn.Parameter) -> int:
        for q, o in zip(self.params, self.offsets):
            if q is p:
                return o
        raise KeyError("parameter not in flat buffer")


class DeviceGeneratorCore:
    """Device PPO generator: env state, flat policy parameters, the fused rollout kernel
    (policy + env + learned reward), GAE and the PPO update kernels, data-parallel plan.
    Shared by the adversarial engines (:class:`DeviceEngineMixin`) and the preference-
    comparison agent (:class:`imitation_amd.engine.preference.DeviceAgentTrainer`).
    Subclasses set ``gen_algo``, ``_reward_net`` and ``debug_use_ground_truth`` and call
    :meth:`_init_generator`."""

    # ------------------------------------------------------------------ stream ordering
    def _dev_event(self, stream: Optional[th.cuda.Stream] = None):
        """An event recorded on ``stream`` (default: the current one) for GPU -> GPU ordering
        and host waits on completion: device-scope release (``_C.DeviceEvent``,
        csrc/bind/events.cpp), so the markers between the round's critical kernels do not write
        back the L2s. Pinned D2H copies the host reads keep torch (system-scope) events.
        IMITATION_AMD_DEVICE_EVENTS=0: torch events everywhere."""
        if os.environ.get("IMITATION_AMD_DEVICE_EVENTS", "1") != "0" and hasattr(self._C, "DeviceEvent"):
            ev = self._C.DeviceEvent(True)
            ev.record(stream.cuda_stream if stream is not None else None)
            return ev
        ev = th.cuda.Event()
        ev.record(stream)
        return ev

    @staticmethod
    def _wait_ev(stream: th.cuda.Stream, ev) -> None:
        """``stream`` waits for ``ev`` (a torch event or a ``_dev_event``)."""
        if isinstance(ev, th.cuda.Event):
            stream.wait_event(ev)
        else:
            ev.wait(stream.cuda_stream)

    def _init_generator(self, venv) -> None:
        self._native = _unwrap_native(venv)
        self._C = ops.native()
        self._dev = self.gen_algo.device
        self._setup_engine()
        self._setup_dp()

    # ------------------------------------------------------------------ setup
    def _setup_engine(self) -> None:
        dev = self._dev
        algo: PPO = self.gen_algo
        pol: ActorCriticPolicy = algo.policy
        nat = self._native
        self.N = nat.num_envs
        self.T = algo.n_steps
        self.D = int(np.prod(nat.observation_space.shape))
        self.discrete = isinstance(nat.action_space, spaces.Discrete)
        self.A = int(nat.action_space.n) if self.discrete else int(np.prod(nat.action_space.shape))
        # env state -> device
        obs0 = nat.reset()
        st = nat.get_state()
        self.state = th.as_tensor(st["state"], device=dev).float().contiguous()
        self.env_rng = th.as_tensor(st["rng"].astype(np.int64), device=dev).contiguous()
        self.elapsed = th.as_tensor(st["elapsed"].astype(np.int32), device=dev).contiguous()
        self.ep_ret = th.zeros(self.N, device=dev)
        self.cur_obs = th.as_tensor(np.asarray(obs0, np.float32), device=dev).reshape(self.N, self.D).contiguous()
        self.cur_start = th.ones(self.N, device=dev)
        self.max_steps = int(nat.max_episode_steps)
        # policy parameters -> one flat buffer (module params become views)
        norm, pl, vl, hid = _policy_nets(pol)
        self.pol_norm = norm
        self.pi_layers, self.vf_layers, self.hidden_act = pl, vl, hid
        plist: List[nn.Parameter] = []
        for l in pl + vl:
            plist += [l.weight, l.bias]
        self.has_log_std = hasattr(pol, "log_std") and not self.discrete
        if self.has_log_std:
            plist.append(pol.log_std)
        self.flat = _FlatParams(plist)
        self.grads = th.zeros_like(self.flat.flat)
        self.exp_avg = th.zeros_like(self.flat.flat)
        self.exp_avg_sq = th.zeros_like(self.flat.flat)
        self.adam_step = th.zeros(1, device=dev)
        if norm is not None:
            self.norm_count = norm.count.detach().float().reshape(1).clone()
        else:
            self.norm_count = None
        if self.discrete:
            self.act_low = self.act_high = None
        else:
            self.act_low = th.as_tensor(nat.action_space.low.reshape(-1), device=dev).float()
            self.act_high = th.as_tensor(nat.action_space.high.reshape(-1), device=dev).float()
        # rollout buffers [T, N, ...]
        T, N, D = self.T, self.N, self.D
        Aw = 1 if self.discrete else self.A
        z = lambda *s: th.zeros(*s, device=dev)
        self.buf = dict(obs_buf=z(T, N, D), act_raw=z(T, N, Aw), act_env=z(T, N, Aw), logp=z(T, N), values=z(T, N),
                        rewards=z(T, N), env_rew=z(T, N), starts=z(T, N), dones=z(T, N), trunc=z(T, N), boot=z(T, N),
                        next_obs=z(T, N, D), ep_ret_out=z(T, N), last_values=z(N))
        self._boot = self.buf["boot"]
        # PPO statistics sums (kernel output) followed by the GAE pass's [N][4] return /
        # advantage moments (train/explained_variance): ONE device buffer, one D2H copy per round
        self._log_dev = z(5 + 4 * N)
        self.stats = self._log_dev[:5]
        self._ev_mom = self._log_dev[5:].view(N, 4)
        self._seed = int(np.random.randint(0, 2**62)) ^ (pdist.rank() * 0x9E3779B97F4A7C15 & ((1 << 62) - 1))
        self._step0 = 0
        self._perm_round = 0
        from imitation_amd.utils.errflag import DeviceErrorFlag

        self._ppo_err = DeviceErrorFlag(self._dev, "PPO update kernel")
        self._ppo_static = self._ppo_args_static()
        self._ep_lens_running = np.zeros(self.N, dtype=np.int64)

    def _wave_mlp(self, lins: Sequence[nn.Linear], hidden_act: int, out_act: int, norm=None) -> Dict[str, Any]:
        d: Dict[str, Any] = dict(W=[l.weight.detach() for l in lins], b=[l.bias.detach() for l in lins],
                                 hidden_act=int(hidden_act), out_act=int(out_act))
        if norm is not None:
            d.update(norm_mean=norm.running_mean.detach().float().contiguous(),
                     norm_var=norm.running_var.detach().float().contiguous(), norm_eps=float(norm.eps))
        return d

    def _reward_spec(self) -> Dict[str, Any]:
        base = self._reward_net.base if isinstance(self._reward_net, reward_nets.NormalizedRewardNet) else self._reward_net
        rnorm, rl, rh, ro = _mlp_layers(base.mlp)
        spec = dict(rew=self._wave_mlp(rl, rh, ro, rnorm), use_state=int(base.use_state), use_action=int(base.use_action),
                    use_next_state=int(base.use_next_state), use_done=int(base.use_done), rew_transform=1)
        return spec

    def _post_rollout_rewards(self) -> None:
        """Hook: rewrite ``buf["rewards"]`` after the rollout kernel (AIRL output normalisation)."""

    def _ppo_args_static(self) -> Dict[str, Any]:
        algo: PPO = self.gen_algo
        fp = self.flat
        pi_dims = [self.D] + [l.out_features for l in self.pi_layers]
        vf_dims = [self.D] + [l.out_features for l in self.vf_layers]
        d = dict(D=self.D, A=self.A, discrete=int(self.discrete), pi_dims=pi_dims, vf_dims=vf_dims,
                 pi_w_off=[fp.offset(l.weight) for l in self.pi_layers], pi_b_off=[fp.offset(l.bias) for l in self.pi_layers],
                 vf_w_off=[fp.offset(l.weight) for l in self.vf_layers], vf_b_off=[fp.offset(l.bias) for l in self.vf_layers],
                 log_std_off=fp.offset(self.gen_algo.policy.log_std) if self.has_log_std else -1,
                 hidden_act=int(self.hidden_act), params=fp.flat, grads=self.grads, exp_avg=self.exp_avg,
                 exp_avg_sq=self.exp_avg_sq, n_params=fp.n, has_norm=int(self.pol_norm is not None),
                 rows=self.T * self.N, batch=int(algo.batch_size), n_epochs=int(algo.n_epochs),
                 ent_coef=float(algo.ent_coef), vf_coef=float(algo.vf_coef), max_grad_norm=float(algo.max_grad_norm),
                 normalize_advantage=int(algo.normalize_advantage), adam_step=self.adam_step, stats=self.stats,
                 err=self._ppo_err.word,
                 # fail-fast knobs of the cooperating-workgroup kernel (tests force a timeout)
                 spin_limit=0, debug_stall=0)  # (tests set these two in _ppo_static)
        opt = algo.policy.optimizer
        g = opt.param_groups[0]
        d.update(beta1=float(g.get("betas", (0.9, 0.999))[0]), beta2=float(g.get("betas", (0.9, 0.999))[1]),
                 adam_eps=float(g.get("eps", 1e-8)))
        if self.pol_norm is not None:
            d.update(norm_mean=self.pol_norm.running_mean, norm_var=self.pol_norm.running_var, norm_count=self.norm_count,
                     norm_eps=float(self.pol_norm.eps))
        self._ppo_is_rc = self._C.engine_ppo_path(d).startswith("rc")
        if not self._ppo_is_rc:
            lds = self._C.engine_ppo_lds(d) if d["batch"] <= 64 else 1 << 30
            if lds > 150 * 1024:
                raise ValueError(f"PPO engine needs {lds} B of LDS (> 150 KiB)")
        return d

    # ------------------------------------------------------------------ one generator round
    _CHAIN_OUT = ("obs_buf", "act_raw", "act_env", "env_rew", "starts", "dones", "trunc", "next_obs", "ep_ret_out")

    @profiling.traced("rollout/chain")
    def _launch_chain(self, explore_mode: Optional[th.Tensor] = None) -> None:
        """The serial part of a rollout (rollout.hip): T steps of actor sampling + env
        physics per env, nothing else on the step chain."""
        algo: PPO = self.gen_algo
        pol = algo.policy
        args = dict(env=self._native.env_id, max_steps=self.max_steps, T=self.T, N=self.N, seed=int(self._seed),
                    step0=int(self._step0), state=self.state, rng=self.env_rng, elapsed=self.elapsed, ep_ret=self.ep_ret,
                    cur_obs=self.cur_obs, cur_start=self.cur_start,
                    pi=self._wave_mlp(self.pi_layers, self.hidden_act, 0, self.pol_norm),
                    log_std=pol.log_std.detach() if self.has_log_std else None, act_low=self.act_low,
                    act_high=self.act_high, n_actions=self.A if self.discrete else 0, explore_mode=explore_mode)
        args.update({k: self.buf[k] for k in self._CHAIN_OUT})
        self._C.engine_rollout(args)
        self._step0 += self.T

    @profiling.traced("rollout/reward_pass")
    def _launch_post(self, reward: bool) -> None:
        """The parallel part (engine.hip): V(s), log-probs, TimeLimit bootstrap and the learned
        reward of all T x N transitions, V of the final observations."""
        algo: PPO = self.gen_algo
        pol = algo.policy
        b = self.buf
        d = dict(T=self.T, N=self.N, D=self.D, A=1 if self.discrete else self.A, n_actions=self.A if self.discrete else 0,
                 gamma=float(algo.gamma), cur_obs=self.cur_obs,
                 pi=self._wave_mlp(self.pi_layers, self.hidden_act, 0, self.pol_norm),
                 vf=self._wave_mlp(self.vf_layers, self.hidden_act, 0, self.pol_norm),
                 log_std=pol.log_std.detach() if self.has_log_std else None, rew_enabled=int(reward))
        d.update({k: b[k] for k in ("obs_buf", "act_raw", "act_env", "next_obs", "dones", "trunc", "env_rew", "values",
                                    "logp", "boot", "rewards", "last_values")})
        if reward:
            d.update(self._reward_spec())
            d.update(self._rollout_extra_bufs())
        self._C.engine_rollout_post(d)

    def _rollout(self) -> None:
        """One training rollout: chain -> parallel pass (-> AIRL output normalisation). The
        learned reward does not feed back into the dynamics, so it leaves the step chain."""
        self._launch_chain()
        reward = not self.debug_use_ground_truth
        self._launch_post(reward)
        if reward:
            self._post_rollout_rewards()

    def _rollout_extra_bufs(self) -> Dict[str, Any]:
        return {}

    @profiling.traced("ppo/update")
    def _ppo_update(self) -> None:
        algo: PPO = self.gen_algo
        rows = self.T * self.N
        world = pdist.world_size()
        # single-rank fast path: the kernel reads / writes the module's int32 count itself and
        # its prep launch zeroes the stats (three small launches fewer between the rollout
        # and the update)
        direct = (world == 1 and getattr(self, "_ppo_is_rc", False)
                  and (self.pol_norm is None or self.pol_norm.count.dtype == th.int32))
        if self.pol_norm is not None and not direct:
            # the policy normaliser may also have been updated outside the engine (the
            # discriminator's log-prob pass runs the policy in training mode, as the
            # reference does): the kernel continues from the module's own count
            self.norm_count.copy_(self.pol_norm.count.reshape(1))
        algo._update_current_progress_remaining(algo.num_timesteps, algo._total_timesteps or algo.num_timesteps)
        lr = float(algo.lr_schedule(algo._current_progress_remaining))
        clip = float(algo.clip_range(algo._current_progress_remaining))
        adv, ret = rl_ops.gae(self.buf["rewards"], self.buf["values"], self.buf["starts"], self.buf["last_values"],
                              self.cur_start, float(algo.gamma), float(algo.gae_lambda), moments=self._ev_mom)
        self._last_clip_range = clip
        self._last_lr = lr
        obs = self.buf["obs_buf"].reshape(rows, self.D)
        acts = self.buf["act_raw"].reshape(rows, -1)
        old_logp = self.buf["logp"].reshape(rows)
        adv = adv.reshape(rows).contiguous()
        ret = ret.reshape(rows).contiguous()
        d = dict(self._ppo_static)
        d.update(clip_range=clip, lr=lr)
        if direct:
            d.update(zero_stats=1, norm_count_i=self.pol_norm.count if self.pol_norm is not None else None)
        else:
            self.stats.zero_()
        if world == 1:
            perm = self._epoch_perms(rows, self._seed)
            d.update(obs=obs, acts=acts, old_logp=old_logp, adv=adv, returns=ret, perm=perm, mode=0)
            self._C.engine_ppo_update(d)
        elif self._dp_replicated:
            self._ppo_update_replicated(d, obs, acts, old_logp, adv, ret)
        else:
            perm = self._epoch_perms(rows, self._seed)
            d.update(obs=obs, acts=acts, old_logp=old_logp, adv=adv, returns=ret, perm=perm)
            n_mb = rows // algo.batch_size
            B = algo.batch_size
            for it in range(algo.n_epochs * n_mb):
                e, mb = divmod(it, n_mb)
                if self.pol_norm is not None:
                    idx = perm[e, mb * B : (mb + 1) * B].long()
                    self._dp_norm_update(obs.index_select(0, idx))
                d["mode"] = 1
                d["mb_index"] = it
                self._C.engine_ppo_update(d)
                pdist.allreduce_grads_flat(self.grads)
                d["mode"] = 2
                self._C.engine_ppo_update(d)
        if self.pol_norm is not None and not direct:
            self.pol_norm.count.copy_(self.norm_count.to(self.pol_norm.count.dtype).reshape(()))
        # one marker behind the update: the round's host wait and the log copies' stream order
        self._ppo_done = self._dev_event()
        algo._n_updates += algo.n_epochs
        self._last_ppo_info = (rows, algo.n_epochs * (rows // algo.batch_size))
        self._stage_ppo_logs()
        # reads the error word of an EARLIER update (non-blocking; its copy on the log stream,
        # off the update -> next chain path); train() ends blocking
        self._ppo_err.check("PPO update", stream=self._log_stream)

    def _stage_ppo_logs(self) -> None:
        """Async D2H copy (stream order: right behind the update) of the update's statistics, the
        explained-variance moments and log_std into pinned memory; :meth:`_ppo_log_values` reads
        them after the copy event -- no blocking read of device tensors at logging time (the next
        round may already be enqueued behind the update)."""
        if getattr(self, "_ppo_log_host", None) is None:
            self._ppo_log_host = th.zeros(self._log_dev.numel(), pin_memory=True)
            self._ppo_std_host = th.zeros(self.A, pin_memory=True) if self.has_log_std else None
        # on a stream of their own: the copies stay off the update -> next rollout chain, and off
        # the side stream the discriminator updates (enqueued after this) run on concurrently
        # with the update. The next round's update, which rewrites these buffers, is enqueued
        # only after the host has waited for this event.
        if getattr(self, "_log_stream", None) is None:
            self._log_stream = shared_stream(self._dev, "engine_log")
        done = getattr(self, "_ppo_done", None)
        if done is not None:
            self._wait_ev(self._log_stream, done)
        else:
            self._log_stream.wait_stream(th.cuda.current_stream(self._dev))
        with th.cuda.stream(self._log_stream):
            self._ppo_log_host.copy_(self._log_dev, non_blocking=True)
            if self._ppo_std_host is not None:
                self._ppo_std_host.copy_(self.gen_algo.policy.log_std.detach().reshape(-1), non_blocking=True)
            self._ppo_log_event = th.cuda.Event()
            self._ppo_log_event.record()

    def _record_round_metrics(self) -> None:
        """The host PPO's per-round records (``rl/ppo.py`` ``train`` + ``rl/base.py``
        ``_dump_logs``) for one device round."""
        algo = self.gen_algo
        lg = self.logger
        vals = self._ppo_log_values()
        self._fail_if_nonfinite({k: v for k, v in vals.items() if k != "train/explained_variance"}, "PPO update")
        for k, v in vals.items():
            lg.record(k, v)
        lg.record("train/n_updates", algo._n_updates, exclude="tensorboard")
        now = time.perf_counter()
        t_prev, n_prev = getattr(self, "_fps_mark", (None, None))
        if t_prev is not None and now > t_prev and algo.num_timesteps > n_prev:
            dt = now - t_prev
            lg.record("time/fps", int((algo.num_timesteps - n_prev) / dt))
            lg.record("time/time_elapsed", int(dt), exclude="tensorboard")
        self._fps_mark = (now, algo.num_timesteps)
        lg.record("time/iterations", 1, exclude="tensorboard")
        lg.record("time/total_timesteps", algo.num_timesteps, exclude="tensorboard")
        if algo.ep_info_buffer:
            lg.record("rollout/ep_rew_mean", float(np.mean([e["r"] for e in algo.ep_info_buffer])))
            lg.record("rollout/ep_len_mean", float(np.mean([e["l"] for e in algo.ep_info_buffer])))

    def _fail_if_nonfinite(self, values: Mapping[str, float], what: str) -> None:
        """Fail fast (the reference raises on broken invariants, e.g.
        ``algorithms/base.py:77-110``): the round's statistics are already on the host, so this
        costs no device sync. A NaN / Inf loss means the weights it came from are poisoned."""
        bad = [k for k, v in values.items() if not np.isfinite(v)]
        if bad:
            from imitation_amd.utils.watchdog import NonFiniteError

            rnd = getattr(self, "_global_step", None)
            raise NonFiniteError(f"non-finite {what} statistics{'' if rnd is None else f' in round {rnd}'}: "
                                 f"{', '.join(bad)}")

    def _ppo_log_values(self) -> Dict[str, float]:
        """SB3 ``PPO.train`` metrics of the latest update (reference keys, ``rl/ppo.py``): means of
        the per-minibatch sums, ``train/loss`` from those means (SB3 logs the last minibatch's),
        explained variance of the round's values vs GAE returns, std of the Gaussian head."""
        self._ppo_log_event.synchronize()
        algo: PPO = self.gen_algo
        h = self._ppo_log_host.numpy()
        rows, n_mb = self._last_ppo_info
        s = h[:5] / max(1, n_mb)
        out = {"train/entropy_loss": float(s[0]), "train/policy_gradient_loss": float(s[1]),
               "train/value_loss": float(s[2]), "train/clip_fraction": float(s[3]), "train/approx_kl": float(s[4]),
               "train/loss": float(s[1] + algo.ent_coef * s[0] + algo.vf_coef * s[2]),
               "train/explained_variance": rl_ops.explained_variance_from_moments(h[5:], rows),
               "train/clip_range": float(self._last_clip_range), "train/learning_rate": float(self._last_lr)}
        if self._ppo_std_host is not None:
            out["train/std"] = float(np.exp(self._ppo_std_host.numpy()).mean())
        return out

    def check_errors(self, blocking: bool = False) -> None:
        """Raise if a cooperating PPO workgroup timed out in any update so far."""
        self._ppo_err.check("PPO update", blocking=blocking)

    def _setup_dp(self) -> None:
        """Data-parallel PPO plan. With the register-chained kernel available for the global
        minibatch (world x batch rows), every rank all-gathers the round's rollout rows
        (ONE collective of rows x (D + A + 3) floats) and runs the identical, deterministic
        update over the global batch -- exactly synchronous DP (averaged minibatch gradients,
        global advantage / normaliser statistics), with no per-minibatch collective. The
        minibatch permutation comes from a generator seeded identically on every rank.
        Otherwise the per-minibatch grad/all-reduce/apply kernels are used."""
        world = pdist.world_size()
        self._dp_replicated = False
        if world <= 1:
            return
        algo: PPO = self.gen_algo
        rows = self.T * self.N
        path = ppo_path(algo.policy, self._native, algo.batch_size * world, rows * world)
        self._dp_replicated = path.startswith("rc")
        self._dp_perm_seed = int(pdist.broadcast_object(int(np.random.randint(0, 2**62))))
        Aw = 1 if self.discrete else self.A
        self._dp_cols = (self.D, Aw)
        self._dp_pack = th.zeros(rows, self.D + Aw + 3, device=self._dev)
        self._dp_global = th.zeros(world * rows, self.D + Aw + 3, device=self._dev)

    def _ppo_update_replicated(self, d: Dict[str, Any], obs, acts, old_logp, adv, ret) -> None:
        algo: PPO = self.gen_algo
        world = pdist.world_size()
        rows = obs.shape[0]
        D, Aw = self._dp_cols
        pk = self._dp_pack
        pk[:, :D] = obs
        pk[:, D : D + Aw] = acts
        pk[:, D + Aw] = old_logp
        pk[:, D + Aw + 1] = adv
        pk[:, D + Aw + 2] = ret
        pdist.all_gather_flat(self._dp_global, pk)
        gl = self._dp_global
        rows_g = world * rows
        perm = self._epoch_perms(rows_g, self._dp_perm_seed)
        d.update(obs=gl[:, :D].contiguous(), acts=gl[:, D : D + Aw].contiguous(),
                 old_logp=gl[:, D + Aw].contiguous(), adv=gl[:, D + Aw + 1].contiguous(),
                 returns=gl[:, D + Aw + 2].contiguous(), perm=perm, rows=rows_g, batch=algo.batch_size * world,
                 mode=0, allow_rc=1)
        self._C.engine_ppo_update(d)
        # stats are sums over the global minibatches; every rank holds the same model

    def _epoch_perms(self, rows: int, base_seed: int) -> th.Tensor:
        """``[n_epochs, rows]`` int32 minibatch orders of this update: one ``perm_feistel``
        launch keyed by (base seed, update counter) -- replicas that share the base seed
        (replicated DP) draw identical orders, and the counter is checkpointed."""
        self._perm_round += 1
        key = (int(base_seed) * 0x9E3779B97F4A7C15 + self._perm_round) & ((1 << 64) - 1)
        return rl_ops.random_permutations(self.gen_algo.n_epochs, rows, key, self._dev)

    def _dp_norm_update(self, batch: th.Tensor) -> None:
        """RunningNorm.update_stats with all-reduced moments (the kernel is told not to update)."""
        norm = self.pol_norm
        mean, var, cnt = pdist.allreduce_moments(batch)
        c0 = self.norm_count
        tot = c0 + cnt
        delta = mean - norm.running_mean
        norm.running_mean.add_(delta * cnt / tot)
        rv = norm.running_var * c0 + var * cnt + delta.square() * c0 * cnt / tot
        norm.running_var.copy_(rv / tot)
        self.norm_count.add_(cnt)

    def _eval_block(self, n: int, seed: int, deterministic: bool, reward: bool):
        """A fresh block of ``n`` native envs (reset from ``seed``) and the scratch buffers of one
        ``max_episode_steps`` launch of the rollout chain (+ the reward pass when ``reward``)."""
        from imitation_amd.envs.vec_env import NativeVecEnv

        dev = self._dev
        ev = NativeVecEnv(self._native.env_id, n, seed=int(seed), max_episode_steps=self.max_steps)
        obs0 = ev.reset()
        st = ev.get_state()
        T = self.max_steps  # every env finishes >= 1 episode per launch (TimeLimit)
        Aw = 1 if self.discrete else self.A
        z = lambda *s: th.zeros(*s, device=dev)  # noqa: E731
        bufs = dict(obs_buf=z(T, n, self.D), act_raw=z(T, n, Aw), act_env=z(T, n, Aw), env_rew=z(T, n),
                    starts=z(T, n), trunc=z(T, n), next_obs=z(T, n, self.D))
        if reward:
            bufs.update(values=z(T, n), logp=z(T, n), boot=z(T, n), rewards=z(T, n), last_values=z(n))
        pol = self.gen_algo.policy
        args = dict(env=self._native.env_id, max_steps=self.max_steps, T=T, N=n,
                    seed=int(seed) * 0x2545F4914F6CDD1D & ((1 << 62) - 1),
                    state=th.as_tensor(st["state"], device=dev).float().contiguous(),
                    rng=th.as_tensor(st["rng"].astype(np.int64), device=dev).contiguous(),
                    elapsed=th.as_tensor(st["elapsed"].astype(np.int32), device=dev).contiguous(), ep_ret=z(n),
                    cur_obs=th.as_tensor(np.asarray(obs0, np.float32), device=dev).reshape(n, self.D).contiguous(),
                    cur_start=th.ones(n, device=dev),
                    pi=self._wave_mlp(self.pi_layers, self.hidden_act, 0, self.pol_norm),
                    log_std=pol.log_std.detach() if self.has_log_std else None, act_low=self.act_low,
                    act_high=self.act_high, n_actions=self.A if self.discrete else 0, deterministic=int(deterministic))
        return T, bufs, args

    def _eval_learned_reward(self, T: int, n: int, bufs: Dict[str, th.Tensor], args: Dict[str, Any],
                             dones: th.Tensor, out: th.Tensor) -> None:
        """The learned reward of one eval launch (the reward pass of training rollouts, written
        without the TimeLimit bootstrap) into ``out`` [T, n]."""
        algo: PPO = self.gen_algo
        pol = algo.policy
        d = dict(T=T, N=n, D=self.D, A=1 if self.discrete else self.A, n_actions=self.A if self.discrete else 0,
                 gamma=float(algo.gamma), cur_obs=args["cur_obs"],
                 pi=self._wave_mlp(self.pi_layers, self.hidden_act, 0, self.pol_norm),
                 vf=self._wave_mlp(self.vf_layers, self.hidden_act, 0, self.pol_norm),
                 log_std=pol.log_std.detach() if self.has_log_std else None, rew_enabled=1, dones=dones)
        d.update({k: bufs[k] for k in ("obs_buf", "act_raw", "act_env", "next_obs", "trunc", "env_rew", "values",
                                       "logp", "boot", "rewards", "last_values")})
        d.update(self._reward_spec())
        self._C.engine_rollout_post(d)
        out.copy_(bufs["rewards"] - bufs["boot"])

    def _eval_supports_learned_reward(self) -> bool:
        """AIRL's output normalisation runs in a separate pass over the training buffers; its
        evaluation-time rewards come from the host path."""
        out_norm = getattr(self, "_output_norm", None)
        return out_norm is None or out_norm() is None

    @profiling.traced("eval/device")
    def device_evaluate(self, n_eval_episodes: int = 10, deterministic: bool = True, n_envs: Optional[int] = None,
                        seed: int = 0) -> Tuple[List[float], List[int]]:
        """``evaluate_policy(policy, venv, n_eval_episodes, deterministic, return_episode_rewards=True)``
        on the GPU (reference ``stable_baselines3.common.evaluation.evaluate_policy``, the metric
        of ``scripts/ingredients/policy_evaluation.py``): a separate block of ``n_envs`` native
        envs (default: the training count) reset from ``seed`` and stepped by the rollout chain
        kernel with the current policy (mean / argmax actions when ``deterministic``), one
        ``max_episode_steps`` launch per episode slot -- no host round trip per step. Env ``i``
        contributes its first ``(n_eval_episodes + i) // n_envs`` episodes, as SB3 counts them;
        returns (episode returns, episode lengths) in completion order. The training envs, the
        policy and every normaliser are untouched."""
        n = int(n_envs or self.N)
        targets = np.array([(n_eval_episodes + i) // n for i in range(n)], dtype=np.int64)
        n_chunks = int(targets.max(initial=0))
        if n_chunks == 0:
            return [], []
        T, bufs, args = self._eval_block(n, seed, deterministic, reward=False)
        dones = th.zeros(n_chunks, T, n, device=self._dev)
        rets = th.zeros(n_chunks, T, n, device=self._dev)
        for c in range(n_chunks):
            args.update(bufs, step0=c * T, dones=dones[c], ep_ret_out=rets[c])
            self._C.engine_rollout(args)
        d = dones.reshape(n_chunks * T, n).cpu().numpy() > 0.5
        r = rets.reshape(n_chunks * T, n).cpu().numpy()
        ts, es = np.nonzero(d)  # row-major: completion step, then env
        ep_rewards: List[float] = []
        ep_lengths: List[int] = []
        last = np.full(n, -1, dtype=np.int64)
        count = np.zeros(n, dtype=np.int64)
        for t, e in zip(ts.tolist(), es.tolist()):
            length = t - last[e]
            last[e] = t
            if count[e] < targets[e]:
                ep_rewards.append(float(r[t, e]))
                ep_lengths.append(int(length))
                count[e] += 1
        return ep_rewards, ep_lengths

    def device_demonstrations(self, min_timesteps: int, deterministic: bool = False, seed: int = 0,
                              n_envs: Optional[int] = None) -> types.Transitions:
        """Rollouts of the current policy as flat demonstration transitions (``rollout.rollout`` +
        ``flatten_trajectories`` of whole episodes, the way the reference's experts are rolled out
        for the benchmarks) from a fresh env block on the GPU: launches of ``max_episode_steps``
        until ``min_timesteps`` transitions of finished episodes are collected; episodes in
        completion order (per launch: by env), each in time order; ``dones`` marks true
        terminations only (a TimeLimit cut is not terminal)."""
        n = int(n_envs or self.N)
        T, bufs, args = self._eval_block(n, seed, deterministic, reward=False)
        parts: Dict[str, List[np.ndarray]] = {k: [] for k in ("obs", "acts", "next_obs", "dones")}
        carry = [dict(obs=[], acts=[], next_obs=[]) for _ in range(n)]  # episodes spanning launches
        got, c = 0, 0
        while got < min_timesteps:
            dones = th.zeros(T, n, device=self._dev)
            args.update(bufs, step0=c * T, dones=dones, ep_ret_out=th.zeros(T, n, device=self._dev))
            self._C.engine_rollout(args)
            c += 1
            d = dones.cpu().numpy() > 0.5
            obs, nxt = bufs["obs_buf"].cpu().numpy(), bufs["next_obs"].cpu().numpy()
            acts = bufs["act_env"].cpu().numpy()
            trunc = bufs["trunc"].cpu().numpy() > 0.5
            for e in range(n):
                cur = carry[e]
                t0 = 0
                for t in np.flatnonzero(d[:, e]).tolist() + [None]:
                    t1 = T if t is None else t + 1
                    cur["obs"].append(obs[t0:t1, e])
                    cur["acts"].append(acts[t0:t1, e])
                    cur["next_obs"].append(nxt[t0:t1, e])
                    if t is not None:
                        length = sum(len(x) for x in cur["acts"])
                        for k in ("obs", "acts", "next_obs"):
                            parts[k].append(np.concatenate(cur[k]))
                            cur[k] = []
                        dn = np.zeros(length, dtype=bool)
                        dn[-1] = not trunc[t, e]
                        parts["dones"].append(dn)
                        got += length
                    t0 = t1
        acts = np.concatenate(parts["acts"])
        if self.discrete:
            acts = acts.reshape(-1).astype(np.int64)
        return types.Transitions(obs=np.concatenate(parts["obs"]).astype(np.float32), acts=acts,
                                 next_obs=np.concatenate(parts["next_obs"]).astype(np.float32),
                                 dones=np.concatenate(parts["dones"]), infos=np.array([{}] * len(acts)))

    @profiling.traced("eval/device_stats")
    def device_rollout_stats(self, n_episodes: int, deterministic: bool = False, seed: Optional[int] = None,
                             n_envs: Optional[int] = None) -> Optional[Dict[str, float]]:
        """``rollout_stats(generate_trajectories(policy, venv_train, make_min_episodes(n)))`` -- the
        CLI's final ``imit_stats`` (reference ``scripts/ingredients/policy_evaluation.py``) -- on the
        GPU: stochastic actions by default (``generate_trajectories``' default), the same
        unbiased stopping (once >= ``n`` episodes are done, every env finishes its episode in
        flight and stops), ``return_*`` from the learned reward the training rollouts see and
        ``monitor_return_*`` / ``len_*`` from the env. A fresh env block reset from ``seed``
        (default: derived from the engine seed); the training state is untouched. Returns None
        where the learned reward is not available on this path (AIRL with output normalisation)."""
        if not self._eval_supports_learned_reward():
            return None
        n = int(n_envs or self.N)
        seed = int(self._seed % (1 << 31)) + 7 if seed is None else int(seed)
        T, bufs, args = self._eval_block(n, seed, deterministic, reward=not self.debug_use_ground_truth)
        dl, rl, wl = [], [], []
        count = 0
        c = 0
        finishing = False
        while True:  # launches until >= n episodes, then one more so every in-flight episode ends
            dones, rets = th.zeros(T, n, device=self._dev), th.zeros(T, n, device=self._dev)
            args.update(bufs, step0=c * T, dones=dones, ep_ret_out=rets)
            self._C.engine_rollout(args)
            if self.debug_use_ground_truth:
                w = bufs["env_rew"].clone()
            else:
                w = th.zeros(T, n, device=self._dev)
                self._eval_learned_reward(T, n, bufs, args, dones, w)
            dl.append(dones)
            rl.append(rets)
            wl.append(w)
            c += 1
            if finishing:
                break
            count += int(dones.sum().item())
            finishing = count >= n_episodes
        d = th.cat(dl).cpu().numpy() > 0.5
        r = th.cat(rl).cpu().numpy()
        wr = th.cat(wl).double().cpu().numpy()
        cs = np.cumsum(wr, axis=0)
        active = np.ones(n, dtype=bool)
        start = np.zeros(n, dtype=np.int64)
        rets, lens, mon = [], [], []
        for t in range(d.shape[0]):
            fin = np.flatnonzero(d[t] & active)
            for e in fin.tolist():
                ln = t - start[e] + 1
                rets.append(float(cs[t, e] - (cs[start[e] - 1, e] if start[e] > 0 else 0.0)))
                lens.append(int(ln))
                mon.append(float(r[t, e]))
            for e in np.flatnonzero(d[t]).tolist():
                start[e] = t + 1
            if len(rets) >= n_episodes:
                active &= ~d[t]
            if not active.any():
                break
        out: Dict[str, float] = {"n_traj": len(rets)}
        for name, vals in (("return", np.asarray(rets)), ("len", np.asarray(lens)), ("monitor_return", np.asarray(mon))):
            for stat in ("min", "mean", "std", "max"):
                out[f"{name}_{stat}"] = getattr(np, stat)(vals).item()
        out["monitor_return_len"] = len(mon)
        return out

    def sync_env_to_host(self) -> None:
        """Copy the device env state back into the native host env (e.g. before host-side evaluation)."""
        self._native.set_state({"state": self.state.cpu().numpy(), "rng": self.env_rng.cpu().numpy(),
                                "elapsed": self.elapsed.cpu().numpy().astype(np.int64)})

    def _stage_rollout_to_host(self):
        """Async D2H copy of (dones, episode returns) into pinned buffers; returns the event
        that marks them ready."""
        wrapped = not self.debug_use_ground_truth
        if not hasattr(self, "_host_stage"):
            self._host_stage = th.empty(4 if wrapped else 2, self.T, self.N, pin_memory=True)
        # on the side stream: the copies stay off the rollout -> GAE -> PPO chain (the host
        # waits for this event before the next rollout can overwrite the buffers)
        side = getattr(self, "_side_stream", None)
        if side is not None:
            self._wait_ev(side, self._dev_event())
        with th.cuda.stream(side) if side is not None else contextlib.nullcontext():
            self._host_stage[0].copy_(self.buf["dones"], non_blocking=True)
            self._host_stage[1].copy_(self.buf["ep_ret_out"], non_blocking=True)
            if wrapped:  # learned reward = rewards - TimeLimit bootstrap (RewardVecEnvWrapper's rews)
                self._host_stage[2].copy_(self.buf["rewards"], non_blocking=True)
                self._host_stage[3].copy_(self._boot, non_blocking=True)
            ev = th.cuda.Event()
            ev.record()
        self._host_staged = True
        return ev

def flatten_order(dones: np.ndarray, ep_lens_running: np.ndarray):
    """Replay order of one round's ``[T, N]`` transitions as BufferingWrapper -> flatten ->
    FIFO store produces it: finished episodes in completion order ((end step, env) row-major),
    each in time order, then every env's unfinished tail, by env. Vectorised (no Python loop
    over steps: this runs on the host between a rollout and its discriminator updates).

    Returns ``(order, fin_t, fin_n, ep_lens, ep_lens_running')``: flat row indices
    ``t * N + n``, the end step / env of each finished episode, its full length (including the
    steps carried from earlier rounds, ``ep_lens_running``) and the updated carry."""
    T, N = dones.shape
    ep_lens_running = np.asarray(ep_lens_running, dtype=np.int64)
    fin_t, fin_n = np.nonzero(dones)  # row-major: by end step, then env
    # episode starts: previous done of the same env + 1 (0 for its first done this round)
    by_env = np.lexsort((fin_t, fin_n))
    t_env, n_env = fin_t[by_env], fin_n[by_env]
    first = np.ones(len(by_env), dtype=bool)
    first[1:] = n_env[1:] != n_env[:-1]
    s_env = np.where(first, 0, np.concatenate(([0], t_env[:-1] + 1)))
    starts = np.empty_like(s_env)
    starts[by_env] = s_env
    is_first = np.empty_like(first)
    is_first[by_env] = first
    lens = fin_t - starts + 1
    ep_lens = (lens + np.where(is_first, ep_lens_running[fin_n], 0)).astype(np.int64)
    # tails: from the last done + 1 (or 0) to T - 1
    seg_start = np.zeros(N, dtype=np.int64)
    last = np.ones(len(by_env), dtype=bool)
    last[:-1] = n_env[:-1] != n_env[1:]
    seg_start[n_env[last]] = t_env[last] + 1
    done_any = np.zeros(N, dtype=bool)
    done_any[n_env] = True
    running = np.where(done_any, T - seg_start, ep_lens_running + T)
    tail_n = np.flatnonzero(seg_start < T)
    tail_s = seg_start[tail_n]
    # concatenated ranges [s, e] -> row indices, episodes first, then tails
    seg_s = np.concatenate((starts, tail_s))
    seg_len = np.concatenate((lens, T - tail_s))
    seg_env = np.concatenate((fin_n, tail_n))
    total = int(seg_len.sum())
    offs = np.repeat(np.cumsum(seg_len) - seg_len, seg_len)
    t_rows = np.repeat(seg_s, seg_len) + (np.arange(total) - offs)
    order = t_rows * N + np.repeat(seg_env, seg_len)
    return order.astype(np.int64), fin_t, fin_n, ep_lens.tolist(), running


class DeviceEngineMixin(DeviceGeneratorCore):
    """Device generator rounds (rollout -> GAE -> PPO -> replay store) and the fused
    discriminator update for an :class:`~imitation_amd.algorithms.adversarial.common.AdversarialTrainer`
    subclass; mixed in front of GAIL (:class:`DeviceGAIL`) or AIRL
    (:class:`imitation_amd.engine.airl.DeviceAIRL`)."""

    _host_cls_name = "the host trainer"

    @staticmethod
    def _supports(venv, gen_algo, reward_net) -> Tuple[bool, str]:
        return supports(venv, gen_algo, reward_net)

    def __init__(self, *, demonstrations, demo_batch_size: int, venv, gen_algo: PPO, reward_net: reward_nets.RewardNet, **kwargs):
        ok, why = self._supports(venv, gen_algo, reward_net)
        if not ok:
            raise ValueError(f"{type(self).__name__} not applicable: {why}; use {self._host_cls_name}")
        super().__init__(demonstrations=demonstrations, demo_batch_size=demo_batch_size, venv=venv, gen_algo=gen_algo,
                         reward_net=reward_net, **kwargs)
        self._init_generator(venv)
        D = self.D
        act_shape = () if self.discrete else (self.A,)
        self._gen_dev = buffer_mod.DeviceBuffer(
            self._gen_replay_buffer.capacity, {"obs": (D,), "acts": act_shape, "next_obs": (D,), "dones": ()},
            {"obs": th.float32, "acts": th.int64 if self.discrete else th.float32, "next_obs": th.float32,
             "dones": th.bool}, self._dev)
        self._setup_fused_disc()

    @profiling.traced("host/replay_store")
    def _store_generator_samples(self) -> None:
        """Replay-buffer content identical to BufferingWrapper -> flatten -> FIFO store."""
        wrapped_rew = None
        if getattr(self, "_host_staged", False):
            dones = self._host_stage[0].numpy().astype(bool)
            ep_ret_host = self._host_stage[1].numpy()
            if self._host_stage.shape[0] == 4:
                wrapped_rew = self._host_stage[2].numpy() - self._host_stage[3].numpy()
            self._host_staged = False
        else:
            dones = self.buf["dones"].to("cpu", non_blocking=False).numpy().astype(bool)  # [T, N] (one sync / round)
            ep_ret_host = None
        T, N = dones.shape
        self._track_wrapped_returns(dones, wrapped_rew)
        order, fin_t, fin_n, ep_lens, self._ep_lens_running = flatten_order(dones, self._ep_lens_running)
        cap = self._gen_dev.capacity
        # pinned + non-blocking: a pageable H2D copy would block the host until the stream
        # reaches it (in an AIRL split round: until the PPO kernel ends, which left the round's
        # staging and the next step chain to be enqueued behind the GPU instead of ahead of it)
        keep = th.from_numpy(np.ascontiguousarray(order[-cap:])).pin_memory().to(self._dev, non_blocking=True)
        rows = T * N
        acts = self.buf["act_env"].reshape(rows, -1)
        if self.discrete:
            acts = acts.reshape(rows).long()
        self._gen_dev.store({
            "obs": self.buf["obs_buf"].reshape(rows, self.D).index_select(0, keep),
            "acts": acts.index_select(0, keep),
            "next_obs": self.buf["next_obs"].reshape(rows, self.D).index_select(0, keep),
            "dones": self.buf["dones"].reshape(rows).index_select(0, keep).bool(),
        })
        local_lens = list(ep_lens)
        if pdist.world_size() > 1 and not self.allow_variable_horizon:
            # global horizon set == {global min, global max}: one 2-float MIN all-reduce
            lo, neg_hi = pdist.allreduce_scalars([min(ep_lens, default=2**31), -max(ep_lens, default=-1)], op="min")
            ep_lens = [] if lo > -neg_hi else sorted({int(lo), int(-neg_hi)})
        self._check_fixed_horizon(ep_lens)
        # Monitor-style episode stats for the generator logger
        if len(fin_t):
            ep_ret = ep_ret_host if ep_ret_host is not None else self.buf["ep_ret_out"].cpu().numpy()
            algo = self.gen_algo
            if algo.ep_info_buffer is None:
                import collections

                algo.ep_info_buffer = collections.deque(maxlen=algo._stats_window_size)
            for t, n, l_full in zip(fin_t.tolist(), fin_n.tolist(), local_lens):
                algo.ep_info_buffer.append({"r": float(ep_ret[t, n]), "l": int(l_full), "t": 0.0})

    def _track_wrapped_returns(self, dones: np.ndarray, rew: Optional[np.ndarray]) -> None:
        """``RewardVecEnvWrapper`` episode bookkeeping (reference ``rewards/reward_wrapper.py:15-37,
        92-133``): per-env running sums of the learned reward, a deque of the last 100 finished
        episodes' sums; ``rollout/ep_rew_wrapped_mean`` is its mean at the START of the rollout
        (``WrappedRewardCallback._on_rollout_start``), i.e. before this round's episodes."""
        import collections

        if getattr(self, "_wrapped_eps", None) is None:
            self._wrapped_eps = collections.deque(maxlen=100)
            self._wrapped_cum = np.zeros(dones.shape[1], dtype=np.float64)
        eps = self._wrapped_eps
        self._wrapped_mean_at_start = (sum(eps) / len(eps)) if eps else None
        if rew is None:
            return
        T, N = dones.shape
        cs = np.cumsum(rew.astype(np.float64), axis=0)  # [T, N] running sums within the round
        fin_t, fin_n = np.nonzero(dones)  # completion order: step, then env (the wrapper's loop)
        prev = np.full(N, -1, dtype=np.int64)
        vals = np.empty(len(fin_t), dtype=np.float64)
        for n in range(N):  # per env: segment sums between consecutive dones (+ the carry)
            sel = np.flatnonzero(fin_n == n)
            if not len(sel):
                continue
            t = fin_t[sel]
            before = np.concatenate(([0.0], cs[t[:-1], n]))
            v = cs[t, n] - before
            v[0] += self._wrapped_cum[n]
            vals[sel] = v
            prev[n] = t[-1]
        eps.extend(vals.tolist())
        last = np.where(prev >= 0, cs[T - 1] - np.where(prev >= 0, cs[np.maximum(prev, 0), np.arange(N)], 0.0),
                        self._wrapped_cum + cs[T - 1])
        self._wrapped_cum = last

    def _gen_sample(self, batch_size: int) -> Dict[str, th.Tensor]:
        if self._gen_dev.size() == 0:
            raise RuntimeError("No generator samples for training. Call `train_gen()` first.")
        return self._gen_dev.sample(batch_size)

    def train_gen(self, total_timesteps: Optional[int] = None, learn_kwargs: Optional[Mapping] = None) -> None:
        """One (or more) device rounds: rollout -> GAE -> PPO update -> replay store."""
        if total_timesteps is None:
            total_timesteps = self.gen_train_timesteps
        algo: PPO = self.gen_algo
        n_rounds = max(1, total_timesteps // (self.T * self.N))
        with self.logger.accumulate_means("gen"):
            for _ in range(n_rounds):
                if algo._total_timesteps < algo.num_timesteps + self.T * self.N:
                    algo._total_timesteps = algo.num_timesteps + self.T * self.N
                self._rollout()
                # episode bookkeeping needs dones / returns on the host: copy them right after
                # the rollout and let the CPU work while the PPO kernel runs
                ready = self._stage_rollout_to_host()
                algo.num_timesteps += self.T * self.N
                self._ppo_update()
                ready.synchronize()
                self._store_generator_samples()
                self._global_step += 1
            self._log_gen()

    @profiling.traced("host/log_gen")
    def _log_gen(self, stats: Optional[th.Tensor] = None) -> None:
        """Record one generator round with the host trainer's key set: SB3 ``PPO.train`` metrics
        (:meth:`_ppo_log_values`), ``OnPolicyAlgorithm._dump_logs`` (``time/*``, Monitor
        ``rollout/ep_*_mean``) and the reward wrapper's ``rollout/ep_rew_wrapped_mean``
        (reference ``adversarial/common.py:234-240, 414-419``). ``time/fps``: env steps per
        second of wall time since the previous round's record (the round's sustained rate; the
        reference's per-round ``learn`` call gives the same quantity). ``stats`` is unused (kept
        for callers that pass the old host copy)."""
        self._record_round_metrics()
        wm = getattr(self, "_wrapped_mean_at_start", None)
        if wm is not None:
            self.logger.record("rollout/ep_rew_wrapped_mean", float(wm))

    # ------------------------------------------------------------------ fused discriminator update
    def _fused_disc_check(self) -> Tuple[bool, str]:
        if type(self).logits_expert_is_high is not GAIL.logits_expert_is_high:
            return False, "custom discriminator logits"
        opt = self._disc_opt
        if type(opt) is not th.optim.Adam or len(opt.param_groups) != 1:
            return False, "discriminator optimizer is not a single-group torch.optim.Adam"
        g = opt.param_groups[0]
        if any(g.get(k) for k in ("amsgrad", "maximize", "capturable", "differentiable", "decoupled_weight_decay")):
            return False, "Adam variant not fused"
        if self._init_tensorboard:
            return False, "tensorboard summaries need per-step logits"
        if not isinstance(self._endless_expert_iterator, common._DeviceDemoSampler):
            return False, "demonstrations are not a flat device transitions set"
        base = self._reward_net.base if isinstance(self._reward_net, reward_nets.NormalizedRewardNet) else self._reward_net
        try:
            norm, lins, _, out_act = _mlp_layers(base.mlp)
        except ValueError as e:
            return False, str(e)
        if norm is not None and type(norm) is not networks.RunningNorm:
            return False, "reward-net input normaliser is not RunningNorm"
        if out_act != 0 or lins[-1].out_features != 1 or len(lins) > 4:
            return False, "reward MLP shape"
        if max([lins[0].in_features] + [l.out_features for l in lins]) > 128:
            return False, "reward MLP wider than 128"
        mlp_params = {id(p) for l in lins for p in (l.weight, l.bias)}
        if {id(p) for p in self._reward_net.parameters()} != mlp_params:
            return False, "reward net has parameters outside its MLP"
        if self.pol_norm is not None and (type(self.pol_norm) is not networks.RunningNorm or not base.use_state):
            return False, "policy normaliser"
        return True, ""

    def _setup_fused_disc(self) -> None:
        ok, why = self._fused_disc_check()
        self._fused_disc = ok
        self._fused_disc_why = why
        if not ok:
            return
        dev = self._dev
        base = self._reward_net.base if isinstance(self._reward_net, reward_nets.NormalizedRewardNet) else self._reward_net
        norm, lins, hid, _ = _mlp_layers(base.mlp)
        self._rnorm = norm
        plist: List[nn.Parameter] = []
        for l in lins:
            plist += [l.weight, l.bias]
        self._rflat = _FlatParams(plist)
        n = self._rflat.n
        self._r_m = th.zeros(n, device=dev)
        self._r_v = th.zeros(n, device=dev)
        self._adopt_disc_opt_state()
        sampler = self._endless_expert_iterator
        ed = sampler.data
        ed["obs"] = ed["obs"].float().contiguous()
        ed["next_obs"] = ed["next_obs"].float().contiguous()
        ed["acts"] = (ed["acts"].long() if self.discrete else ed["acts"].float()).reshape(ed["acts"].shape[0], -1)
        ed["acts"] = ed["acts"].reshape(-1).contiguous() if self.discrete else ed["acts"].contiguous()
        ed["dones"] = ed["dones"].bool().contiguous()
        gd = self._gen_dev._arrays
        B, mb = self.demo_batch_size, self.demo_minibatch_size
        dims = [lins[0].in_features] + [l.out_features for l in lins]
        gblk, fblk, n_params = self._C.disc_plan_sizes(dims, mb)
        assert n_params == n, (n_params, n)
        n_mb = B // mb
        z = lambda *sh, dt=th.float32: th.zeros(*sh, device=dev, dtype=dt)  # noqa: E731
        self._disc_ws = dict(X=z(2 * mb, dims[0]), partials=z(gblk * 2 * dims[0]), slab=z(n_mb * fblk * n),
                             stats_slab=z(n_mb * fblk * 8), grads=z(n), sums=z(2 * dims[0], dt=th.float64))
        self._disc_stats = z(max(1, self.n_disc_updates_per_round), 8)
        g = self._disc_opt.param_groups[0]
        d = dict(batch=B, minibatch=mb, W=[l.weight for l in lins], b=[l.bias for l in lins], hidden_act=int(hid),
                 rew_mean=norm.running_mean if norm is not None else None,
                 rew_var=norm.running_var if norm is not None else None,
                 rew_count=norm.count if norm is not None else None, rew_eps=float(norm.eps) if norm is not None else 1e-5,
                 obs_dim=self.D, act_width=self.A, use_state=int(base.use_state), use_action=int(base.use_action),
                 use_next_state=int(base.use_next_state), use_done=int(base.use_done), act_discrete=int(self.discrete),
                 e_obs=ed["obs"], e_next_obs=ed["next_obs"], e_acts=ed["acts"], e_dones=ed["dones"],
                 g_obs=gd["obs"], g_next_obs=gd["next_obs"], g_acts=gd["acts"], g_dones=gd["dones"],
                 pol_mean=self.pol_norm.running_mean if self.pol_norm is not None else None,
                 pol_var=self.pol_norm.running_var if self.pol_norm is not None else None,
                 pol_count=self.pol_norm.count if self.pol_norm is not None else None,
                 params=self._rflat.flat, exp_avg=self._r_m, exp_avg_sq=self._r_v,
                 beta1=float(g["betas"][0]), beta2=float(g["betas"][1]), eps=float(g["eps"]),
                 weight_decay=float(g.get("weight_decay", 0.0)), **self._disc_ws)
        self._disc_plan = self._C.DiscPlan(d)
        # Overlap (see train()): the round's discriminator updates run on a side stream
        # concurrently with its PPO update. They only read the expert set, the replay ring
        # and the reward net; their one write the PPO kernel also makes -- the policy
        # RunningNorm merge of the disc batch (GAIL's log-prob side effect) -- is recorded
        # per minibatch and applied in order after PPO, so the result is bitwise that of
        # the serial order.
        self._overlap_disc = os.environ.get("IMITATION_AMD_DISC_OVERLAP", "1") != "0"
        self._side_stream = shared_stream(dev, "engine_side") if self._overlap_disc else None
        self._pol_defer_buf = None
        if self._overlap_disc and self.pol_norm is not None and self._disc_plan.pol_cols > 0:
            self._ensure_pol_defer(max(1, self.n_disc_updates_per_round))
        self._disc_stats_host = th.zeros(max(1, self.n_disc_updates_per_round), 8, pin_memory=True)

    def _ensure_pol_defer(self, n_updates: int) -> None:
        slots = n_updates * self._disc_plan.n_minibatches
        if self._pol_defer_buf is None or self._pol_defer_buf.shape[0] < slots:
            self._pol_defer_buf = th.zeros(slots, 2 * self._disc_plan.pol_cols + 1, device=self._dev)
            self._disc_plan.set_pol_defer(self._pol_defer_buf)

    def _adopt_disc_opt_state(self) -> None:
        """Make the torch Adam state of every reward parameter a view of the flat moment
        buffers the fused kernel updates (copying in any state the optimizer already has,
        e.g. after ``load_state_dict``), so both update paths and checkpoints agree."""
        opt = self._disc_opt
        for p, off in zip(self._rflat.params, self._rflat.offsets):
            k = p.numel()
            m = self._r_m[off : off + k].view_as(p)
            v = self._r_v[off : off + k].view_as(p)
            st = opt.state.get(p)
            if st and st.get("exp_avg") is not None and st["exp_avg"].data_ptr() == m.data_ptr() \
                    and st["exp_avg_sq"].data_ptr() == v.data_ptr():
                continue
            step = th.tensor(0.0)
            if st:
                with th.no_grad():
                    m.copy_(st["exp_avg"])
                    v.copy_(st["exp_avg_sq"])
                step = st["step"] if isinstance(st["step"], th.Tensor) else th.tensor(float(st["step"]))
            else:
                m.zero_()
                v.zero_()
            opt.state[p] = {"step": step, "exp_avg": m, "exp_avg_sq": v}

    @profiling.traced("disc/update")
    def _fused_disc_update(self, slot: int, defer_pol: bool = False) -> None:
        """One discriminator optimizer step (== AdversarialTrainer.train_disc) with no host sync.
        ``defer_pol``: record the policy-norm merges in slots ``slot * n_minibatches + k`` of
        the deferred-merge buffer instead of applying them (see :meth:`train`)."""
        if self._gen_dev.size() == 0:
            raise RuntimeError("No generator samples for training. Call `train_gen()` first.")
        opt = self._disc_opt
        self._adopt_disc_opt_state()
        g = opt.param_groups[0]
        t = float(opt.state[self._rflat.params[0]]["step"]) + 1.0
        beta1, beta2 = g["betas"]
        lr = float(g["lr"])
        step_size = lr / (1.0 - beta1**t)
        bc2_sqrt = (1.0 - beta2**t) ** 0.5
        B, mb = self.demo_batch_size, self.demo_minibatch_size
        e_idx = self._endless_expert_iterator.next_indices()
        g_idx = th.randint(0, self._gen_dev.size(), (B,), device=self._dev)
        merge_rew = self._rnorm is not None and self._rnorm.training
        merge_pol = self.pol_norm is not None and self.pol_norm.training
        plan = self._disc_plan
        stats_out = self._disc_stats[slot]
        base = slot * plan.n_minibatches if (defer_pol and merge_pol) else -1
        if pdist.world_size() == 1:
            plan.update(e_idx, g_idx, step_size, bc2_sqrt, merge_rew, merge_pol, stats_out, base)
        else:
            world = pdist.world_size()
            for k in range(B // mb):
                plan.gather(k, e_idx, g_idx)
                if merge_rew or merge_pol:
                    ds = base + k if base >= 0 else -1
                    if pdist.norm_sync_active():
                        plan.norm(1, 0, merge_rew, merge_pol)
                        pdist.allreduce_sum_(self._disc_ws["sums"])
                        plan.norm(2, 2 * mb * world, merge_rew, merge_pol, ds)
                    else:
                        plan.norm(0, 0, merge_rew, merge_pol, ds)
                plan.fwd_bwd(k)
            plan.adam(1, 0, 0.0, 1.0, stats_out)
            pdist.allreduce_grads_flat(self._disc_ws["grads"])
            plan.adam(0, 1, step_size, bc2_sqrt, None)
        for p in self._rflat.params:
            opt.state[p]["step"] += 1
        self._disc_step += 1

    def _disc_stats_dict(self, v: Sequence[float]) -> Mapping[str, float]:
        B, mb = self.demo_batch_size, self.demo_minibatch_size
        rows = 2 * mb
        return common.train_stats_from_sums(
            [v[0] / rows * (mb / B), v[1] / rows, float(mb), v[2], v[3], v[4], v[5] / rows], float(rows))

    @profiling.traced("host/log_disc")
    def _record_disc(self, stats: Mapping[str, float], disc_step: int) -> None:
        self.logger.record("global_step", self._global_step)
        for k, v in stats.items():
            self.logger.record(k, v)
        self.logger.dump(disc_step)

    def train_disc(self, *, expert_samples: Optional[Mapping] = None, gen_samples: Optional[Mapping] = None) -> Mapping[str, float]:
        if not self._fused_disc or expert_samples is not None or gen_samples is not None:
            return super().train_disc(expert_samples=expert_samples, gen_samples=gen_samples)
        with self.logger.accumulate_means("disc"):
            self._fused_disc_update(0)
            stats = self._disc_stats_dict(self._disc_stats[0].tolist())
            self._record_disc(stats, self._disc_step)
        return stats

    # ------------------------------------------------------------------ graphed generic discriminator update
    def _graphed_disc_ok(self) -> bool:
        """The generic (autograd) discriminator step -- e.g. AIRL's shaped reward net, which
        the fused kernels do not cover -- as one HIP-graph replay per update: single
        process (no gradient all-reduce / norm collectives), a capturable optimiser, the
        device demo sampler, and no per-step tensorboard summaries (a host sync)."""
        from imitation_amd.utils import graphs

        # under DP the gradient mean and the normaliser moments go through the one-shot
        # all-reduce kernel, which a graph can hold (RCCL / gloo collectives cannot)
        single = pdist.world_size() == 1 and self._disc_bucket is None
        return (not self._fused_disc and (single or pdist.oneshot_active())
                and graphs.graphs_enabled(self._dev, "IMITATION_AMD_DISC_GRAPH")
                and graphs.supports_capture(self._disc_opt) and not self._init_tensorboard
                and isinstance(self._endless_expert_iterator, common._DeviceDemoSampler))

    def _generic_disc_fn(self, e_obs, e_acts, e_next, e_dones, g_idx) -> th.Tensor:
        """``AdversarialTrainer.train_disc``'s minibatch losses, backward and optimiser step
        over device batches (expert rows given, generator rows gathered from the device replay
        buffer by ``g_idx``); returns the last minibatch's statistics sums (device)."""
        import torch.nn.functional as F

        from imitation_amd.ops import optim as optim_ops
        from imitation_amd.ops.rl import gather_rows

        ga = self._gen_dev._arrays
        keys = ("obs", "acts", "next_obs", "dones")
        gen = dict(zip(keys, gather_rows([ga[k] for k in keys], g_idx)))  # one launch
        ex = {"obs": e_obs, "acts": e_acts, "next_obs": e_next, "dones": e_dones}
        # a single minibatch per update (the tuned configs): its gradients go straight into
        # FusedAdam's (zeroed) bucket, no accumulate-add per parameter
        into_buckets = (isinstance(self._disc_opt, optim_ops.FusedAdam)
                        and self.demo_minibatch_size == self.demo_batch_size)
        for batch in self._make_disc_train_batches(gen_samples=gen, expert_samples=ex):
            logits = self.logits_expert_is_high(batch["state"], batch["action"], batch["next_state"], batch["done"],
                                                batch["log_policy_act_prob"])
            loss = F.binary_cross_entropy_with_logits(logits, batch["labels_expert_is_one"].float())
            loss = loss * (self.demo_minibatch_size / self.demo_batch_size)
            if into_buckets:
                self._disc_opt.backward_into_buckets(loss)
            else:
                loss.backward()
        if pdist.world_size() > 1:  # mean over ranks of the flat bucket(s): one-shot, in-graph
            pdist.FlatGradBucket(self._disc_opt).allreduce()
        self._disc_opt.step()
        return common.train_stats_vec(logits, batch["labels_expert_is_one"], loss)

    def _graphed_disc_update(self, slot: int) -> None:
        from imitation_amd.utils import graphs

        if self._gen_dev.size() == 0:
            raise RuntimeError("No generator samples for training. Call `train_gen()` first.")
        if getattr(self, "_disc_graph", None) is None:
            # torch Adam's capturable step is ~30 multi-tensor launches; the flat-bucket
            # FusedAdam (same hyper-parameters and state) is one
            from imitation_amd.ops import optim as optim_ops

            self._disc_opt = optim_ops.to_fused(self._disc_opt)
            self._disc_graph = graphs.GraphedTrainStep(self._generic_disc_fn, self._disc_opt)
        ex = self._next_expert_batch()
        g_idx = th.randint(0, self._gen_dev.size(), (self.demo_batch_size,), device=self._dev)
        out = self._disc_graph(ex["obs"], ex["acts"], ex["next_obs"], ex["dones"], g_idx)
        self._disc_stats_gen[slot].copy_(out)
        self._disc_step += 1

    def _train_graphed_generic(self, total_timesteps: int, callback=None) -> None:
        n_rounds = total_timesteps // self.gen_train_timesteps
        assert n_rounds >= 1, (
            f"No updates (need at least {self.gen_train_timesteps} timesteps, have only total_timesteps={total_timesteps})!")
        n = self.n_disc_updates_per_round
        if getattr(self, "_disc_stats_gen", None) is None or self._disc_stats_gen.shape[0] < n:
            self._disc_stats_gen = th.zeros(max(n, 1), 7, device=self._dev)
        rows = float(2 * self.demo_minibatch_size)
        for r in range(n_rounds):
            self.train_gen(self.gen_train_timesteps)
            steps = []
            with networks.training(self.reward_train):
                for i in range(n):
                    self._graphed_disc_update(i)
                    steps.append(self._disc_step)
            vals = self._disc_stats_gen[:n].tolist() if n else []  # one host sync per round
            pdist.check_comm("adversarial round")
            self._fail_if_nonfinite({f"update {i} sum {j}": float(v) for i in range(n) for j, v in enumerate(vals[i])},
                                    "discriminator")
            for i in range(n):
                with self.logger.accumulate_means("disc"):
                    self._record_disc(common.train_stats_from_sums(vals[i], rows), steps[i])
            if callback:
                callback(r)
            self.logger.dump(self._global_step)
        self.check_errors(blocking=True)

    #: Keep the round pipeline when ``train`` is given a callback: round ``r + 1``'s rollout
    #: (chain + reward pass) is already enqueued when ``callback(r)`` runs. The callback sees
    #: round ``r``'s final weights and may read (e.g. checkpoint) any state; it must not mutate
    #: the env state, the policy or the reward net in place (the in-flight rollout reads them).
    #: The CLI's checkpoint callback (reference ``scripts/train_adversarial.py:156-160``) only
    #: saves. False: every callback runs with the device idle, as a host-loop trainer would.
    pipeline_callbacks = True

    @gcfreeze.during
    def train(self, total_timesteps: int, callback=None) -> None:
        """Rounds of device generator training + fused discriminator updates; the
        discriminator statistics of a round are fetched with one host sync and logged
        per update exactly as the reference's ``train_disc`` does. At the end the host env
        mirrors the device env state: a host-side evaluation on ``venv_train`` (the reference
        CLI's final ``eval_policy``, e.g. AIRL with output normalisation) then continues from
        the training env state, as the reference's does, whether or not a checkpoint or a
        resume copied it before."""
        if not self._fused_disc:
            if self._graphed_disc_ok():
                self._train_graphed_generic(total_timesteps, callback)
            else:
                super().train(total_timesteps, callback)
        else:
            self._train_fused(total_timesteps, callback)
        self.sync_env_to_host()

    def _train_fused(self, total_timesteps: int, callback=None) -> None:
        n_rounds = total_timesteps // self.gen_train_timesteps
        assert n_rounds >= 1, (
            f"No updates (need at least {self.gen_train_timesteps} timesteps, have only total_timesteps={total_timesteps})!")
        n = self.n_disc_updates_per_round
        if n > self._disc_stats.shape[0]:
            self._disc_stats = th.zeros(n, 8, device=self._dev)
            self._disc_stats_host = th.zeros(n, 8, pin_memory=True)
        overlap = self._overlap_disc and n > 0 and self.gen_train_timesteps == self.T * self.N
        nxt = None
        self._fps_mark = (time.perf_counter(), self.gen_algo.num_timesteps)
        timer = profiling.StepTimer(roctx=False)
        timer.n0 = self.gen_algo.num_timesteps
        for r in range(n_rounds):
            if overlap:
                # the next rollout is enqueued before this round's logging and callback (see
                # pipeline_callbacks), so the device never waits for the host between rounds
                launch = r + 1 < n_rounds and (callback is None or self.pipeline_callbacks)
                steps, nxt = self._overlapped_round(n, nxt, launch_next=launch)
                vals = self._disc_stats_host[:n].tolist()
            else:
                self.train_gen(self.gen_train_timesteps)
                steps = []
                with networks.training(self.reward_train):
                    for i in range(n):
                        self._fused_disc_update(i)
                        steps.append(self._disc_step)
                vals = self._disc_stats[:n].tolist() if n else []
            pdist.check_comm("GAIL round")
            if n:
                self._fail_if_nonfinite({f"update {i} sum {j}": float(v) for i in range(n) for j, v in enumerate(vals[i][:6])},
                                        "discriminator")
                for i in range(n):
                    with self.logger.accumulate_means("disc"):
                        self._record_disc(self._disc_stats_dict(vals[i]), steps[i])
            if callback:
                callback(r)
            self.logger.dump(self._global_step)
        pdist.check_comm("GAIL training", blocking=True)
        self.check_errors(blocking=True)
        self._report_throughput(timer)

    def _report_throughput(self, timer: "profiling.StepTimer") -> None:
        """Per-rank and whole-node env-steps/s of this ``train`` call: host wall
        time of the call (its rounds are pipelined, so this is the sustained rate), one small
        all-reduce under DP. Recorded as ``perf/*`` and kept in ``last_train_perf``."""
        timer.add_env_steps(self.gen_algo.num_timesteps - timer.n0)
        rep = timer.report()
        self.last_train_perf = rep
        for k in ("rank_env_steps_per_s", "node_env_steps_per_s", "elapsed_s", "world_size"):
            self.logger.record(f"perf/{k}", rep[k])
        self.logger.dump(self._global_step)

    def _launch_rollout(self) -> th.cuda.Event:
        """Enqueue one rollout (chain + post pass) and the async copy of its dones / returns to
        pinned host memory; returns the event that marks both done."""
        self._rollout()
        return self._stage_rollout_to_host()

    def _overlapped_round(self, n: int, ready: Optional[th.cuda.Event] = None,
                          launch_next: bool = False) -> Tuple[List[int], Optional[th.cuda.Event]]:
        """One GAIL round with its ``n`` discriminator updates on the side stream, concurrent
        with the PPO update (the round's rewards were already computed from the previous
        discriminator, so nothing PPO reads changes).

        ``ready``: the round's rollout was already enqueued (by the previous call) and this
        is its staging event. ``launch_next``: enqueue the next round's rollout behind this
        round's PPO + deferred merges BEFORE waiting for PPO on the host, so the GPU never
        idles while the host logs. Returns (disc steps, next round's staging event); the
        disc stats are in ``_disc_stats_host`` when this returns."""
        algo: PPO = self.gen_algo
        main = th.cuda.current_stream(self._dev)
        # AIRL (_disc_on_main): log pi needs the post-PPO policy, so the updates queue behind PPO
        # on the main stream -- the round is still pipelined: nothing waits on the host between
        # PPO, the updates and the next rollout
        side = main if getattr(self, "_disc_on_main", False) else self._side_stream
        pol_merge = self.pol_norm is not None and self.pol_norm.training
        defer = pol_merge and self._pol_defer_buf is not None
        if defer:
            self._ensure_pol_defer(n)
        # serial when the disc would write the norm PPO is using, or when both would issue
        # per-step collectives: the non-replicated DP PPO all-reduces every minibatch through
        # the same one-shot communicator as the disc, and two kernels in flight on it would
        # pair one rank's PPO gradients with another rank's disc sums
        serial = (pol_merge and not defer) or (pdist.world_size() > 1 and not self._dp_replicated)
        steps: List[int] = []
        nxt = None
        # AIRL split rounds: the updates' gathers + norm merges (the only part the next rollout's
        # step chain depends on, through the policy RunningNorm) are staged on the main stream;
        # the fwd/bwd + Adam applies run on the side stream concurrently with that chain, and
        # the rollout's reward pass waits for them
        # (single rank only; the policy-norm merges are on the main stream, ahead of the chain)
        split = getattr(self, "_disc_split", False) and n > 0
        with self.logger.accumulate_means("gen"):
            if algo._total_timesteps < algo.num_timesteps + self.T * self.N:
                algo._total_timesteps = algo.num_timesteps + self.T * self.N
            if ready is None:
                ready = self._launch_rollout()
            algo.num_timesteps += self.T * self.N
            self._ppo_update()
            ppo_done = self._ppo_done
            ready.synchronize()
            if split:
                return self._split_round(n, ppo_done, launch_next, steps)
            if serial:
                self._wait_ev(side, ppo_done)
            else:
                side.wait_event(ready)
            with th.cuda.stream(side):
                self._store_generator_samples()
                with networks.training(self.reward_train):
                    for i in range(n):
                        self._fused_disc_update(i, defer_pol=defer)
                        steps.append(self._disc_step)
                disc_dev = self._dev_event(side)
                self._disc_stats_host[:n].copy_(self._disc_stats[:n], non_blocking=True)
                disc_done = th.cuda.Event()
                disc_done.record(side)
            self._wait_ev(main, disc_dev)
            if defer:
                self._disc_plan.pol_norm_merge(n * self._disc_plan.n_minibatches)
            self._global_step += 1
            if launch_next:
                nxt = self._launch_rollout()
            ppo_done.synchronize()
            self._log_gen()
        disc_done.synchronize()
        return steps, nxt

    def _stage_during_ppo(self) -> bool:
        """Split-round staging on the side stream, concurrent with PPO. Under data parallelism
        only with the replicated PPO update, which issues no collective: the staging's normaliser
        all-reduces are then the only users of the communicator while they run.
        IMITATION_AMD_AIRL_EARLY_STAGE=0: stage behind PPO on the main stream."""
        return ((pdist.world_size() == 1 or self._dp_replicated) and getattr(self, "_host_staged", False)
                and os.environ.get("IMITATION_AMD_AIRL_EARLY_STAGE", "1") != "0")

    def _split_round(self, n: int, ppo_done: th.cuda.Event, launch_next: bool,
                     steps: List[int]) -> Tuple[List[int], Optional[th.cuda.Event]]:
        """Rest of an AIRL split round after PPO (see _overlapped_round): stage the updates on
        the main stream, apply them on the side stream while the next rollout's step chain runs,
        then the rollout's reward pass behind the applies."""
        main = th.cuda.current_stream(self._dev)
        side = self._side_stream
        if self._stage_during_ppo():
            # replay store, gathers and base / potential merges on the side stream while PPO
            # runs (none of it touches the policy norm or the policy); then the policy-norm
            # merges, one launch, behind PPO on the main stream. The side stream is already
            # ordered after the rollout (_stage_rollout_to_host).
            with th.cuda.stream(side):
                self._store_generator_samples()
                with networks.training(self.reward_train):
                    scal = self._stage_disc_updates(n, defer_q=True)
                side_staged = self._dev_event(side)
            self._wait_ev(main, side_staged)
            self._merge_deferred_q(n)
            self._early_staged_rounds = getattr(self, "_early_staged_rounds", 0) + 1
        else:
            self._store_generator_samples()
            with networks.training(self.reward_train):
                scal = self._stage_disc_updates(n)
        staged = self._dev_event(main)
        # the next step chain is enqueued before the applies (host order only: it depends on
        # the staging, not on the applies), so a slow host never delays its start
        if launch_next:
            self._launch_chain()
        self._wait_ev(side, staged)
        with th.cuda.stream(side):
            self._apply_disc_updates(scal, steps)
            disc_dev = self._dev_event(side)
            self._disc_stats_host[:n].copy_(self._disc_stats[:n], non_blocking=True)
            disc_done = th.cuda.Event()
            disc_done.record(side)
        self._global_step += 1
        nxt = None
        if launch_next:
            self._wait_ev(main, disc_dev)
            reward = not self.debug_use_ground_truth
            self._launch_post(reward)
            if reward:
                self._post_rollout_rewards()
            nxt = self._stage_rollout_to_host()
        else:
            self._wait_ev(main, disc_dev)
        ppo_done.synchronize()
        self._log_gen()
        disc_done.synchronize()
        return steps, nxt

    # ------------------------------------------------------------------ checkpoint / resume
    _ENGINE_TENSORS = ("exp_avg", "exp_avg_sq", "adam_step", "state", "env_rng", "elapsed", "ep_ret", "cur_obs", "cur_start")

    def engine_state(self) -> Dict[str, Any]:
        """Device-engine state not covered by module ``state_dict``s (used by
        :mod:`imitation_amd.utils.checkpoint`); parameters live in the policy modules."""
        st: Dict[str, Any] = {k: getattr(self, k).detach().cpu().clone() for k in self._ENGINE_TENSORS}
        if self.norm_count is not None:
            if self.pol_norm is not None:  # (the single-rank update keeps the module's count only)
                self.norm_count.copy_(self.pol_norm.count.reshape(1))
            st["norm_count"] = self.norm_count.cpu().clone()
        if getattr(self, "_wrapped_eps", None) is not None:
            st["wrapped_eps"] = th.tensor(list(self._wrapped_eps), dtype=th.float64)
            st["wrapped_cum"] = th.as_tensor(self._wrapped_cum, dtype=th.float64)
        st.update(step0=int(self._step0), seed=int(self._seed), perm_round=int(self._perm_round), ep_lens_running=th.as_tensor(self._ep_lens_running),
                  gen_dev={k: v.cpu().clone() for k, v in self._gen_dev._arrays.items()},
                  gen_dev_idx=int(self._gen_dev._idx), gen_dev_n=int(self._gen_dev._n_data))
        return st

    def load_engine_state(self, st: Dict[str, Any]) -> None:
        with th.no_grad():
            for k in self._ENGINE_TENSORS:
                getattr(self, k).copy_(st[k].to(self._dev))
            if self.norm_count is not None and "norm_count" in st:
                self.norm_count.copy_(st["norm_count"].to(self._dev))
            for k, v in st["gen_dev"].items():
                self._gen_dev._arrays[k].copy_(v.to(self._dev))
        self._step0, self._seed = st["step0"], st["seed"]
        self._perm_round = int(st.get("perm_round", 0))
        self._ep_lens_running = st["ep_lens_running"].numpy().copy()
        if "wrapped_eps" in st:
            import collections

            self._wrapped_eps = collections.deque(st["wrapped_eps"].tolist(), maxlen=100)
            self._wrapped_cum = st["wrapped_cum"].numpy().copy()
        self._gen_dev._idx, self._gen_dev._n_data = st["gen_dev_idx"], st["gen_dev_n"]
        self.sync_env_to_host()


class DeviceGAIL(DeviceEngineMixin, GAIL):
    """GAIL whose generator rounds run entirely on the GPU (see module docstring)."""

    _host_cls_name = "algorithms.adversarial.gail.GAIL"


def smoke_round(device) -> None:
    """Tiny end-to-end device round (used by ``__graft_entry__.smoke``)."""
    from imitation_amd.data import rollout as rollout_mod
    from imitation_amd.policies.base import FeedForward32Policy, NormalizeFeaturesExtractor
    from imitation_amd.util import logger as imit_logger
    from imitation_amd.util.util import make_vec_env

    rng = np.random.default_rng(0)
    venv = make_vec_env("seals/HalfCheetah-v1", rng=rng, n_envs=8)
    demo_env = make_vec_env("seals/HalfCheetah-v1", rng=np.random.default_rng(1), n_envs=4)
    demos = rollout_mod.flatten_trajectories(
        rollout_mod.generate_trajectories(None, demo_env, rollout_mod.make_min_timesteps(2048), rng=rng))
    gen = PPO(FeedForward32Policy, venv, n_steps=64, batch_size=64, n_epochs=2, device=device,
              policy_kwargs=dict(features_extractor_class=NormalizeFeaturesExtractor))
    rn = reward_nets.BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=networks.RunningNorm)
    tr = DeviceGAIL(demonstrations=demos, demo_batch_size=256, venv=venv, gen_algo=gen, reward_net=rn,
                    n_disc_updates_per_round=2, custom_logger=imit_logger.configure("/tmp/ia_smoke", format_strs=[]))
    tr.train(2 * 64 * 8)
    th.cuda.synchronize()
    assert all(th.isfinite(p).all() for p in gen.policy.parameters())

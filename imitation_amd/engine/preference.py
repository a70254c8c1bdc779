"""Device-resident agent for preference comparisons (DRLHP) -- the MI355X fast path of
:class:`imitation_amd.algorithms.preference_comparisons.AgentTrainer`.

Reference: ``src/imitation/algorithms/preference_comparisons.py:127-316``.
The reference agent is SB3 PPO stepping a ``RewardVecEnvWrapper(BufferingWrapper(venv))``
on the host: every env step crosses numpy <-> device twice (policy, learned reward) and
the BufferingWrapper accumulates per-env partial trajectories in Python lists. Here:

=================================  ==================================================
reference                          this engine
=================================  ==================================================
``algorithm.learn(steps)``         device rounds: ONE rollout kernel per round (policy
(collect_rollouts + PPO.train)     + env physics + ``reward_net.predict_processed``,
                                   incl. NormalizedRewardNet output norm), GAE kernel,
                                   persistent PPO kernel (:mod:`.gail`'s generator core)
``BufferingWrapper`` trajectories  the round's (obs, act, env reward, done, terminal
                                   obs) land in pinned host memory with one async copy
                                   that overlaps the PPO kernel; episodes are cut on the
                                   host with numpy slices
extra ``generate_trajectories``    envs reset (as ``generate_trajectories`` does) then
(policy, stochastic)               rollout-kernel rounds without the reward MLP until
                                   enough episodes finished
``ExplorationWrapper`` rollouts    same kernel with a per-step explore schedule drawn
                                   from the trainer's rng with the wrapper's switching
                                   rule (uniform ``Box``/``Discrete`` actions)
=================================  ==================================================

Trajectories are ``TrajectoryWithRew`` objects with the same content as the
BufferingWrapper's (obs incl. terminal obs, clipped env actions, env rewards,
``terminal=True``), so fragmenting, gathering and reward training are unchanged.
"""

from __future__ import annotations

import math
import os
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch as th

from imitation_amd.algorithms.preference_comparisons import AgentTrainer, _get_trajectories
from imitation_amd.data import types
from imitation_amd.engine.airl import OutputNormMixin
from imitation_amd.engine.gail import DeviceGeneratorCore, _mlp_layers, supports_generator
from imitation_amd.rewards import reward_nets
from imitation_amd.util import networks


def _split(reward_net) -> Tuple[Any, Any]:
    if isinstance(reward_net, reward_nets.NormalizedRewardNet):
        return reward_net.normalize_output_layer, reward_net.base
    return None, reward_net


def _ensemble_of(reward_fn) -> Tuple[Optional[reward_nets.RewardEnsemble], Optional[float]]:
    """(stackable RewardEnsemble, std coefficient) behind ``reward_fn`` or (None, None):
    a bare ensemble rewards its member mean, ``AddSTDRewardWrapper`` mean + alpha * std."""
    alpha = 0.0
    ens = reward_fn
    if isinstance(reward_fn, reward_nets.AddSTDRewardWrapper):
        ens, alpha = reward_fn.base, float(reward_fn.default_alpha)
    if isinstance(ens, reward_nets.RewardEnsemble) and ens.stack() is not None:
        return ens, alpha
    return None, None


def supports(venv, algorithm, reward_fn) -> Tuple[bool, str]:
    """Whether :class:`DeviceAgentTrainer` can run this agent (reason when not)."""
    ok, why = supports_generator(venv, algorithm)
    if not ok:
        return ok, why
    if not isinstance(reward_fn, reward_nets.RewardNet):
        return False, "reward_fn is not a RewardNet"
    ens, _ = _ensemble_of(reward_fn)
    if ens is not None:
        return (True, "") if ens.device.type == "cuda" else (False, "ensemble not on the GPU")
    if isinstance(reward_fn, (reward_nets.RewardEnsemble, reward_nets.AddSTDRewardWrapper)):
        return False, "ensemble members do not stack (not identical BasicRewardNet MLPs)"
    out_norm, base = _split(reward_fn)
    if out_norm is not None and type(out_norm) is not networks.RunningNorm:
        return False, "output normaliser is not RunningNorm"
    if type(base) is not reward_nets.BasicRewardNet:
        return False, "reward net is not a BasicRewardNet"
    try:
        norm, lins, _, _ = _mlp_layers(base.mlp)
    except ValueError as e:
        return False, str(e)
    if norm is not None and not isinstance(norm, networks.BaseNorm):
        return False, "unsupported input normaliser"
    if len(lins) > 4 or max([lins[0].in_features] + [l.out_features for l in lins]) > 64:
        return False, "reward MLP too wide / deep for the rollout kernel"
    return True, ""


class DeviceAgentTrainer(OutputNormMixin, DeviceGeneratorCore, AgentTrainer):
    """:class:`AgentTrainer` whose PPO agent trains and samples on the GPU (module docstring)."""

    def __init__(self, algorithm, reward_fn, venv, rng: np.random.Generator, exploration_frac: float = 0.0,
                 switch_prob: float = 0.5, random_prob: float = 0.5, custom_logger=None) -> None:
        ok, why = supports(venv, algorithm, reward_fn)
        if not ok:
            raise ValueError(f"DeviceAgentTrainer not applicable: {why}; use preference_comparisons.AgentTrainer")
        super().__init__(algorithm=algorithm, reward_fn=reward_fn, venv=venv, rng=rng, exploration_frac=exploration_frac,
                         switch_prob=switch_prob, random_prob=random_prob, custom_logger=custom_logger)
        self.gen_algo = algorithm
        self._reward_net = reward_fn
        self.debug_use_ground_truth = False
        self.switch_prob = switch_prob
        self.random_prob = random_prob
        self._init_generator(venv)
        # the ExplorationWrapper drew its initial policy from ``rng`` at construction
        ew = self.exploration_wrapper
        self._explore_random = ew.current_policy == ew._random_policy
        T, N = self.T, self.N
        self._rew_raw = th.zeros(T, N, device=self._dev)
        self._onorm_count = th.zeros(1, device=self._dev)
        self._explore_dev = th.zeros(T, dtype=th.int32, device=self._dev)
        Aw = 1 if self.discrete else self.A
        self._stage_cols = (self.D, self.D, Aw, 1, 1, 1)  # obs, next_obs, act_env, env_rew, dones, wrapped rew
        self._stage_host = th.empty(T, N, sum(self._stage_cols), pin_memory=True)
        self._stage_dev = th.empty(T, N, sum(self._stage_cols), device=self._dev)
        self._reset_accumulator()
        self._finished: List[types.TrajectoryWithRew] = []
        self._n_since_pop = 0
        self._wrapped_ret = np.zeros(N, dtype=np.float64)

    # ------------------------------------------------------------------ kernels
    def _rollout(self) -> None:
        """Single reward nets run inside the post pass; an ensemble (active selection,
        ``AddSTDRewardWrapper``) is scored afterwards for all T x N transitions with ONE
        grouped launch over its stacked members, then mean (+ alpha * unbiased std)."""
        ens, alpha = _ensemble_of(self._reward_net)
        if ens is None or self.debug_use_ground_truth:
            return super()._rollout()
        self._launch_chain()
        self._launch_post(False)  # values, log-probs, TimeLimit bootstrap
        b = self.buf
        T, N = self.T, self.N
        st = ens.stack()
        flat = lambda t: t.reshape(T * N, -1)  # noqa: E731
        acts = b["act_env"].reshape(T * N) if self.discrete else flat(b["act_env"])
        with th.no_grad():
            s, a, ns, d = ens.members[0].preprocess(flat(b["obs_buf"]), acts, flat(b["next_obs"]), b["dones"].reshape(-1))
            r_all = st.forward(st.features(s, a, ns, d), st.gather_params(), st.gather_norm())  # [M, T*N]
            r = r_all.mean(0)
            if alpha:
                r = r + alpha * r_all.var(0, unbiased=True).sqrt()
            b["rewards"].copy_(r.view(T, N) + self._boot)

    def _reward_spec(self) -> Dict[str, Any]:
        """``reward_net.predict_processed``: the base MLP's raw output (eval-mode input norm)."""
        _, base = _split(self._reward_net)
        rnorm, rl, rh, ro = _mlp_layers(base.mlp)
        return dict(rew=self._wave_mlp(rl, rh, ro, rnorm), use_state=int(base.use_state), use_action=int(base.use_action),
                    use_next_state=int(base.use_next_state), use_done=int(base.use_done), rew_transform=0)

    def _rollout_extra_bufs(self) -> Dict[str, Any]:
        return {"rew_raw": self._rew_raw}

    def _sample_rollout(self, explore: bool) -> None:
        """One rollout-kernel round of the current (stochastic) policy without the learned
        reward -- ``generate_trajectories`` / ExplorationWrapper sampling. Only the serial
        chain runs: values, log-probs and rewards are not needed for sampling."""
        explore_mode = None
        if explore:
            sched = np.zeros(self.T, dtype=np.int32)
            for t in range(self.T):  # ExplorationWrapper.__call__: act, then maybe switch
                sched[t] = int(self._explore_random)
                if self.rng.random() < self.switch_prob:
                    self._explore_random = bool(self.rng.random() < self.random_prob)
            self._explore_dev.copy_(th.from_numpy(sched))
            explore_mode = self._explore_dev
        self._launch_chain(explore_mode)

    def _stage(self) -> th.cuda.Event:
        """Pack the round's trajectory columns on device, one async D2H into pinned memory."""
        T, N = self.T, self.N
        b = self.buf
        wrapped = b["rewards"] - self._boot  # learned reward as the RewardVecEnvWrapper returns it
        th.cat([b["obs_buf"], b["next_obs"], b["act_env"], b["env_rew"].unsqueeze(-1), b["dones"].unsqueeze(-1),
                wrapped.unsqueeze(-1)], dim=-1, out=self._stage_dev)
        self._stage_host.copy_(self._stage_dev, non_blocking=True)
        ev = th.cuda.Event()
        ev.record()
        return ev

    # ------------------------------------------------------------------ host trajectory accumulation
    def _reset_accumulator(self) -> None:
        self._partial: List[List[Tuple[np.ndarray, np.ndarray, np.ndarray]]] = [[] for _ in range(self.N)]

    def _accumulate(self, track_wrapped: bool) -> int:
        """Cut the staged round into finished episodes (BufferingWrapper order: by end step,
        then env index) and per-env partial segments; returns the finished transitions."""
        D, Dn, Aw = self._stage_cols[:3]
        st = self._stage_host.numpy()
        obs, nxt = st[..., :D], st[..., D : D + Dn]
        acts = st[..., D + Dn : D + Dn + Aw]
        rews = st[..., D + Dn + Aw]
        dones = st[..., D + Dn + Aw + 1] > 0.5
        wrapped = st[..., D + Dn + Aw + 2]
        T, N = dones.shape
        self._n_since_pop += T * N
        ends: List[Tuple[int, int, int]] = []
        seg_start = np.zeros(N, dtype=np.int64)
        for t, n in zip(*np.nonzero(dones)):
            ends.append((int(t), int(n), int(seg_start[n])))
            seg_start[n] = t + 1
        added = 0
        for t, n, s in ends:  # np.nonzero walks t-major: end-step order, then env index
            pieces = self._partial[n] + [(obs[s : t + 1, n], acts[s : t + 1, n], rews[s : t + 1, n])]
            self._partial[n] = []
            o = np.concatenate([p[0] for p in pieces] + [nxt[t, n][None]], axis=0)
            a = np.concatenate([p[1] for p in pieces], axis=0)
            r = np.concatenate([p[2] for p in pieces], axis=0).astype(np.float32)
            if self.discrete:
                a = a.reshape(-1).astype(np.int64)
            self._finished.append(types.TrajectoryWithRew(obs=o, acts=a, infos=None, terminal=True, rews=r))
            added += len(a)
        for n in range(N):
            if seg_start[n] < T:
                s = int(seg_start[n])
                self._partial[n].append((obs[s:, n].copy(), acts[s:, n].copy(), rews[s:, n].copy()))
        if track_wrapped:  # WrappedRewardCallback: episode returns of the learned reward
            for t in range(T):
                self._wrapped_ret += wrapped[t]
                for n in np.flatnonzero(dones[t]):
                    self.reward_venv_wrapper.episode_rewards.append(float(self._wrapped_ret[n]))
                    self._wrapped_ret[n] = 0.0
        return added

    def _pop_finished(self) -> List[types.TrajectoryWithRew]:
        out, self._finished = self._finished, []
        self._n_since_pop = 0
        return out

    def _reset_envs(self) -> None:
        """``venv.reset()`` at the start of ``generate_trajectories``: fresh episodes on every
        env (their partial trajectories are dropped, as the BufferingWrapper does)."""
        nat = self._native
        self.sync_env_to_host()
        obs0 = nat.reset()
        st = nat.get_state()
        self.state.copy_(th.as_tensor(st["state"]).float())
        self.env_rng.copy_(th.as_tensor(st["rng"].astype(np.int64)))
        self.elapsed.copy_(th.as_tensor(st["elapsed"].astype(np.int32)))
        self.cur_obs.copy_(th.as_tensor(np.asarray(obs0, np.float32)).reshape(self.N, self.D))
        self.cur_start.fill_(1.0)
        self.ep_ret.zero_()
        self._wrapped_ret[:] = 0.0
        self._reset_accumulator()

    def _generate(self, min_timesteps: int, explore: bool) -> List[types.TrajectoryWithRew]:
        """``generate_trajectories(sample_until=min_timesteps)`` followed by
        ``pop_finished_trajectories``: device rounds until enough episodes finished."""
        self._reset_envs()
        got = 0
        while got < min_timesteps:
            self._sample_rollout(explore)
            self._stage().synchronize()
            got += self._accumulate(track_wrapped=False)
        return self._pop_finished()

    # ------------------------------------------------------------------ AgentTrainer API
    def train(self, steps: int, **kwargs) -> None:
        """``algorithm.learn(total_timesteps=steps, reset_num_timesteps=False)`` as device rounds."""
        if self._n_since_pop:
            raise RuntimeError(f"There are {self._n_since_pop} transitions left in the buffer. "
                               "Call AgentTrainer.sample() first to clear them.")
        algo = self.gen_algo
        per_round = self.T * self.N
        n_rounds = max(1, math.ceil(steps / per_round))
        target = algo.num_timesteps + n_rounds * per_round
        algo._total_timesteps = max(algo._total_timesteps or 0, target)
        self._fps_mark = (time.perf_counter(), algo.num_timesteps)
        logged = True
        defer = os.environ.get("IMITATION_AMD_PREF_DEFER_LOG", "1") != "0"
        for _ in range(n_rounds):
            self._rollout()
            ready = self._stage()
            if not logged:
                # the previous round's records (its PPO statistics wait for its update) are
                # written only now, with this round's rollout already queued behind that update:
                # the GPU does not idle while the host logs. Same values, steps and order as
                # logging at the end of each round (the PPO statistics are staged copies; the
                # wrapped-return deque does not change until this round's _accumulate).
                self._log_round()
            algo.num_timesteps += per_round
            self._ppo_update()  # PPO kernel runs while the host cuts the episodes
            ready.synchronize()
            self._accumulate(track_wrapped=True)
            logged = False
            if not defer:
                self._log_round()
                logged = True
        if not logged:
            self._log_round()
        self.sync_env_to_host()  # (a host-side evaluation continues from the training env state)

    def _log_round(self) -> None:
        algo = self.gen_algo
        lg = self.logger
        self._record_round_metrics()
        ep = self.reward_venv_wrapper.episode_rewards
        if len(ep):
            lg.record("rollout/ep_rew_wrapped_mean", float(np.mean(ep)))
        lg.dump(step=algo.num_timesteps)

    def sample(self, steps: int) -> Sequence[types.TrajectoryWithRew]:
        agent_trajs = self._pop_finished()[::-1]  # newest first
        avail_steps = sum(len(t) for t in agent_trajs)
        exploration_steps = int(self.exploration_frac * steps)
        if self.exploration_frac > 0 and exploration_steps == 0:
            self.logger.warn(f"No exploration steps included: exploration_frac = {self.exploration_frac} > 0 "
                             f"but steps={steps} is too small.")
        agent_steps = steps - exploration_steps
        if avail_steps < agent_steps:
            self.logger.log(f"Requested {agent_steps} transitions but only {avail_steps} in buffer. "
                            f"Sampling {agent_steps - avail_steps} additional transitions.")
            agent_trajs = agent_trajs + self._generate(agent_steps - avail_steps, explore=False)
        trajectories = list(_get_trajectories(agent_trajs, agent_steps))
        if exploration_steps > 0:
            self.logger.log(f"Sampling {exploration_steps} exploratory transitions.")
            trajectories.extend(_get_trajectories(self._generate(exploration_steps, explore=True), exploration_steps))
        return trajectories

    # ------------------------------------------------------------------ checkpoint
    _ENGINE_TENSORS = ("exp_avg", "exp_avg_sq", "adam_step", "state", "env_rng", "elapsed", "ep_ret", "cur_obs", "cur_start")

    def engine_state(self) -> Dict[str, Any]:
        st: Dict[str, Any] = {k: getattr(self, k).detach().cpu().clone() for k in self._ENGINE_TENSORS}
        if self.norm_count is not None:
            if self.pol_norm is not None:  # (the single-rank update keeps the module's count only)
                self.norm_count.copy_(self.pol_norm.count.reshape(1))
            st["norm_count"] = self.norm_count.cpu().clone()
        st.update(step0=int(self._step0), seed=int(self._seed), perm_round=int(self._perm_round),
                  explore_random=bool(self._explore_random))
        return st

    def buffer_state(self) -> Dict[str, Any]:
        """The host-side episode cutter between iterations: finished trajectories not yet
        sampled, per-env partial segments, the learned-reward episode returns in flight."""
        from imitation_amd.utils import checkpoint

        return {"finished": [checkpoint.traj_state(t) for t in self._finished],
                "partial": [[tuple(th.as_tensor(np.ascontiguousarray(x)) for x in seg) for seg in segs]
                            for segs in self._partial],
                "n_since_pop": int(self._n_since_pop), "wrapped_ret": th.as_tensor(self._wrapped_ret.copy())}

    def load_buffer_state(self, st: Dict[str, Any]) -> None:
        from imitation_amd.utils import checkpoint

        self._finished = [checkpoint.traj_load(t) for t in st["finished"]]
        self._partial = [[tuple(x.numpy() for x in seg) for seg in segs] for segs in st["partial"]]
        self._n_since_pop = st["n_since_pop"]
        self._wrapped_ret = st["wrapped_ret"].numpy().copy()

    def load_engine_state(self, st: Dict[str, Any]) -> None:
        with th.no_grad():
            for k in self._ENGINE_TENSORS:
                getattr(self, k).copy_(st[k].to(self._dev))
            if self.norm_count is not None and "norm_count" in st:
                self.norm_count.copy_(st["norm_count"].to(self._dev))
        self._step0, self._seed = st["step0"], st["seed"]
        self._perm_round = int(st.get("perm_round", 0))  # the PPO minibatch permutations' round counter
        self._explore_random = st["explore_random"]
        self._reset_accumulator()
        self.sync_env_to_host()

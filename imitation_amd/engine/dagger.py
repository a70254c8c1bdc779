"""Device DAgger collection: env stepping, frame rendering, both policies and the β-mix on the GPU.

The reference collects every DAgger round through a host VecEnv wrapper
(``src/imitation/algorithms/dagger.py:151-287`` InteractiveTrajectoryCollector +
``data/rollout.py:426-554`` generate_trajectories): per step the frames cross the
host/device boundary for the expert forward, again for the learner forward, the
actions come back, the env steps on the CPU and every finished episode is pickled to
disk before BC re-reads everything. Here one round is:

* K env steps per HIP-graph replay (``chunk``): expert CNN forward (deterministic,
  as ``generate_trajectories(deterministic_policy=True)``), learner forward with
  sampling (``policy.predict`` default), ``rand > β`` mask, the executed action into
  ``dagger_env_step`` (csrc/kernels/dagger.hip: the IA_HD physics of the host env +
  in-place frame-stack rendering, TimeLimit, auto-reset with terminal frames), and the
  expert action / observation recorded into the round's device buffers;
* one pinned D2H copy of the chunk's done flags per replay, which drives the
  reference's unbiased stopping rule on the host (``sample_until`` over finished
  episodes, then each env runs out its current episode; steps of inactive envs are
  ignored);
* the round's finished episodes are gathered on the device into the flat demo
  aggregate BC trains on (:class:`DeviceDemoAggregate`, DP all-gathered over RCCL),
  and copied to the host once for the reference-format demo files, which a
  background thread writes (:class:`AsyncDemoWriter`).
"""

from __future__ import annotations

import os
import queue
import threading
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch as th

from imitation_amd import ops
from imitation_amd.data import types
from imitation_amd.envs import spaces
from imitation_amd.parallel import dist as pdist
from imitation_amd.rl.distributions import CategoricalDistribution, DiagGaussianDistribution
from imitation_amd.rl.policies import ActorCriticPolicy


def _unwrap_native(venv):
    from imitation_amd.envs.vec_env import NativeVecEnv

    e = venv
    while e is not None:
        if isinstance(e, NativeVecEnv):
            return e
        e = getattr(e, "venv", None)
    return None


def supports(venv, expert_policy, learner_policy) -> Tuple[bool, str]:
    """Whether :class:`DeviceDAggerCollector` can collect for this configuration."""
    if os.environ.get("IMITATION_AMD_DAGGER_DEVICE", "1") == "0":
        return False, "disabled by IMITATION_AMD_DAGGER_DEVICE=0"
    if not th.cuda.is_available():
        return False, "no GPU"
    nat = _unwrap_native(venv)
    from imitation_amd.data.wrappers import VecRolloutInfoWrapper

    # RolloutInfoWrapper only mirrors obs/rewards into infos, which device demos do not carry
    if nat is None or not (venv is nat or (isinstance(venv, VecRolloutInfoWrapper) and venv.venv is nat)):
        return False, "env is not a native vector env (optionally under RolloutInfoWrapper)"
    for name, pol in (("expert", expert_policy), ("learner", learner_policy)):
        if not isinstance(pol, ActorCriticPolicy):
            return False, f"{name} policy is not an ActorCriticPolicy"
        if pol.device.type != "cuda":
            return False, f"{name} policy is not on the GPU"
        if pol.squash_output:
            return False, f"{name} policy squashes its output"
        if type(pol.action_dist) not in (CategoricalDistribution, DiagGaussianDistribution):
            return False, f"{name} policy action distribution {type(pol.action_dist).__name__}"
    if isinstance(nat.observation_space, spaces.Dict):
        return False, "dict observations"
    if not isinstance(nat.action_space, (spaces.Discrete, spaces.Box)):
        return False, "action space"
    return True, ""


def policy_actions(policy: ActorCriticPolicy, obs: th.Tensor, deterministic: bool) -> th.Tensor:
    """``policy.predict`` on a device batch without host syncs (capturable): argmax / mean
    when deterministic, else Gumbel-max sampling of the categorical or mean + std * N(0, 1);
    Box actions are clipped to the space like ``predict`` does."""
    dist = policy.get_distribution(obs)
    if isinstance(dist, CategoricalDistribution):
        logits = dist.logits
        if deterministic:
            return logits.argmax(-1)
        u = th.rand_like(logits).clamp_(1e-20, 1.0)
        return (logits - th.log(-th.log(u))).argmax(-1)
    mean = dist.mean_actions
    a = mean if deterministic else mean + th.exp(dist.log_std) * th.randn_like(mean)
    low = th.as_tensor(policy.action_space.low, device=a.device, dtype=a.dtype)
    high = th.as_tensor(policy.action_space.high, device=a.device, dtype=a.dtype)
    return th.max(th.min(a, high), low)


class DeviceDemoAggregate:
    """Flat device-resident (obs, acts) of every aggregated DAgger demonstration, grown by
    capacity doubling; under DP each append is all-gathered so replicas hold the same rows
    in (round, rank) order."""

    def __init__(self, device):
        self.device = th.device(device)
        self.obs: Optional[th.Tensor] = None
        self.acts: Optional[th.Tensor] = None
        self.n = 0

    def append(self, obs: th.Tensor, acts: th.Tensor, gather: bool = True) -> int:
        if gather and pdist.world_size() > 1:
            obs, acts = pdist.all_gather_rows(obs), pdist.all_gather_rows(acts)
        k = obs.shape[0]
        if k == 0:
            return 0
        need = self.n + k
        if self.obs is None or need > self.obs.shape[0]:
            cap = max(need, 2 * (0 if self.obs is None else self.obs.shape[0]), 1024)
            new_obs = th.empty((cap,) + tuple(obs.shape[1:]), dtype=obs.dtype, device=self.device)
            new_acts = th.empty((cap,) + tuple(acts.shape[1:]), dtype=acts.dtype, device=self.device)
            if self.n:
                new_obs[: self.n].copy_(self.obs[: self.n])
                new_acts[: self.n].copy_(self.acts[: self.n])
            self.obs, self.acts = new_obs, new_acts
        self.obs[self.n : need].copy_(obs)
        self.acts[self.n : need].copy_(acts)
        self.n = need
        return k

    def __len__(self) -> int:
        return self.n


class DeviceTransitionsLoader:
    """Shuffled, drop-last minibatches straight from a :class:`DeviceDemoAggregate`: one
    ``perm_feistel`` launch per epoch and two ``index_select`` per batch; yields the batch
    dict BC consumes (``obs`` / ``acts`` device tensors)."""

    def __init__(self, agg: DeviceDemoAggregate, batch_size: int, seed: int):
        self.agg = agg
        self.batch_size = batch_size
        self._seed = int(seed)
        self._epoch = 0

    def __len__(self) -> int:
        return len(self.agg) // self.batch_size

    def __iter__(self):
        from imitation_amd.ops import rl as rl_ops

        n = len(self.agg)
        self._epoch += 1
        perm = rl_ops.random_permutations(1, n, self._seed * 1000003 + self._epoch, self.agg.device)[0].long()
        obs, acts = self.agg.obs, self.agg.acts
        for s in range(0, n - n % self.batch_size, self.batch_size):
            idx = perm[s : s + self.batch_size]
            yield {"obs": obs.index_select(0, idx), "acts": acts.index_select(0, idx)}


class AsyncDemoWriter:
    """Background thread that writes demo files (``fn(trajectory, index)``) in order; the
    collector hands trajectories over and goes on. ``flush()`` waits for the queue."""

    def __init__(self):
        self._q: "queue.Queue[Optional[Tuple[Callable, tuple]]]" = queue.Queue()
        self._err: Optional[BaseException] = None
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while True:
            item = self._q.get()
            try:
                if item is None:
                    return
                fn, args = item
                if self._err is None:
                    fn(*args)
            except BaseException as e:  # surfaced by flush()
                self._err = e
            finally:
                self._q.task_done()

    def submit(self, fn: Callable, *args) -> None:
        self._q.put((fn, args))

    def flush(self) -> None:
        self._q.join()
        if self._err is not None:
            err, self._err = self._err, None
            raise err

    def close(self) -> None:
        self.flush()
        self._q.put(None)
        self._t.join(timeout=5)


class DeviceDAggerCollector:
    """Collects DAgger rounds on the GPU (see module docstring).

    ``collect(beta, min_timesteps=..., min_episodes=...)`` returns the round's finished
    episodes as host :class:`~imitation_amd.data.types.TrajectoryWithRew` (expert actions,
    true rewards, ``infos=None``) and leaves their flat transitions on the device in
    ``last_obs`` / ``last_acts``. The host env's state is synced back afterwards."""

    def __init__(self, venv, expert_policy: ActorCriticPolicy, learner_policy: ActorCriticPolicy,
                 rng: np.random.Generator, chunk: int = 32, use_graph: Optional[bool] = None):
        self.venv = venv
        self.nat = _unwrap_native(venv)
        self.expert = expert_policy
        self.learner = learner_policy
        self.rng = rng
        self.chunk = int(chunk)
        self.device = learner_policy.device
        self._C = ops.native()
        self.N = self.nat.num_envs
        self.img = bool(self.nat._is_image)
        self.obs_shape = tuple(self.nat.observation_space.shape)
        self.discrete = isinstance(self.nat.action_space, spaces.Discrete)
        self.act_shape = () if self.discrete else tuple(self.nat.action_space.shape)
        self.use_graph = (os.environ.get("IMITATION_AMD_DAGGER_GRAPH", "1") != "0") if use_graph is None else use_graph
        dev, N, K = self.device, self.N, self.chunk
        odt = th.uint8 if self.img else th.float32
        adt = th.int64 if self.discrete else th.float32
        st = self.nat.get_state()
        self.state = th.as_tensor(st["state"], device=dev).float().contiguous()
        self.env_rng = th.as_tensor(st["rng"].astype(np.int64), device=dev).contiguous()
        self.elapsed = th.as_tensor(st["elapsed"].astype(np.int32), device=dev).contiguous()
        self.ep_ret = th.zeros(N, device=dev)
        self.obs = th.zeros((N,) + self.obs_shape, dtype=odt, device=dev)
        # one chunk of step records (graph-static)
        self.c_obs = th.zeros((K, N) + self.obs_shape, dtype=odt, device=dev)
        self.c_term_obs = th.zeros((K, N) + self.obs_shape, dtype=odt, device=dev)
        self.c_acts = th.zeros((K, N) + self.act_shape, dtype=adt, device=dev)
        self.c_rew = th.zeros(K, N, device=dev)
        self.c_term = th.zeros(K, N, dtype=th.uint8, device=dev)
        self.c_trunc = th.zeros(K, N, dtype=th.uint8, device=dev)
        self.c_ep_ret = th.zeros(K, N, device=dev)
        self.c_ep_len = th.zeros(K, N, dtype=th.int32, device=dev)
        self._beta = th.ones((), device=dev)
        self._host_flags = th.zeros(2, K, N, dtype=th.uint8, pin_memory=True)
        self._graph = None
        self._max_steps = int(self.nat.max_episode_steps)
        self.last_obs: Optional[th.Tensor] = None
        self.last_acts: Optional[th.Tensor] = None
        self.steps_collected = 0

    # -------------------------------------------------------------- device steps
    def _env_args(self, mode: int, k: int = 0, actions: Optional[th.Tensor] = None) -> Dict:
        d = dict(env=self.nat.env_id, N=self.N, max_steps=self._max_steps, mode=mode, state=self.state, rng=self.env_rng,
                 elapsed=self.elapsed, ep_ret=self.ep_ret, obs=self.obs)
        if mode == 0:
            d.update(actions=actions, rew=self.c_rew[k], term=self.c_term[k], trunc=self.c_trunc[k],
                     term_obs=self.c_term_obs[k], ep_ret_out=self.c_ep_ret[k], ep_len_out=self.c_ep_len[k])
        return d

    def _step(self, k: int) -> None:
        obs = self.obs
        with th.no_grad():
            a_exp = policy_actions(self.expert, obs, True)
            a_rob = policy_actions(self.learner, obs, False)
        learner_turn = th.rand(self.N, device=self.device) > self._beta
        if not self.discrete:
            learner_turn = learner_turn.reshape((self.N,) + (1,) * len(self.act_shape))
        a_exec = th.where(learner_turn, a_rob.to(a_exp.dtype), a_exp)
        self.c_obs[k].copy_(obs)
        self.c_acts[k].copy_(a_exp.reshape(self.c_acts[k].shape))
        self._C.dagger_env_step(self._env_args(0, k, a_exec.contiguous() if self.discrete else a_exec.float().contiguous()))

    def _run_chunk(self) -> None:
        if not self.use_graph:
            for k in range(self.chunk):
                self._step(k)
            return
        if self._graph is None:
            # the first chunk runs eagerly (also the allocator warm-up); later chunks replay
            for k in range(self.chunk):
                self._step(k)
            g = th.cuda.CUDAGraph()
            try:
                # capture only: nothing in this block executes until replay()
                with th.cuda.graph(g):
                    for k in range(self.chunk):
                        self._step(k)
                self._graph = g
            except RuntimeError as e:  # e.g. an op that syncs: stay eager
                import logging

                logging.getLogger(__name__).warning("DAgger step graph capture failed (%s); stepping eagerly", e)
                self.use_graph = False
            return
        self._graph.replay()

    def reset(self) -> None:
        self._C.dagger_env_step(self._env_args(1))

    # -------------------------------------------------------------- one round
    def collect(self, beta: float, *, min_timesteps: int, min_episodes: int) -> List[types.TrajectoryWithRew]:
        """One round with the reference's ``generate_trajectories`` stopping rule."""
        dev, N, K = self.device, self.N, self.chunk
        self._beta.fill_(float(beta))
        self.reset()
        rec_obs: List[th.Tensor] = []  # per chunk [K, N, ...] copies
        rec_term: List[th.Tensor] = []
        rec_acts: List[th.Tensor] = []
        rec_rew: List[th.Tensor] = []
        active = np.ones(N, dtype=bool)
        start = np.zeros(N, dtype=np.int64)
        finished: List[Tuple[int, int, int]] = []  # (env, first step, last step)
        n_steps_done = 0
        t_base = 0
        satisfied = False
        while active.any():
            self._run_chunk()
            rec_obs.append(self.c_obs.clone())
            rec_term.append(self.c_term_obs.clone())
            rec_acts.append(self.c_acts.clone())
            rec_rew.append(self.c_rew.clone())
            self._host_flags[0].copy_(self.c_term, non_blocking=True)
            self._host_flags[1].copy_(self.c_trunc, non_blocking=True)
            th.cuda.current_stream(dev).synchronize()
            done_chunk = (self._host_flags[0].numpy() | self._host_flags[1].numpy()).astype(bool)
            for k in range(K):
                if not active.any():
                    break
                t = t_base + k
                dones = done_chunk[k] & active
                for n in np.flatnonzero(dones):
                    finished.append((int(n), int(start[n]), t))
                    n_steps_done += t - int(start[n]) + 1
                    start[n] = t + 1
                if not satisfied:
                    satisfied = len(finished) >= min_episodes and n_steps_done >= min_timesteps
                if satisfied:
                    active &= ~dones
            t_base += K
        self.steps_collected = t_base * N
        obs_all = th.cat(rec_obs)  # [T, N, ...]
        term_all = th.cat(rec_term)
        acts_all = th.cat(rec_acts)
        rew_all = th.cat(rec_rew)
        # flat row indices (t * N + n) of every finished episode, in finishing order
        rows = np.concatenate([np.arange(s, e + 1) * N + n for (n, s, e) in finished]) if finished else np.zeros(0, np.int64)
        ends = np.asarray([e * N + n for (n, s, e) in finished], dtype=np.int64)
        ridx = th.as_tensor(rows, device=dev)
        flat = lambda x: x.reshape((-1,) + tuple(x.shape[2:]))  # noqa: E731
        self.last_obs = flat(obs_all).index_select(0, ridx)
        self.last_acts = flat(acts_all).index_select(0, ridx)
        # one D2H copy for the host trajectories (demo files / stats)
        h_obs = self.last_obs.cpu().numpy()
        h_acts = self.last_acts.cpu().numpy()
        h_rew = flat(rew_all).index_select(0, ridx).cpu().numpy()
        h_term = flat(term_all).index_select(0, th.as_tensor(ends, device=dev)).cpu().numpy()
        trajs: List[types.TrajectoryWithRew] = []
        off = 0
        for j, (n, s, e) in enumerate(finished):
            L = e - s + 1
            o = np.concatenate([h_obs[off : off + L], h_term[j : j + 1]])
            trajs.append(types.TrajectoryWithRew(obs=o, acts=h_acts[off : off + L], infos=None, terminal=True,
                                                 rews=h_rew[off : off + L].astype(np.float32)))
            off += L
        self.sync_env_to_host()
        return trajs

    def sync_env_to_host(self) -> None:
        st = {"state": self.state.cpu().numpy(), "rng": self.env_rng.cpu().numpy(),
              "elapsed": self.elapsed.cpu().numpy().astype(np.int64)}
        if self.img:
            st["frames"] = self.obs.cpu().numpy()
        self.nat.set_state(st)

"""Device-resident RL buffers (SB3 ``buffers`` surface).

* :class:`RolloutBuffer` -- on-policy storage ``[n_steps, n_envs, ...]`` kept on
  the training device (SB3 keeps it in host numpy and re-uploads every
  minibatch); GAE runs as one HIP kernel (``imitation_amd.ops.rl.gae``).
* :class:`ReplayBuffer` -- off-policy ring buffer ``[capacity, n_envs, ...]`` on
  the device with uniform with-replacement sampling by device-side index gather
  (SURVEY §2.3 K23). Sized by bytes, it can use a large share of the 288 GB HBM.
"""

from __future__ import annotations

from typing import Any, Dict, Generator, List, NamedTuple, Optional, Union

import numpy as np
import torch as th

from imitation_amd.envs import spaces
from imitation_amd.rl.preprocessing import get_action_dim, get_obs_shape


class RolloutBufferSamples(NamedTuple):
    observations: th.Tensor
    actions: th.Tensor
    old_values: th.Tensor
    old_log_prob: th.Tensor
    advantages: th.Tensor
    returns: th.Tensor


class ReplayBufferSamples(NamedTuple):
    observations: th.Tensor
    actions: th.Tensor
    next_observations: th.Tensor
    dones: th.Tensor
    rewards: th.Tensor


def _torch_dtype(space: spaces.Space):
    if isinstance(space, spaces.Box):
        return th.uint8 if space.dtype == np.uint8 else th.float32
    if isinstance(space, (spaces.Discrete, spaces.MultiDiscrete)):
        return th.int64
    return th.float32


def _to_t(x, device, dtype=None) -> th.Tensor:
    if isinstance(x, th.Tensor):
        return x.to(device=device, dtype=dtype if dtype is not None else x.dtype)
    return th.as_tensor(np.asarray(x), device=device, dtype=dtype)


class BaseBuffer:
    def __init__(self, buffer_size: int, observation_space: spaces.Space, action_space: spaces.Space,
                 device: Union[th.device, str] = "auto", n_envs: int = 1):
        from imitation_amd.rl.policies import get_device

        self.buffer_size = buffer_size
        self.observation_space = observation_space
        self.action_space = action_space
        self.obs_shape = get_obs_shape(observation_space)
        self.action_dim = get_action_dim(action_space)
        self.pos = 0
        self.full = False
        self.device = get_device(device)
        self.n_envs = n_envs

    def size(self) -> int:
        return self.buffer_size if self.full else self.pos

    def reset(self) -> None:
        self.pos = 0
        self.full = False

    def to_torch(self, array, copy: bool = True) -> th.Tensor:
        if isinstance(array, th.Tensor):
            return array.to(self.device)
        return th.tensor(array, device=self.device) if copy else th.as_tensor(array, device=self.device)


class RolloutBuffer(BaseBuffer):
    def __init__(self, buffer_size: int, observation_space: spaces.Space, action_space: spaces.Space,
                 device: Union[th.device, str] = "auto", gae_lambda: float = 1, gamma: float = 0.99, n_envs: int = 1):
        super().__init__(buffer_size, observation_space, action_space, device, n_envs=n_envs)
        self.gae_lambda = gae_lambda
        self.gamma = gamma
        self.generator_ready = False
        self.reset()

    def reset(self) -> None:
        T, N, dev = self.buffer_size, self.n_envs, self.device
        self.observations = th.zeros((T, N, *self.obs_shape), dtype=_torch_dtype(self.observation_space), device=dev)
        act_dtype = th.int64 if isinstance(self.action_space, (spaces.Discrete, spaces.MultiDiscrete)) else th.float32
        self.actions = th.zeros((T, N, self.action_dim), dtype=act_dtype, device=dev)
        self.rewards = th.zeros((T, N), dtype=th.float32, device=dev)
        self.returns = th.zeros((T, N), dtype=th.float32, device=dev)
        self.episode_starts = th.zeros((T, N), dtype=th.float32, device=dev)
        self.values = th.zeros((T, N), dtype=th.float32, device=dev)
        self.log_probs = th.zeros((T, N), dtype=th.float32, device=dev)
        self.advantages = th.zeros((T, N), dtype=th.float32, device=dev)
        self.generator_ready = False
        super().reset()

    def compute_returns_and_advantage(self, last_values: th.Tensor, dones) -> None:
        from imitation_amd.ops import rl as rl_ops

        last_values = last_values.reshape(-1).float().to(self.device)
        dones_t = _to_t(dones, self.device, th.float32).reshape(-1)
        self.advantages, self.returns = rl_ops.gae(
            self.rewards, self.values, self.episode_starts, last_values, dones_t, self.gamma, self.gae_lambda
        )

    def add(self, obs, action, reward, episode_start, value: th.Tensor, log_prob: th.Tensor) -> None:
        if len(log_prob.shape) == 0:
            log_prob = log_prob.reshape(-1, 1)
        if isinstance(self.observation_space, spaces.Discrete):
            obs = _to_t(obs, self.device).reshape((self.n_envs, *self.obs_shape))
        self.observations[self.pos].copy_(_to_t(obs, self.device, self.observations.dtype).reshape(self.observations[self.pos].shape))
        self.actions[self.pos].copy_(_to_t(action, self.device, self.actions.dtype).reshape((self.n_envs, self.action_dim)))
        self.rewards[self.pos].copy_(_to_t(reward, self.device, th.float32).reshape(-1))
        self.episode_starts[self.pos].copy_(_to_t(episode_start, self.device, th.float32).reshape(-1))
        self.values[self.pos].copy_(value.detach().reshape(-1).float())
        self.log_probs[self.pos].copy_(log_prob.detach().reshape(-1).float())
        self.pos += 1
        if self.pos == self.buffer_size:
            self.full = True

    def _flat(self):
        T, N = self.buffer_size, self.n_envs
        return dict(
            observations=self.observations.reshape(T * N, *self.obs_shape),
            actions=self.actions.reshape(T * N, self.action_dim),
            values=self.values.reshape(-1),
            log_probs=self.log_probs.reshape(-1),
            advantages=self.advantages.reshape(-1),
            returns=self.returns.reshape(-1),
        )

    def get(self, batch_size: Optional[int] = None, generator: Optional[th.Generator] = None) -> Generator[RolloutBufferSamples, None, None]:
        assert self.full, ""
        total = self.buffer_size * self.n_envs
        indices = th.randperm(total, device=self.device, generator=generator)
        flat = self._flat()
        if batch_size is None:
            batch_size = total
        start = 0
        while start < total:
            yield self._get_samples(flat, indices[start : start + batch_size])
            start += batch_size

    def _get_samples(self, flat, idx: th.Tensor) -> RolloutBufferSamples:
        acts = flat["actions"][idx]
        if isinstance(self.action_space, spaces.Discrete):
            acts = acts.reshape(-1)
        return RolloutBufferSamples(
            flat["observations"][idx], acts, flat["values"][idx], flat["log_probs"][idx], flat["advantages"][idx], flat["returns"][idx]
        )


class DictRolloutBuffer(RolloutBuffer):
    """:class:`RolloutBuffer` for ``spaces.Dict`` observations (SB3 ``DictRolloutBuffer``): one
    device tensor ``[n_steps, n_envs, *shape]`` per observation key; minibatches carry a dict."""

    def reset(self) -> None:
        T, N, dev = self.buffer_size, self.n_envs, self.device
        self.observations = {k: th.zeros((T, N, *shp), dtype=_torch_dtype(self.observation_space.spaces[k]), device=dev)
                             for k, shp in self.obs_shape.items()}
        act_dtype = th.int64 if isinstance(self.action_space, (spaces.Discrete, spaces.MultiDiscrete)) else th.float32
        self.actions = th.zeros((T, N, self.action_dim), dtype=act_dtype, device=dev)
        for name in ("rewards", "returns", "episode_starts", "values", "log_probs", "advantages"):
            setattr(self, name, th.zeros((T, N), dtype=th.float32, device=dev))
        self.generator_ready = False
        BaseBuffer.reset(self)

    def add(self, obs, action, reward, episode_start, value: th.Tensor, log_prob: th.Tensor) -> None:
        for k, buf in self.observations.items():
            buf[self.pos].copy_(_to_t(obs[k], self.device, buf.dtype).reshape(buf[self.pos].shape))
        if len(log_prob.shape) == 0:
            log_prob = log_prob.reshape(-1, 1)
        self.actions[self.pos].copy_(_to_t(action, self.device, self.actions.dtype).reshape((self.n_envs, self.action_dim)))
        self.rewards[self.pos].copy_(_to_t(reward, self.device, th.float32).reshape(-1))
        self.episode_starts[self.pos].copy_(_to_t(episode_start, self.device, th.float32).reshape(-1))
        self.values[self.pos].copy_(value.detach().reshape(-1).float())
        self.log_probs[self.pos].copy_(log_prob.detach().reshape(-1).float())
        self.pos += 1
        if self.pos == self.buffer_size:
            self.full = True

    def _flat(self):
        T, N = self.buffer_size, self.n_envs
        return dict(
            observations={k: v.reshape(T * N, *v.shape[2:]) for k, v in self.observations.items()},
            actions=self.actions.reshape(T * N, self.action_dim),
            values=self.values.reshape(-1),
            log_probs=self.log_probs.reshape(-1),
            advantages=self.advantages.reshape(-1),
            returns=self.returns.reshape(-1),
        )

    def _get_samples(self, flat, idx: th.Tensor) -> RolloutBufferSamples:
        acts = flat["actions"][idx]
        if isinstance(self.action_space, spaces.Discrete):
            acts = acts.reshape(-1)
        obs = {k: v[idx] for k, v in flat["observations"].items()}
        return RolloutBufferSamples(obs, acts, flat["values"][idx], flat["log_probs"][idx], flat["advantages"][idx],
                                    flat["returns"][idx])


class ReplayBuffer(BaseBuffer):
    """Off-policy ring buffer on the device (SB3 ``ReplayBuffer`` semantics incl. timeout handling)."""

    def __init__(self, buffer_size: int, observation_space: spaces.Space, action_space: spaces.Space,
                 device: Union[th.device, str] = "auto", n_envs: int = 1, optimize_memory_usage: bool = False,
                 handle_timeout_termination: bool = True):
        super().__init__(buffer_size, observation_space, action_space, device, n_envs=n_envs)
        self.buffer_size = max(buffer_size // n_envs, 1)
        self.optimize_memory_usage = optimize_memory_usage
        self.handle_timeout_termination = handle_timeout_termination
        S, N, dev = self.buffer_size, self.n_envs, self.device
        odt = _torch_dtype(observation_space)
        self.observations = th.zeros((S, N, *self.obs_shape), dtype=odt, device=dev)
        self.next_observations = th.zeros((S, N, *self.obs_shape), dtype=odt, device=dev)
        adt = th.int64 if isinstance(action_space, (spaces.Discrete, spaces.MultiDiscrete)) else th.float32
        self.actions = th.zeros((S, N, self.action_dim), dtype=adt, device=dev)
        self.rewards = th.zeros((S, N), dtype=th.float32, device=dev)
        self.dones = th.zeros((S, N), dtype=th.float32, device=dev)
        self.timeouts = th.zeros((S, N), dtype=th.float32, device=dev)

    def add(self, obs, next_obs, action, reward, done, infos: List[Dict[str, Any]]) -> None:
        p = self.pos
        self.observations[p].copy_(_to_t(obs, self.device, self.observations.dtype).reshape(self.observations[p].shape))
        self.next_observations[p].copy_(_to_t(next_obs, self.device, self.next_observations.dtype).reshape(self.observations[p].shape))
        self.actions[p].copy_(_to_t(action, self.device, self.actions.dtype).reshape((self.n_envs, self.action_dim)))
        self.rewards[p].copy_(_to_t(reward, self.device, th.float32).reshape(-1).expand(self.n_envs))
        self.dones[p].copy_(_to_t(done, self.device, th.float32).reshape(-1).expand(self.n_envs))
        if self.handle_timeout_termination:
            self.timeouts[p].copy_(
                th.tensor([float(info.get("TimeLimit.truncated", False)) for info in infos], device=self.device)
            )
        self.pos += 1
        if self.pos == self.buffer_size:
            self.full = True
            self.pos = 0

    def extend(self, obs, next_obs, action, reward, done) -> None:
        """Bulk-append ``n`` single-env transitions (``n_envs == 1``) with one device copy per field."""
        assert self.n_envs == 1
        obs = _to_t(obs, self.device, self.observations.dtype)
        n = obs.shape[0]
        idx = (th.arange(n, device=self.device) + self.pos) % self.buffer_size
        self.observations[idx, 0] = obs.reshape((n, *self.obs_shape))
        self.next_observations[idx, 0] = _to_t(next_obs, self.device, self.next_observations.dtype).reshape((n, *self.obs_shape))
        self.actions[idx, 0] = _to_t(action, self.device, self.actions.dtype).reshape((n, self.action_dim))
        self.rewards[idx, 0] = _to_t(reward, self.device, th.float32).reshape(-1).expand(n)
        self.dones[idx, 0] = _to_t(done, self.device, th.float32).reshape(-1).expand(n)
        self.timeouts[idx, 0] = 0.0
        if self.pos + n >= self.buffer_size:
            self.full = True
        self.pos = (self.pos + n) % self.buffer_size

    def sample(self, batch_size: int, env=None) -> ReplayBufferSamples:
        upper = self.buffer_size if self.full else self.pos
        batch_inds = th.randint(0, upper, (batch_size,), device=self.device)
        return self._get_samples(batch_inds, env=env)

    def _get_samples(self, batch_inds: th.Tensor, env=None) -> ReplayBufferSamples:
        from imitation_amd.ops.rl import gather_rows

        env_inds = th.randint(0, self.n_envs, (len(batch_inds),), device=self.device)
        # every field of the (step, env) rows in one gather launch (csrc/kernels/gather.hip)
        SN = self.buffer_size * self.n_envs
        obs, next_obs, acts, d, tmo, rews = gather_rows(
            [self.observations.view(SN, *self.obs_shape), self.next_observations.view(SN, *self.obs_shape),
             self.actions.view(SN, self.action_dim), self.dones.view(SN), self.timeouts.view(SN), self.rewards.view(SN)],
            batch_inds, env_inds, self.n_envs)
        if env is not None and hasattr(env, "normalize_obs"):
            obs = self.to_torch(env.normalize_obs(obs.cpu().numpy()))
            next_obs = self.to_torch(env.normalize_obs(next_obs.cpu().numpy()))
        dones = (d * (1 - tmo)).reshape(-1, 1)
        rews = rews.reshape(-1, 1)
        if env is not None and hasattr(env, "normalize_reward"):
            rews = self.to_torch(env.normalize_reward(rews.cpu().numpy())).float()
        return ReplayBufferSamples(
            observations=obs.float() if obs.dtype != th.uint8 else obs,
            actions=acts,
            next_observations=next_obs.float() if next_obs.dtype != th.uint8 else next_obs,
            dones=dones,
            rewards=rews,
        )


class DictReplayBuffer(ReplayBuffer):
    """:class:`ReplayBuffer` for ``spaces.Dict`` observations (SB3 ``DictReplayBuffer``): one device
    ring ``[capacity, n_envs, *shape]`` per key for observations and next observations; a sample
    gathers every key's rows together with the other fields (<= 8 tensors per gather launch)."""

    def __init__(self, buffer_size: int, observation_space: spaces.Space, action_space: spaces.Space,
                 device: Union[th.device, str] = "auto", n_envs: int = 1, optimize_memory_usage: bool = False,
                 handle_timeout_termination: bool = True):
        assert not optimize_memory_usage, "DictReplayBuffer does not support optimize_memory_usage"
        BaseBuffer.__init__(self, buffer_size, observation_space, action_space, device, n_envs=n_envs)
        self.buffer_size = max(buffer_size // n_envs, 1)
        self.optimize_memory_usage = False
        self.handle_timeout_termination = handle_timeout_termination
        S, N, dev = self.buffer_size, self.n_envs, self.device

        def rings():
            return {k: th.zeros((S, N, *shp), dtype=_torch_dtype(observation_space.spaces[k]), device=dev)
                    for k, shp in self.obs_shape.items()}

        self.observations = rings()
        self.next_observations = rings()
        adt = th.int64 if isinstance(action_space, (spaces.Discrete, spaces.MultiDiscrete)) else th.float32
        self.actions = th.zeros((S, N, self.action_dim), dtype=adt, device=dev)
        self.rewards = th.zeros((S, N), dtype=th.float32, device=dev)
        self.dones = th.zeros((S, N), dtype=th.float32, device=dev)
        self.timeouts = th.zeros((S, N), dtype=th.float32, device=dev)

    def add(self, obs, next_obs, action, reward, done, infos: List[Dict[str, Any]]) -> None:
        p = self.pos
        for k, ring in self.observations.items():
            ring[p].copy_(_to_t(obs[k], self.device, ring.dtype).reshape(ring[p].shape))
        for k, ring in self.next_observations.items():
            ring[p].copy_(_to_t(next_obs[k], self.device, ring.dtype).reshape(ring[p].shape))
        self.actions[p].copy_(_to_t(action, self.device, self.actions.dtype).reshape((self.n_envs, self.action_dim)))
        self.rewards[p].copy_(_to_t(reward, self.device, th.float32).reshape(-1).expand(self.n_envs))
        self.dones[p].copy_(_to_t(done, self.device, th.float32).reshape(-1).expand(self.n_envs))
        if self.handle_timeout_termination:
            self.timeouts[p].copy_(
                th.tensor([float(info.get("TimeLimit.truncated", False)) for info in infos], device=self.device)
            )
        self.pos += 1
        if self.pos == self.buffer_size:
            self.full = True
            self.pos = 0

    def extend(self, obs, next_obs, action, reward, done) -> None:
        """Bulk-append ``n`` single-env transitions (``n_envs == 1``); ``obs`` / ``next_obs`` map keys to ``[n, ...]``."""
        assert self.n_envs == 1
        n_all = len(next(iter(obs.values())))
        # FIFO: only the newest ``buffer_size`` rows survive; scattering more than that would
        # repeat ring indices, and which duplicate write wins in an index_put is unspecified
        n = min(n_all, self.buffer_size)
        skip = n_all - n
        start = (self.pos + skip) % self.buffer_size
        idx = (th.arange(n, device=self.device) + start) % self.buffer_size

        def tail(x, dtype, shape):
            t = _to_t(x, self.device, dtype)
            t = t.reshape(-1).expand(n_all) if shape is None else t.reshape((n_all, *shape))
            return t[skip:]

        for src, rings in ((obs, self.observations), (next_obs, self.next_observations)):
            for k, ring in rings.items():
                ring[idx, 0] = tail(src[k], ring.dtype, self.obs_shape[k])
        self.actions[idx, 0] = tail(action, self.actions.dtype, (self.action_dim,))
        self.rewards[idx, 0] = tail(reward, th.float32, None)
        self.dones[idx, 0] = tail(done, th.float32, None)
        self.timeouts[idx, 0] = 0.0
        if self.pos + n_all >= self.buffer_size:
            self.full = True
        self.pos = (self.pos + n_all) % self.buffer_size

    def _get_samples(self, batch_inds: th.Tensor, env=None) -> ReplayBufferSamples:
        from imitation_amd.ops.rl import gather_rows

        env_inds = th.randint(0, self.n_envs, (len(batch_inds),), device=self.device)
        SN = self.buffer_size * self.n_envs
        keys = list(self.observations)
        srcs = [self.observations[k].view(SN, *self.obs_shape[k]) for k in keys]
        srcs += [self.next_observations[k].view(SN, *self.obs_shape[k]) for k in keys]
        srcs += [self.actions.view(SN, self.action_dim), self.dones.view(SN), self.timeouts.view(SN), self.rewards.view(SN)]
        out: List[th.Tensor] = []
        for i in range(0, len(srcs), 8):
            out += list(gather_rows(srcs[i : i + 8], batch_inds, env_inds, self.n_envs))
        nk = len(keys)
        obs = dict(zip(keys, out[:nk]))
        next_obs = dict(zip(keys, out[nk : 2 * nk]))
        acts, d, tmo, rews = out[2 * nk :]
        if env is not None and hasattr(env, "normalize_obs"):
            obs = {k: self.to_torch(v) for k, v in env.normalize_obs({k: v.cpu().numpy() for k, v in obs.items()}).items()}
            next_obs = {k: self.to_torch(v) for k, v in
                        env.normalize_obs({k: v.cpu().numpy() for k, v in next_obs.items()}).items()}
        rews = rews.reshape(-1, 1)
        if env is not None and hasattr(env, "normalize_reward"):
            rews = self.to_torch(env.normalize_reward(rews.cpu().numpy())).float()
        as_f = lambda t: t.float() if t.dtype != th.uint8 else t  # noqa: E731
        return ReplayBufferSamples(
            observations={k: as_f(v) for k, v in obs.items()},
            actions=acts,
            next_observations={k: as_f(v) for k, v in next_obs.items()},
            dones=(d * (1 - tmo)).reshape(-1, 1),
            rewards=rews,
        )

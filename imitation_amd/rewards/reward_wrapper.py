"""Env wrapper that substitutes a learned reward (reference: ``src/imitation/rewards/reward_wrapper.py``).

:class:`RewardVecEnvWrapper` (``reward_wrapper.py:40-133``) replaces the env
reward with ``reward_fn(obs, acts, next_obs, dones)``, using
``info["terminal_observation"]`` as ``next_obs`` on episode ends, keeps the
env's own reward in ``info["original_env_rew"]`` and tracks wrapped episode
returns for :class:`WrappedRewardCallback` (``rollout/ep_rew_wrapped_mean``).
"""

from __future__ import annotations

import collections
from typing import Deque

import numpy as np

from imitation_amd.data import types
from imitation_amd.envs.vec_env import VecEnv, VecEnvWrapper
from imitation_amd.rl.callbacks import BaseCallback


class WrappedRewardCallback(BaseCallback):
    """Logs the mean wrapped-reward episode return at every rollout start."""

    def __init__(self, episode_rewards: Deque[float], *args, **kwargs):
        self.episode_rewards = episode_rewards
        super().__init__(*args, **kwargs)

    def _on_step(self) -> bool:
        return True

    def _on_rollout_start(self) -> None:
        if len(self.episode_rewards) == 0:
            return
        self.logger.record("rollout/ep_rew_wrapped_mean", sum(self.episode_rewards) / len(self.episode_rewards))


class RewardVecEnvWrapper(VecEnvWrapper):
    """Replace ``step()`` rewards with ``reward_fn``; resets the inner VecEnv on construction."""

    def __init__(self, venv: VecEnv, reward_fn, ep_history: int = 100):
        assert not isinstance(venv, RewardVecEnvWrapper)
        super().__init__(venv)
        self.episode_rewards: Deque = collections.deque(maxlen=ep_history)
        self._cumulative_rew = np.zeros((venv.num_envs,))
        self.reward_fn = reward_fn
        self._old_obs = None
        self._actions = None
        self.reset()

    def make_log_callback(self) -> WrappedRewardCallback:
        return WrappedRewardCallback(self.episode_rewards)

    @property
    def envs(self):
        return self.venv.envs

    def reset(self):
        self._old_obs = self.venv.reset()
        return self._old_obs

    def step_async(self, actions):
        self._actions = actions
        return self.venv.step_async(actions)

    def step_wait(self):
        obs, old_rews, dones, infos = self.venv.step_wait()
        wrapped = types.maybe_wrap_in_dictobs(obs)
        if isinstance(wrapped, types.DictObs):
            fixed = [types.maybe_wrap_in_dictobs(infos[i]["terminal_observation"]) if d else o
                     for i, (o, d) in enumerate(zip(wrapped, dones))]
            obs_fixed = types.maybe_unwrap_dictobs(types.DictObs.stack(fixed))
        else:
            obs_fixed = np.array(obs, copy=True)
            for i in np.flatnonzero(dones):
                obs_fixed[i] = infos[i]["terminal_observation"]
        rews = self.reward_fn(self._old_obs, self._actions, obs_fixed, np.array(dones))
        assert len(rews) == len(obs), "must return one rew for each env"
        done_mask = np.asarray(dones, dtype="bool").reshape((len(dones),))
        self._cumulative_rew += rews
        for d, ep_rew in zip(dones, self._cumulative_rew):
            if d:
                self.episode_rewards.append(ep_rew)
        self._cumulative_rew[done_mask] = 0
        self._old_obs = obs
        for info, old_rew in zip(infos, old_rews):
            info["original_env_rew"] = old_rew
        return obs, rews, dones, infos

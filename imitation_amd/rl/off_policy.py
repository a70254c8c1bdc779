"""Off-policy algorithm base (SAC / DQN; SB3 ``OffPolicyAlgorithm`` semantics).

Transitions go into a device-resident :class:`~imitation_amd.rl.buffers.ReplayBuffer`;
``train_freq`` / ``gradient_steps`` / ``learning_starts`` / Polyak ``tau`` follow SB3.
"""

from __future__ import annotations

from typing import Any, Dict, NamedTuple, Optional, Tuple, Type, Union

import numpy as np
import torch as th

from imitation_amd.envs import spaces
from imitation_amd.parallel import dist as pdist
from imitation_amd.rl.base import BaseAlgorithm
from imitation_amd.rl.buffers import DictReplayBuffer, ReplayBuffer
from imitation_amd.rl.callbacks import BaseCallback


class RolloutReturn(NamedTuple):
    episode_timesteps: int
    n_episodes: int
    continue_training: bool


class TrainFreq(NamedTuple):
    frequency: int
    unit: str  # "step" | "episode"


def polyak_update(params, target_params, tau: float) -> None:
    with th.no_grad():
        ps = list(params)
        ts = list(target_params)
        if ps:
            th._foreach_mul_(ts, 1 - tau)
            th._foreach_add_(ts, ps, alpha=tau)


class OffPolicyAlgorithm(BaseAlgorithm):
    def __init__(self, policy, env, learning_rate, buffer_size: int = 1_000_000, learning_starts: int = 100,
                 batch_size: int = 256, tau: float = 0.005, gamma: float = 0.99,
                 train_freq: Union[int, Tuple[int, str]] = (1, "step"), gradient_steps: int = 1, action_noise=None,
                 replay_buffer_class: Optional[Type] = None, replay_buffer_kwargs: Optional[Dict[str, Any]] = None,
                 optimize_memory_usage: bool = False, policy_kwargs=None, stats_window_size: int = 100,
                 tensorboard_log=None, verbose: int = 0, device="auto", support_multi_env: bool = True,
                 monitor_wrapper: bool = True, seed=None, use_sde: bool = False, sde_sample_freq: int = -1,
                 use_sde_at_warmup: bool = False, sde_support: bool = True, supported_action_spaces=None):
        super().__init__(policy=policy, env=env, learning_rate=learning_rate, policy_kwargs=policy_kwargs,
                         stats_window_size=stats_window_size, tensorboard_log=tensorboard_log, verbose=verbose,
                         device=device, support_multi_env=support_multi_env, monitor_wrapper=monitor_wrapper,
                         seed=seed, use_sde=use_sde, sde_sample_freq=sde_sample_freq,
                         supported_action_spaces=supported_action_spaces)
        self.buffer_size = buffer_size
        self.batch_size = batch_size
        self.learning_starts = learning_starts
        self.tau = tau
        self.gamma = gamma
        self.gradient_steps = gradient_steps
        self.action_noise = action_noise
        self.optimize_memory_usage = optimize_memory_usage
        self.replay_buffer: Optional[ReplayBuffer] = None
        self.replay_buffer_class = replay_buffer_class
        self.replay_buffer_kwargs = replay_buffer_kwargs or {}
        self.train_freq = train_freq
        self.use_sde_at_warmup = use_sde_at_warmup

    def _convert_train_freq(self) -> None:
        if not isinstance(self.train_freq, TrainFreq):
            tf = self.train_freq
            if not isinstance(tf, tuple):
                tf = (tf, "step")
            self.train_freq = TrainFreq(int(tf[0]), str(tf[1]))

    def _setup_model(self) -> None:
        self._setup_lr_schedule()
        self.set_random_seed(self.seed)
        if self.replay_buffer_class is None:
            self.replay_buffer_class = DictReplayBuffer if isinstance(self.observation_space, spaces.Dict) else ReplayBuffer
        if self.replay_buffer is None:
            kwargs = dict(self.replay_buffer_kwargs)
            self.replay_buffer = self.replay_buffer_class(self.buffer_size, self.observation_space, self.action_space,
                                                          device=self.device, n_envs=self.n_envs,
                                                          optimize_memory_usage=self.optimize_memory_usage, **kwargs)
        self.policy = self.policy_class(self.observation_space, self.action_space, self.lr_schedule, **self.policy_kwargs)
        self.policy = self.policy.to(self.device)
        pdist.broadcast_module(self.policy)
        self._convert_train_freq()

    def _sample_action(self, learning_starts: int, action_noise=None, n_envs: int = 1) -> Tuple[np.ndarray, np.ndarray]:
        if self.num_timesteps < learning_starts and not (self.use_sde and self.use_sde_at_warmup):
            unscaled_action = np.array([self.action_space.sample() for _ in range(n_envs)])
        else:
            unscaled_action, _ = self.predict(self._last_obs, deterministic=False)
        if isinstance(self.action_space, spaces.Box):
            scaled_action = self.policy.scale_action(unscaled_action)
            if action_noise is not None:
                scaled_action = np.clip(scaled_action + action_noise(), -1, 1)
            buffer_action = scaled_action
            action = self.policy.unscale_action(scaled_action)
        else:
            buffer_action = unscaled_action
            action = buffer_action
        return action, buffer_action

    def _store_transition(self, replay_buffer: ReplayBuffer, buffer_action, new_obs, reward, dones, infos) -> None:
        if self._vec_normalize_env is not None:
            new_obs_ = self._vec_normalize_env.get_original_obs()
            reward_ = self._vec_normalize_env.get_original_reward()
        else:
            self._last_original_obs, new_obs_, reward_ = self._last_obs, new_obs, reward
        if isinstance(new_obs_, dict):  # Dict observation spaces: one array per key
            next_obs = {k: np.array(v, copy=True) for k, v in new_obs_.items()}
            for i, done in enumerate(dones):
                if done and infos[i].get("terminal_observation") is not None:
                    for k in next_obs:
                        next_obs[k][i] = infos[i]["terminal_observation"][k]
        else:
            next_obs = np.array(new_obs_, copy=True)
            for i, done in enumerate(dones):
                if done and infos[i].get("terminal_observation") is not None:
                    next_obs[i] = infos[i]["terminal_observation"]
        replay_buffer.add(self._last_original_obs, next_obs, buffer_action, reward_, dones, infos)
        self._last_obs = new_obs
        if self._vec_normalize_env is not None:
            self._last_original_obs = new_obs_

    def _on_step(self) -> None:
        pass

    def collect_rollouts(self, env, callback: BaseCallback, train_freq: TrainFreq, replay_buffer: ReplayBuffer,
                         action_noise=None, learning_starts: int = 0, log_interval: Optional[int] = None) -> RolloutReturn:
        self.policy.set_training_mode(False)
        num_collected_steps, num_collected_episodes = 0, 0
        callback.on_rollout_start()
        continue_training = True

        def should_collect() -> bool:
            if train_freq.unit == "step":
                return num_collected_steps < train_freq.frequency
            return num_collected_episodes < train_freq.frequency

        while should_collect():
            actions, buffer_actions = self._sample_action(learning_starts, action_noise, env.num_envs)
            new_obs, rewards, dones, infos = env.step(actions)
            self.num_timesteps += env.num_envs
            num_collected_steps += 1
            callback.update_locals(locals())
            if not callback.on_step():
                return RolloutReturn(num_collected_steps * env.num_envs, num_collected_episodes, continue_training=False)
            self._update_info_buffer(infos, dones)
            self._store_transition(replay_buffer, buffer_actions, new_obs, rewards, dones, infos)
            self._update_current_progress_remaining(self.num_timesteps, self._total_timesteps)
            self._on_step()
            for idx, done in enumerate(dones):
                if done:
                    num_collected_episodes += 1
                    self._episode_num += 1
                    if action_noise is not None and hasattr(action_noise, "reset"):
                        # only the finished env's noise process (SB3: indices=[idx] when n_envs > 1)
                        action_noise.reset(**({"indices": [idx]} if env.num_envs > 1 else {}))
                    if log_interval is not None and self._episode_num % log_interval == 0:
                        self._dump_logs()
        callback.on_rollout_end()
        return RolloutReturn(num_collected_steps * env.num_envs, num_collected_episodes, continue_training)

    def _dump_logs(self) -> None:
        self.logger.record("time/episodes", self._episode_num, exclude="tensorboard")
        self._dump_logs_common()
        self.logger.dump(step=self.num_timesteps)

    def train(self, gradient_steps: int, batch_size: int) -> None:
        raise NotImplementedError

    def learn(self, total_timesteps: int, callback=None, log_interval: int = 4, tb_log_name: str = "run",
              reset_num_timesteps: bool = True, progress_bar: bool = False):
        total_timesteps, callback = self._setup_learn(total_timesteps, callback, reset_num_timesteps, tb_log_name, progress_bar)
        callback.on_training_start(locals(), globals())
        assert self.env is not None
        while self.num_timesteps < total_timesteps:
            rollout = self.collect_rollouts(self.env, train_freq=self.train_freq, action_noise=self.action_noise,
                                            callback=callback, learning_starts=self.learning_starts,
                                            replay_buffer=self.replay_buffer, log_interval=log_interval)
            if not rollout.continue_training:
                break
            if self.num_timesteps > 0 and self.num_timesteps > self.learning_starts:
                gradient_steps = self.gradient_steps if self.gradient_steps >= 0 else rollout.episode_timesteps
                if gradient_steps > 0:
                    self.train(batch_size=self.batch_size, gradient_steps=gradient_steps)
        callback.on_training_end()
        return self

    def _post_load_init(self, data):
        for k in ("buffer_size", "batch_size", "learning_starts", "tau", "gamma", "gradient_steps"):
            if data.get(k) is not None:
                setattr(self, k, data[k])
        tf = data.get("train_freq")
        self.train_freq = tuple(tf) if isinstance(tf, list) else (tf or (1, "step"))
        self.replay_buffer = None
        self.replay_buffer_class = None
        self.replay_buffer_kwargs = {}
        self.optimize_memory_usage = False
        self.action_noise = None
        self.use_sde_at_warmup = False

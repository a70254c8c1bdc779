"""DQN -- the SQIL default learner (``src/imitation/algorithms/sqil.py:42``;
``scripts/ingredients/sqil.py:32-33``). SB3 semantics: Q-network MLP ([64, 64] by
default), target network synced every ``target_update_interval`` env steps,
ε-greedy with a linear exploration schedule, Huber loss, gradient clipping; the
replay buffer is device resident and DP averages the Q gradients per step."""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple, Type, Union

import numpy as np
import torch as th
from torch import nn
from torch.nn import functional as F

from imitation_amd.envs import spaces
from imitation_amd.parallel import dist as pdist
from imitation_amd.rl.off_policy import OffPolicyAlgorithm, polyak_update
from imitation_amd.rl.policies import BasePolicy, get_schedule_fn
from imitation_amd.rl.torch_layers import BaseFeaturesExtractor, CombinedExtractor, FlattenExtractor, NatureCNN, create_mlp


def get_linear_fn(start: float, end: float, end_fraction: float):
    def func(progress_remaining: float) -> float:
        if (1 - progress_remaining) > end_fraction:
            return end
        return start + (1 - progress_remaining) * (end - start) / end_fraction

    return func


class QNetwork(BasePolicy):
    def __init__(self, observation_space, action_space, features_extractor: BaseFeaturesExtractor, features_dim: int,
                 net_arch: Optional[List[int]] = None, activation_fn: Type[nn.Module] = nn.ReLU, normalize_images: bool = True):
        super().__init__(observation_space, action_space, features_extractor=features_extractor, normalize_images=normalize_images)
        if net_arch is None:
            net_arch = [64, 64]
        self.net_arch = net_arch
        self.activation_fn = activation_fn
        self.features_dim = features_dim
        action_dim = int(self.action_space.n)
        self.q_net = nn.Sequential(*create_mlp(self.features_dim, action_dim, self.net_arch, self.activation_fn))

    def forward(self, obs) -> th.Tensor:
        return self.q_net(self.extract_features(obs, self.features_extractor))

    def _predict(self, observation, deterministic: bool = True) -> th.Tensor:
        return self(observation).argmax(dim=1).reshape(-1)


class DQNPolicy(BasePolicy):
    def __init__(self, observation_space, action_space, lr_schedule, net_arch: Optional[List[int]] = None,
                 activation_fn: Type[nn.Module] = nn.ReLU, features_extractor_class=FlattenExtractor,
                 features_extractor_kwargs: Optional[Dict[str, Any]] = None, normalize_images: bool = True,
                 optimizer_class: Type[th.optim.Optimizer] = th.optim.Adam, optimizer_kwargs: Optional[Dict[str, Any]] = None):
        super().__init__(observation_space, action_space, features_extractor_class, features_extractor_kwargs,
                         optimizer_class=optimizer_class, optimizer_kwargs=optimizer_kwargs, normalize_images=normalize_images)
        if net_arch is None:
            net_arch = [] if features_extractor_class == NatureCNN else [64, 64]
        self.net_arch = net_arch
        self.activation_fn = activation_fn
        self._build(lr_schedule)

    def make_q_net(self) -> QNetwork:
        fe = self.make_features_extractor()
        return QNetwork(self.observation_space, self.action_space, fe, fe.features_dim, self.net_arch, self.activation_fn,
                        self.normalize_images)

    def _build(self, lr_schedule) -> None:
        self.q_net = self.make_q_net()
        self.q_net_target = self.make_q_net()
        self.q_net_target.load_state_dict(self.q_net.state_dict())
        self.q_net_target.set_training_mode(False)
        self.optimizer = self.optimizer_class(self.q_net.parameters(), lr=lr_schedule(1), **self.optimizer_kwargs)

    def forward(self, obs, deterministic: bool = True) -> th.Tensor:
        return self._predict(obs, deterministic=deterministic)

    def _predict(self, obs, deterministic: bool = True) -> th.Tensor:
        return self.q_net._predict(obs, deterministic=deterministic)

    def set_training_mode(self, mode: bool) -> None:
        self.q_net.set_training_mode(mode)
        self.training = mode


MlpPolicy = DQNPolicy


class CnnPolicy(DQNPolicy):
    def __init__(self, *args, features_extractor_class=NatureCNN, **kwargs):
        super().__init__(*args, features_extractor_class=features_extractor_class, **kwargs)


class MultiInputPolicy(DQNPolicy):
    """Q-network over ``spaces.Dict`` observations (per-key features concatenated)."""

    def __init__(self, *args, features_extractor_class=CombinedExtractor, **kwargs):
        super().__init__(*args, features_extractor_class=features_extractor_class, **kwargs)


class DQN(OffPolicyAlgorithm):
    policy_aliases = {"MlpPolicy": DQNPolicy, "CnnPolicy": CnnPolicy, "MultiInputPolicy": MultiInputPolicy}

    def __init__(self, policy, env, learning_rate=1e-4, buffer_size: int = 1_000_000, learning_starts: int = 100,
                 batch_size: int = 32, tau: float = 1.0, gamma: float = 0.99, train_freq=4, gradient_steps: int = 1,
                 replay_buffer_class=None, replay_buffer_kwargs=None, optimize_memory_usage: bool = False,
                 target_update_interval: int = 10000, exploration_fraction: float = 0.1,
                 exploration_initial_eps: float = 1.0, exploration_final_eps: float = 0.05, max_grad_norm: float = 10,
                 stats_window_size: int = 100, tensorboard_log=None, policy_kwargs=None, verbose: int = 0, seed=None,
                 device="auto", _init_setup_model: bool = True):
        super().__init__(policy, env, learning_rate, buffer_size, learning_starts, batch_size, tau, gamma, train_freq,
                         gradient_steps, action_noise=None, replay_buffer_class=replay_buffer_class,
                         replay_buffer_kwargs=replay_buffer_kwargs, policy_kwargs=policy_kwargs,
                         stats_window_size=stats_window_size, tensorboard_log=tensorboard_log, verbose=verbose,
                         device=device, seed=seed, sde_support=False, optimize_memory_usage=optimize_memory_usage,
                         supported_action_spaces=(spaces.Discrete,))
        self.exploration_initial_eps = exploration_initial_eps
        self.exploration_final_eps = exploration_final_eps
        self.exploration_fraction = exploration_fraction
        self.target_update_interval = target_update_interval
        self._n_calls = 0
        self.max_grad_norm = max_grad_norm
        self.exploration_rate = 0.0
        if _init_setup_model:
            self._setup_model()

    def _setup_model(self) -> None:
        super()._setup_model()
        self.q_net = self.policy.q_net
        self.q_net_target = self.policy.q_net_target
        self.exploration_schedule = get_linear_fn(self.exploration_initial_eps, self.exploration_final_eps, self.exploration_fraction)
        if self.n_envs > 1 and self.n_envs > self.target_update_interval:
            self.target_update_interval = max(self.target_update_interval // self.n_envs, 1)
        self._q_bucket = pdist.GradBucket(self.q_net.parameters()) if pdist.world_size() > 1 else None

    def _on_step(self) -> None:
        self._n_calls += 1
        if self._n_calls % max(self.target_update_interval // self.n_envs, 1) == 0:
            polyak_update(self.q_net.parameters(), self.q_net_target.parameters(), self.tau)
            polyak_update(list(self.q_net.buffers()), list(self.q_net_target.buffers()), 1.0)
        self.exploration_rate = self.exploration_schedule(self._current_progress_remaining)
        self.logger.record("rollout/exploration_rate", self.exploration_rate)

    def train(self, gradient_steps: int, batch_size: int = 100) -> None:
        self.policy.set_training_mode(True)
        self._update_learning_rate(self.policy.optimizer)
        losses = []
        for _ in range(gradient_steps):
            rd = self.replay_buffer.sample(batch_size, env=self._vec_normalize_env)
            with th.no_grad():
                next_q = self.q_net_target(rd.next_observations).max(dim=1).values.reshape(-1, 1)
                target_q = rd.rewards + (1 - rd.dones) * self.gamma * next_q
            current_q = th.gather(self.q_net(rd.observations), dim=1, index=rd.actions.long().reshape(-1, 1))
            loss = F.smooth_l1_loss(current_q, target_q)
            losses.append(loss.detach())
            self.policy.optimizer.zero_grad()
            loss.backward()
            if self._q_bucket is not None:
                pdist.allreduce_grads(self._q_bucket.params)
            th.nn.utils.clip_grad_norm_(self.policy.parameters(), self.max_grad_norm)
            self.policy.optimizer.step()
        self._n_updates += gradient_steps
        self.logger.record("train/n_updates", self._n_updates, exclude="tensorboard")
        self.logger.record("train/loss", float(th.stack(losses).mean()))

    def predict(self, observation, state=None, episode_start=None, deterministic: bool = False):
        if not deterministic and np.random.rand() < self.exploration_rate:
            if self.policy.is_vectorized_observation(observation):
                n_batch = observation[next(iter(observation))].shape[0] if isinstance(observation, dict) else observation.shape[0]
                action = np.array([self.action_space.sample() for _ in range(n_batch)])
            else:
                action = np.array(self.action_space.sample())
            return action, state
        return self.policy.predict(observation, state, episode_start, deterministic)

    def learn(self, total_timesteps: int, callback=None, log_interval: int = 4, tb_log_name: str = "DQN",
              reset_num_timesteps: bool = True, progress_bar: bool = False):
        return super().learn(total_timesteps=total_timesteps, callback=callback, log_interval=log_interval,
                             tb_log_name=tb_log_name, reset_num_timesteps=reset_num_timesteps, progress_bar=progress_bar)

    def _excluded_save_params(self):
        return super()._excluded_save_params() | {"q_net", "q_net_target", "_q_bucket", "exploration_schedule"}

"""Soft Actor-Critic (the reference's ``rl.sac`` named config and GAIL+SAC GPU test;
``scripts/ingredients/rl.py:83-98``, ``tests/algorithms/test_adversarial.py:438-466``).

SB3-equivalent: tanh-squashed Gaussian actor (``get_action_dist_params``,
``action_log_prob``), twin Q critics with Polyak target, automatic entropy
coefficient (``ent_coef="auto"``), target entropy ``-|A|``. Each update is one
actor + one critic optimizer step; under DP each step's gradients are averaged
with one bucketed all-reduce.
"""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple, Type, Union

import numpy as np
import torch as th
from torch import nn
from torch.nn import functional as F

from imitation_amd.envs import spaces
from imitation_amd.parallel import dist as pdist
from imitation_amd.rl.distributions import SquashedDiagGaussianDistribution
from imitation_amd.rl.off_policy import OffPolicyAlgorithm, polyak_update
from imitation_amd.rl.policies import BasePolicy, get_schedule_fn
from imitation_amd.rl.preprocessing import get_action_dim
from imitation_amd.rl.torch_layers import (BaseFeaturesExtractor, CombinedExtractor, FlattenExtractor, NatureCNN, create_mlp,
                                           get_actor_critic_arch)

LOG_STD_MAX = 2
LOG_STD_MIN = -20


class Actor(BasePolicy):
    def __init__(self, observation_space, action_space, net_arch: List[int], features_extractor: nn.Module, features_dim: int,
                 activation_fn: Type[nn.Module] = nn.ReLU, use_sde: bool = False, log_std_init: float = -3,
                 full_std: bool = True, use_expln: bool = False, clip_mean: float = 2.0, normalize_images: bool = True):
        super().__init__(observation_space, action_space, features_extractor=features_extractor, normalize_images=normalize_images,
                         squash_output=True)
        self.net_arch = net_arch
        self.features_dim = features_dim
        self.activation_fn = activation_fn
        action_dim = get_action_dim(self.action_space)
        latent_pi_net = create_mlp(features_dim, -1, net_arch, activation_fn)
        self.latent_pi = nn.Sequential(*latent_pi_net)
        last = net_arch[-1] if len(net_arch) > 0 else features_dim
        self.action_dist = SquashedDiagGaussianDistribution(action_dim)
        self.mu = nn.Linear(last, action_dim)
        self.log_std = nn.Linear(last, action_dim)

    def get_action_dist_params(self, obs) -> Tuple[th.Tensor, th.Tensor, Dict[str, th.Tensor]]:
        features = self.extract_features(obs, self.features_extractor)
        latent_pi = self.latent_pi(features)
        mean_actions = self.mu(latent_pi)
        log_std = th.clamp(self.log_std(latent_pi), LOG_STD_MIN, LOG_STD_MAX)
        return mean_actions, log_std, {}

    def forward(self, obs, deterministic: bool = False) -> th.Tensor:
        mean_actions, log_std, kwargs = self.get_action_dist_params(obs)
        return self.action_dist.actions_from_params(mean_actions, log_std, deterministic=deterministic, **kwargs)

    def action_log_prob(self, obs) -> Tuple[th.Tensor, th.Tensor]:
        mean_actions, log_std, kwargs = self.get_action_dist_params(obs)
        return self.action_dist.log_prob_from_params(mean_actions, log_std, **kwargs)

    def _predict(self, observation, deterministic: bool = False) -> th.Tensor:
        return self(observation, deterministic)


class ContinuousCritic(BasePolicy):
    def __init__(self, observation_space, action_space, net_arch: List[int], features_extractor: nn.Module, features_dim: int,
                 activation_fn: Type[nn.Module] = nn.ReLU, normalize_images: bool = True, n_critics: int = 2,
                 share_features_extractor: bool = True):
        super().__init__(observation_space, action_space, features_extractor=features_extractor, normalize_images=normalize_images)
        action_dim = get_action_dim(self.action_space)
        self.share_features_extractor = share_features_extractor
        self.n_critics = n_critics
        self.q_networks: List[nn.Module] = []
        for idx in range(n_critics):
            q_net = nn.Sequential(*create_mlp(features_dim + action_dim, 1, net_arch, activation_fn))
            self.add_module(f"qf{idx}", q_net)
            self.q_networks.append(q_net)

    def forward(self, obs, actions: th.Tensor) -> Tuple[th.Tensor, ...]:
        with th.set_grad_enabled(not self.share_features_extractor):
            features = self.extract_features(obs, self.features_extractor)
        qvalue_input = th.cat([features, actions], dim=1)
        return tuple(q(qvalue_input) for q in self.q_networks)

    def q1_forward(self, obs, actions: th.Tensor) -> th.Tensor:
        with th.no_grad():
            features = self.extract_features(obs, self.features_extractor)
        return self.q_networks[0](th.cat([features, actions], dim=1))


class SACPolicy(BasePolicy):
    def __init__(self, observation_space, action_space, lr_schedule, net_arch=None, activation_fn: Type[nn.Module] = nn.ReLU,
                 use_sde: bool = False, log_std_init: float = -3, use_expln: bool = False, clip_mean: float = 2.0,
                 features_extractor_class: Type[BaseFeaturesExtractor] = FlattenExtractor,
                 features_extractor_kwargs=None, normalize_images: bool = True,
                 optimizer_class: Type[th.optim.Optimizer] = th.optim.Adam, optimizer_kwargs=None, n_critics: int = 2,
                 share_features_extractor: bool = False):
        super().__init__(observation_space, action_space, features_extractor_class, features_extractor_kwargs,
                         optimizer_class=optimizer_class, optimizer_kwargs=optimizer_kwargs, squash_output=True,
                         normalize_images=normalize_images)
        if net_arch is None:
            net_arch = [256, 256]
        actor_arch, critic_arch = get_actor_critic_arch(net_arch)
        self.net_arch = net_arch
        self.activation_fn = activation_fn
        self.actor_kwargs = dict(observation_space=observation_space, action_space=action_space, net_arch=actor_arch,
                                 activation_fn=activation_fn, normalize_images=normalize_images)
        self.critic_kwargs = dict(self.actor_kwargs)
        self.critic_kwargs.update(n_critics=n_critics, net_arch=critic_arch, share_features_extractor=share_features_extractor)
        self.share_features_extractor = share_features_extractor
        self._lr_schedule = lr_schedule
        self._build(lr_schedule)

    def _build(self, lr_schedule) -> None:
        self.actor = self.make_actor()
        self.actor.optimizer = self.optimizer_class(self.actor.parameters(), lr=lr_schedule(1), **self.optimizer_kwargs)
        if self.share_features_extractor:
            self.critic = self.make_critic(features_extractor=self.actor.features_extractor)
            critic_parameters = [p for n, p in self.critic.named_parameters() if "features_extractor" not in n]
        else:
            self.critic = self.make_critic(features_extractor=None)
            critic_parameters = list(self.critic.parameters())
        self.critic_target = self.make_critic(features_extractor=None)
        self.critic_target.load_state_dict(self.critic.state_dict())
        self.critic.optimizer = self.optimizer_class(critic_parameters, lr=lr_schedule(1), **self.optimizer_kwargs)
        self.critic_target.set_training_mode(False)

    def make_actor(self, features_extractor=None) -> Actor:
        fe = features_extractor or self.make_features_extractor()
        return Actor(features_extractor=fe, features_dim=fe.features_dim, **self.actor_kwargs)

    def make_critic(self, features_extractor=None) -> ContinuousCritic:
        fe = features_extractor or self.make_features_extractor()
        return ContinuousCritic(features_extractor=fe, features_dim=fe.features_dim, **self.critic_kwargs)

    def _get_constructor_parameters(self) -> Dict[str, Any]:
        data = super()._get_constructor_parameters()
        data.update(dict(net_arch=self.net_arch, activation_fn=self.activation_fn, lr_schedule=self._dummy_schedule,
                         optimizer_class=self.optimizer_class, optimizer_kwargs=self.optimizer_kwargs,
                         features_extractor_class=self.features_extractor_class,
                         features_extractor_kwargs=self.features_extractor_kwargs))
        return data

    def forward(self, obs, deterministic: bool = False) -> th.Tensor:
        return self._predict(obs, deterministic=deterministic)

    def _predict(self, observation, deterministic: bool = False) -> th.Tensor:
        return self.actor(observation, deterministic)

    def set_training_mode(self, mode: bool) -> None:
        self.actor.set_training_mode(mode)
        self.critic.set_training_mode(mode)
        self.training = mode


class SAC(OffPolicyAlgorithm):
    policy_aliases = {"MlpPolicy": SACPolicy}  # + "MultiInputPolicy" (defined below)

    def __init__(self, policy, env, learning_rate=3e-4, buffer_size: int = 1_000_000, learning_starts: int = 100,
                 batch_size: int = 256, tau: float = 0.005, gamma: float = 0.99, train_freq=1, gradient_steps: int = 1,
                 action_noise=None, replay_buffer_class=None, replay_buffer_kwargs=None, optimize_memory_usage: bool = False,
                 ent_coef: Union[str, float] = "auto", target_update_interval: int = 1,
                 target_entropy: Union[str, float] = "auto", use_sde: bool = False, sde_sample_freq: int = -1,
                 use_sde_at_warmup: bool = False, stats_window_size: int = 100, tensorboard_log=None,
                 policy_kwargs=None, verbose: int = 0, seed=None, device="auto", _init_setup_model: bool = True):
        super().__init__(policy, env, learning_rate, buffer_size, learning_starts, batch_size, tau, gamma, train_freq,
                         gradient_steps, action_noise, replay_buffer_class=replay_buffer_class,
                         replay_buffer_kwargs=replay_buffer_kwargs, policy_kwargs=policy_kwargs,
                         stats_window_size=stats_window_size, tensorboard_log=tensorboard_log, verbose=verbose,
                         device=device, seed=seed, use_sde=use_sde, sde_sample_freq=sde_sample_freq,
                         use_sde_at_warmup=use_sde_at_warmup, optimize_memory_usage=optimize_memory_usage,
                         supported_action_spaces=(spaces.Box,))
        self.target_entropy = target_entropy
        self.log_ent_coef = None
        self.ent_coef = ent_coef
        self.target_update_interval = target_update_interval
        self.ent_coef_optimizer = None
        if _init_setup_model:
            self._setup_model()

    def _setup_model(self) -> None:
        super()._setup_model()
        self.actor = self.policy.actor
        self.critic = self.policy.critic
        self.critic_target = self.policy.critic_target
        if self.target_entropy == "auto":
            self.target_entropy = float(-np.prod(self.env.action_space.shape if self.env is not None else self.action_space.shape).astype(np.float32))
        else:
            self.target_entropy = float(self.target_entropy)
        if isinstance(self.ent_coef, str) and self.ent_coef.startswith("auto"):
            init_value = 1.0
            if "_" in self.ent_coef:
                init_value = float(self.ent_coef.split("_")[1])
                assert init_value > 0.0
            self.log_ent_coef = th.log(th.ones(1, device=self.device) * init_value).requires_grad_(True)
            self.ent_coef_optimizer = th.optim.Adam([self.log_ent_coef], lr=self.lr_schedule(1))
        else:
            self.ent_coef_tensor = th.tensor(float(self.ent_coef), device=self.device)
        self._actor_bucket = pdist.GradBucket(self.actor.parameters()) if pdist.world_size() > 1 else None
        self._critic_bucket = pdist.GradBucket([p for g in self.critic.optimizer.param_groups for p in g["params"]]) if pdist.world_size() > 1 else None

    def train(self, gradient_steps: int, batch_size: int = 64) -> None:
        self.policy.set_training_mode(True)
        optimizers = [self.actor.optimizer, self.critic.optimizer]
        if self.ent_coef_optimizer is not None:
            optimizers += [self.ent_coef_optimizer]
        self._update_learning_rate(optimizers)
        ent_coef_losses, ent_coefs, actor_losses, critic_losses = [], [], [], []
        for gradient_step in range(gradient_steps):
            replay_data = self.replay_buffer.sample(batch_size, env=self._vec_normalize_env)
            actions_pi, log_prob = self.actor.action_log_prob(replay_data.observations)
            log_prob = log_prob.reshape(-1, 1)
            ent_coef_loss = None
            if self.ent_coef_optimizer is not None and self.log_ent_coef is not None:
                ent_coef = th.exp(self.log_ent_coef.detach())
                ent_coef_loss = -(self.log_ent_coef * (log_prob + self.target_entropy).detach()).mean()
                ent_coef_losses.append(ent_coef_loss.detach())
            else:
                ent_coef = self.ent_coef_tensor
            ent_coefs.append(ent_coef.detach().reshape(()))
            if ent_coef_loss is not None and self.ent_coef_optimizer is not None:
                self.ent_coef_optimizer.zero_grad()
                ent_coef_loss.backward()
                if pdist.world_size() > 1:
                    pdist.allreduce_grads([self.log_ent_coef])
                self.ent_coef_optimizer.step()
            with th.no_grad():
                next_actions, next_log_prob = self.actor.action_log_prob(replay_data.next_observations)
                next_q_values = th.cat(self.critic_target(replay_data.next_observations, next_actions), dim=1)
                next_q_values, _ = th.min(next_q_values, dim=1, keepdim=True)
                next_q_values = next_q_values - ent_coef * next_log_prob.reshape(-1, 1)
                target_q_values = replay_data.rewards + (1 - replay_data.dones) * self.gamma * next_q_values
            current_q_values = self.critic(replay_data.observations, replay_data.actions)
            critic_loss = 0.5 * sum(F.mse_loss(q, target_q_values) for q in current_q_values)
            critic_losses.append(critic_loss.detach())
            self.critic.optimizer.zero_grad()
            critic_loss.backward()
            if self._critic_bucket is not None:
                pdist.allreduce_grads(self._critic_bucket.params)
            self.critic.optimizer.step()
            q_values_pi = th.cat(self.critic(replay_data.observations, actions_pi), dim=1)
            min_qf_pi, _ = th.min(q_values_pi, dim=1, keepdim=True)
            actor_loss = (ent_coef * log_prob - min_qf_pi).mean()
            actor_losses.append(actor_loss.detach())
            self.actor.optimizer.zero_grad()
            actor_loss.backward()
            if self._actor_bucket is not None:
                pdist.allreduce_grads(self._actor_bucket.params)
            self.actor.optimizer.step()
            if gradient_step % self.target_update_interval == 0:
                polyak_update(self.critic.parameters(), self.critic_target.parameters(), self.tau)
        self._n_updates += gradient_steps
        self.logger.record("train/n_updates", self._n_updates, exclude="tensorboard")
        self.logger.record("train/ent_coef", float(th.stack(ent_coefs).mean()))
        self.logger.record("train/actor_loss", float(th.stack(actor_losses).mean()))
        self.logger.record("train/critic_loss", float(th.stack(critic_losses).mean()))
        if ent_coef_losses:
            self.logger.record("train/ent_coef_loss", float(th.stack(ent_coef_losses).mean()))

    def _excluded_save_params(self):
        return super()._excluded_save_params() | {"actor", "critic", "critic_target", "_actor_bucket", "_critic_bucket", "ent_coef_tensor"}


class MultiInputPolicy(SACPolicy):
    """:class:`SACPolicy` over ``spaces.Dict`` observations (SB3 ``MultiInputPolicy``): the
    per-key features are concatenated by :class:`CombinedExtractor`."""

    def __init__(self, observation_space, action_space, lr_schedule, net_arch=None, activation_fn: Type[nn.Module] = nn.ReLU,
                 use_sde: bool = False, log_std_init: float = -3, use_expln: bool = False, clip_mean: float = 2.0,
                 features_extractor_class: Type[BaseFeaturesExtractor] = CombinedExtractor, features_extractor_kwargs=None,
                 normalize_images: bool = True, optimizer_class: Type[th.optim.Optimizer] = th.optim.Adam,
                 optimizer_kwargs=None, n_critics: int = 2, share_features_extractor: bool = False):
        super().__init__(observation_space, action_space, lr_schedule, net_arch, activation_fn, use_sde, log_std_init,
                         use_expln, clip_mean, features_extractor_class, features_extractor_kwargs, normalize_images,
                         optimizer_class, optimizer_kwargs, n_critics, share_features_extractor)


SAC.policy_aliases["MultiInputPolicy"] = MultiInputPolicy

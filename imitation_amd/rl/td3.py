"""TD3 and DDPG (SB3 ``td3`` / ``ddpg`` semantics; the reference's SQIL tests train both:
``tests/algorithms/test_sqil.py:14-15, 97-112, 150-174``).

Deterministic tanh actor, twin Q critics (DDPG: one), target-policy smoothing (clipped Gaussian
noise on the target action), delayed actor / Polyak updates every ``policy_delay`` critic steps.
DDPG is TD3 with ``policy_delay=1``, one critic and no target smoothing. Under data parallelism
each optimiser step's gradients are averaged with one bucketed all-reduce, as in SAC.
"""

from __future__ import annotations

from typing import Any, Dict, List, Optional, Type

import torch as th
from torch import nn
from torch.nn import functional as F

from imitation_amd.envs import spaces
from imitation_amd.parallel import dist as pdist
from imitation_amd.rl.off_policy import OffPolicyAlgorithm, polyak_update
from imitation_amd.rl.policies import BasePolicy
from imitation_amd.rl.preprocessing import get_action_dim
from imitation_amd.rl.sac import ContinuousCritic
from imitation_amd.rl.torch_layers import (BaseFeaturesExtractor, CombinedExtractor, FlattenExtractor, create_mlp,
                                           get_actor_critic_arch)


class Actor(BasePolicy):
    """``mu(s) = tanh(MLP(features))`` in the scaled action box."""

    def __init__(self, observation_space, action_space, net_arch: List[int], features_extractor: nn.Module, features_dim: int,
                 activation_fn: Type[nn.Module] = nn.ReLU, normalize_images: bool = True):
        super().__init__(observation_space, action_space, features_extractor=features_extractor, normalize_images=normalize_images,
                         squash_output=True)
        self.net_arch = net_arch
        self.features_dim = features_dim
        self.activation_fn = activation_fn
        action_dim = get_action_dim(self.action_space)
        self.mu = nn.Sequential(*create_mlp(features_dim, action_dim, net_arch, activation_fn, squash_output=True))

    def forward(self, obs) -> th.Tensor:
        return self.mu(self.extract_features(obs, self.features_extractor))

    def _predict(self, observation, deterministic: bool = False) -> th.Tensor:
        return self(observation)


class TD3Policy(BasePolicy):
    def __init__(self, observation_space, action_space, lr_schedule, net_arch=None, activation_fn: Type[nn.Module] = nn.ReLU,
                 features_extractor_class: Type[BaseFeaturesExtractor] = FlattenExtractor, features_extractor_kwargs=None,
                 normalize_images: bool = True, optimizer_class: Type[th.optim.Optimizer] = th.optim.Adam,
                 optimizer_kwargs=None, n_critics: int = 2, share_features_extractor: bool = False):
        super().__init__(observation_space, action_space, features_extractor_class, features_extractor_kwargs,
                         optimizer_class=optimizer_class, optimizer_kwargs=optimizer_kwargs, squash_output=True,
                         normalize_images=normalize_images)
        if net_arch is None:
            net_arch = [400, 300] if features_extractor_class is FlattenExtractor else [256, 256]
        actor_arch, critic_arch = get_actor_critic_arch(net_arch)
        self.net_arch = net_arch
        self.activation_fn = activation_fn
        self.n_critics = n_critics
        self.actor_kwargs = dict(observation_space=observation_space, action_space=action_space, net_arch=actor_arch,
                                 activation_fn=activation_fn, normalize_images=normalize_images)
        self.critic_kwargs = dict(self.actor_kwargs)
        self.critic_kwargs.update(n_critics=n_critics, net_arch=critic_arch, share_features_extractor=share_features_extractor)
        self.share_features_extractor = share_features_extractor
        self._build(lr_schedule)

    def _build(self, lr_schedule) -> None:
        self.actor = self.make_actor()
        self.actor_target = self.make_actor()
        self.actor_target.load_state_dict(self.actor.state_dict())
        self.actor.optimizer = self.optimizer_class(self.actor.parameters(), lr=lr_schedule(1), **self.optimizer_kwargs)
        if self.share_features_extractor:
            self.critic = self.make_critic(features_extractor=self.actor.features_extractor)
            self.critic_target = self.make_critic(features_extractor=self.actor_target.features_extractor)
            critic_parameters = [p for n, p in self.critic.named_parameters() if "features_extractor" not in n]
        else:
            self.critic = self.make_critic()
            self.critic_target = self.make_critic()
            critic_parameters = list(self.critic.parameters())
        self.critic_target.load_state_dict(self.critic.state_dict())
        self.critic.optimizer = self.optimizer_class(critic_parameters, lr=lr_schedule(1), **self.optimizer_kwargs)
        self.actor_target.set_training_mode(False)
        self.critic_target.set_training_mode(False)

    def make_actor(self, features_extractor=None) -> Actor:
        fe = features_extractor or self.make_features_extractor()
        return Actor(features_extractor=fe, features_dim=fe.features_dim, **self.actor_kwargs)

    def make_critic(self, features_extractor=None) -> ContinuousCritic:
        fe = features_extractor or self.make_features_extractor()
        return ContinuousCritic(features_extractor=fe, features_dim=fe.features_dim, **self.critic_kwargs)

    def _get_constructor_parameters(self) -> Dict[str, Any]:
        data = super()._get_constructor_parameters()
        data.update(dict(net_arch=self.net_arch, activation_fn=self.activation_fn, n_critics=self.n_critics,
                         lr_schedule=self._dummy_schedule, optimizer_class=self.optimizer_class,
                         optimizer_kwargs=self.optimizer_kwargs, features_extractor_class=self.features_extractor_class,
                         features_extractor_kwargs=self.features_extractor_kwargs,
                         share_features_extractor=self.share_features_extractor))
        return data

    def forward(self, obs, deterministic: bool = False) -> th.Tensor:
        return self._predict(obs, deterministic=deterministic)

    def _predict(self, observation, deterministic: bool = False) -> th.Tensor:
        return self.actor(observation)  # deterministic either way; exploration is action noise

    def set_training_mode(self, mode: bool) -> None:
        self.actor.set_training_mode(mode)
        self.critic.set_training_mode(mode)
        self.training = mode


class MultiInputPolicy(TD3Policy):
    """:class:`TD3Policy` over ``spaces.Dict`` observations (per-key features concatenated)."""

    def __init__(self, observation_space, action_space, lr_schedule, net_arch=None, activation_fn: Type[nn.Module] = nn.ReLU,
                 features_extractor_class: Type[BaseFeaturesExtractor] = CombinedExtractor, features_extractor_kwargs=None,
                 normalize_images: bool = True, optimizer_class: Type[th.optim.Optimizer] = th.optim.Adam,
                 optimizer_kwargs=None, n_critics: int = 2, share_features_extractor: bool = False):
        super().__init__(observation_space, action_space, lr_schedule, net_arch, activation_fn, features_extractor_class,
                         features_extractor_kwargs, normalize_images, optimizer_class, optimizer_kwargs, n_critics,
                         share_features_extractor)


class TD3(OffPolicyAlgorithm):
    policy_aliases = {"MlpPolicy": TD3Policy, "MultiInputPolicy": MultiInputPolicy}

    def __init__(self, policy, env, learning_rate=1e-3, buffer_size: int = 1_000_000, learning_starts: int = 100,
                 batch_size: int = 256, tau: float = 0.005, gamma: float = 0.99, train_freq=1, gradient_steps: int = 1,
                 action_noise=None, replay_buffer_class=None, replay_buffer_kwargs=None, optimize_memory_usage: bool = False,
                 policy_delay: int = 2, target_policy_noise: float = 0.2, target_noise_clip: float = 0.5,
                 stats_window_size: int = 100, tensorboard_log=None, policy_kwargs=None, verbose: int = 0, seed=None,
                 device="auto", _init_setup_model: bool = True):
        super().__init__(policy, env, learning_rate, buffer_size, learning_starts, batch_size, tau, gamma, train_freq,
                         gradient_steps, action_noise, replay_buffer_class=replay_buffer_class,
                         replay_buffer_kwargs=replay_buffer_kwargs, policy_kwargs=policy_kwargs,
                         stats_window_size=stats_window_size, tensorboard_log=tensorboard_log, verbose=verbose,
                         device=device, seed=seed, sde_support=False, optimize_memory_usage=optimize_memory_usage,
                         supported_action_spaces=(spaces.Box,))
        self.policy_delay = policy_delay
        self.target_noise_clip = target_noise_clip
        self.target_policy_noise = target_policy_noise
        if _init_setup_model:
            self._setup_model()

    def _setup_model(self) -> None:
        super()._setup_model()
        self.actor = self.policy.actor
        self.actor_target = self.policy.actor_target
        self.critic = self.policy.critic
        self.critic_target = self.policy.critic_target
        world = pdist.world_size()
        self._actor_bucket = pdist.GradBucket(self.actor.parameters()) if world > 1 else None
        self._critic_bucket = pdist.GradBucket([p for g in self.critic.optimizer.param_groups for p in g["params"]]) if world > 1 else None

    def train(self, gradient_steps: int, batch_size: int = 100) -> None:
        self.policy.set_training_mode(True)
        self._update_learning_rate([self.actor.optimizer, self.critic.optimizer])
        actor_losses, critic_losses = [], []
        for _ in range(gradient_steps):
            self._n_updates += 1
            replay_data = self.replay_buffer.sample(batch_size, env=self._vec_normalize_env)
            with th.no_grad():
                # target policy smoothing: clipped Gaussian noise on the target action
                noise = replay_data.actions.clone().normal_(0, self.target_policy_noise)
                noise = noise.clamp(-self.target_noise_clip, self.target_noise_clip)
                next_actions = (self.actor_target(replay_data.next_observations) + noise).clamp(-1, 1)
                next_q_values = th.cat(self.critic_target(replay_data.next_observations, next_actions), dim=1)
                next_q_values, _ = th.min(next_q_values, dim=1, keepdim=True)
                target_q_values = replay_data.rewards + (1 - replay_data.dones) * self.gamma * next_q_values
            current_q_values = self.critic(replay_data.observations, replay_data.actions)
            critic_loss = sum(F.mse_loss(q, target_q_values) for q in current_q_values)
            critic_losses.append(critic_loss.detach())
            self.critic.optimizer.zero_grad()
            critic_loss.backward()
            if self._critic_bucket is not None:
                pdist.allreduce_grads(self._critic_bucket.params)
            self.critic.optimizer.step()
            if self._n_updates % self.policy_delay == 0:
                actor_loss = -self.critic.q1_forward(replay_data.observations, self.actor(replay_data.observations)).mean()
                actor_losses.append(actor_loss.detach())
                self.actor.optimizer.zero_grad()
                actor_loss.backward()
                if self._actor_bucket is not None:
                    pdist.allreduce_grads(self._actor_bucket.params)
                self.actor.optimizer.step()
                polyak_update(self.critic.parameters(), self.critic_target.parameters(), self.tau)
                polyak_update(self.actor.parameters(), self.actor_target.parameters(), self.tau)
        self.logger.record("train/n_updates", self._n_updates, exclude="tensorboard")
        if actor_losses:
            self.logger.record("train/actor_loss", float(th.stack(actor_losses).mean()))
        self.logger.record("train/critic_loss", float(th.stack(critic_losses).mean()))

    def _excluded_save_params(self):
        return super()._excluded_save_params() | {"actor", "critic", "actor_target", "critic_target", "_actor_bucket",
                                                   "_critic_bucket"}


class DDPG(TD3):
    """TD3 with one critic, no target smoothing and an actor update every critic step."""

    def __init__(self, policy, env, learning_rate=1e-3, buffer_size: int = 1_000_000, learning_starts: int = 100,
                 batch_size: int = 256, tau: float = 0.005, gamma: float = 0.99, train_freq=1, gradient_steps: int = 1,
                 action_noise=None, replay_buffer_class=None, replay_buffer_kwargs=None, optimize_memory_usage: bool = False,
                 stats_window_size: int = 100, tensorboard_log=None, policy_kwargs=None, verbose: int = 0, seed=None,
                 device="auto", _init_setup_model: bool = True):
        policy_kwargs = dict(policy_kwargs or {})
        policy_kwargs.setdefault("n_critics", 1)
        super().__init__(policy, env, learning_rate, buffer_size, learning_starts, batch_size, tau, gamma, train_freq,
                         gradient_steps, action_noise, replay_buffer_class, replay_buffer_kwargs, optimize_memory_usage,
                         policy_delay=1, target_policy_noise=0.0, target_noise_clip=0.0,
                         stats_window_size=stats_window_size, tensorboard_log=tensorboard_log, policy_kwargs=policy_kwargs,
                         verbose=verbose, seed=seed, device=device, _init_setup_model=_init_setup_model)

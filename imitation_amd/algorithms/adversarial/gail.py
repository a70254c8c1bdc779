"""GAIL (reference: ``src/imitation/algorithms/adversarial/gail.py``).

The discriminator is the reward net's logit; the generator reward is
``-log σ(-logit)`` (``gail.py:82-83``), computed by the fused log-sigmoid kernel
when the logits live on the GPU.
"""

from __future__ import annotations

from typing import Optional

import torch as th

from imitation_amd.algorithms import base
from imitation_amd.algorithms.adversarial import common
from imitation_amd.rewards import reward_nets


class RewardNetFromDiscriminatorLogit(reward_nets.RewardNet):
    """Converts a discriminator-logit net into a reward: ``-log(1 - D) = -log σ(-logit)``."""

    def __init__(self, base: reward_nets.RewardNet):
        super().__init__(observation_space=base.observation_space, action_space=base.action_space, normalize_images=base.normalize_images)
        self.base = base

    def forward(self, state: th.Tensor, action: th.Tensor, next_state: th.Tensor, done: th.Tensor) -> th.Tensor:
        logits = self.base.forward(state, action, next_state, done)
        return th.nn.functional.softplus(logits)  # -log(1 - sigmoid(logits))


class GAIL(common.AdversarialTrainer):
    """Generative Adversarial Imitation Learning (Ho & Ermon 2016)."""

    def __init__(self, *, demonstrations: base.AnyTransitions, demo_batch_size: int, venv, gen_algo, reward_net: reward_nets.RewardNet, **kwargs):
        reward_net = reward_net.to(gen_algo.device)
        self._processed_reward = RewardNetFromDiscriminatorLogit(reward_net)
        super().__init__(demonstrations=demonstrations, demo_batch_size=demo_batch_size, venv=venv, gen_algo=gen_algo,
                         reward_net=reward_net, **kwargs)

    def logits_expert_is_high(self, state, action, next_state, done, log_policy_act_prob: Optional[th.Tensor] = None) -> th.Tensor:
        del log_policy_act_prob
        logits = self._reward_net(state, action, next_state, done)
        assert logits.shape == state.shape[:1]
        return logits

    @property
    def reward_train(self) -> reward_nets.RewardNet:
        return self._processed_reward

    @property
    def reward_test(self) -> reward_nets.RewardNet:
        return self._processed_reward

"""AIRL (reference: ``src/imitation/algorithms/adversarial/airl.py``).

Discriminator logit ``r_θ(s,a,s',d) - log π(a|s)`` (``airl.py:114-119``) -- requires
a stochastic generator policy; the test reward strips every wrapper down to the
unshaped base net (``:126-132``).
"""

from __future__ import annotations

from typing import Optional

import torch as th

from imitation_amd.algorithms import base
from imitation_amd.algorithms.adversarial import common
from imitation_amd.rewards import reward_nets
from imitation_amd.rl.policies import ActorCriticPolicy


def _stochastic_policies():
    from imitation_amd.rl.sac import SACPolicy

    return (ActorCriticPolicy, SACPolicy)


STOCHASTIC_POLICIES = (ActorCriticPolicy,)


class AIRL(common.AdversarialTrainer):
    """Adversarial Inverse Reinforcement Learning (Fu et al. 2018)."""

    def __init__(self, *, demonstrations: base.AnyTransitions, demo_batch_size: int, venv, gen_algo, reward_net: reward_nets.RewardNet, **kwargs):
        super().__init__(demonstrations=demonstrations, demo_batch_size=demo_batch_size, venv=venv, gen_algo=gen_algo,
                         reward_net=reward_net, **kwargs)
        if not isinstance(self.gen_algo.policy, _stochastic_policies()):
            raise TypeError("AIRL needs a stochastic policy to compute the discriminator output.")

    def logits_expert_is_high(self, state, action, next_state, done, log_policy_act_prob: Optional[th.Tensor] = None) -> th.Tensor:
        if log_policy_act_prob is None:
            raise TypeError("Non-None `log_policy_act_prob` is required for this method.")
        return self._reward_net(state, action, next_state, done) - log_policy_act_prob

    @property
    def reward_train(self) -> reward_nets.RewardNet:
        return self._reward_net

    @property
    def reward_test(self) -> reward_nets.RewardNet:
        reward_net = self._reward_net
        while isinstance(reward_net, reward_nets.RewardNetWrapper):
            reward_net = reward_net.base
        return reward_net

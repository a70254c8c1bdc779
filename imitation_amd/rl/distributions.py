"""Action distributions (SB3 ``distributions`` surface).

Categorical / MultiCategorical / Bernoulli (discrete), DiagGaussian with a
state-independent ``log_std`` (continuous PPO/BC/AIRL), SquashedDiagGaussian
(SAC). Log-probs and entropies are computed in fp32 with stable forms
(log-softmax, closed-form Gaussian entropy).
"""

from __future__ import annotations

import math
from typing import List, Optional, Tuple

import numpy as np
import torch as th
from torch import nn
from torch.nn import functional as F

from imitation_amd.envs import spaces

_LOG_2PI = math.log(2 * math.pi)


def sum_independent_dims(t: th.Tensor) -> th.Tensor:
    return t.sum(dim=1) if t.dim() > 1 else t.sum()


class Distribution:
    """Base class: parametrise with ``proba_distribution``, then query."""

    def proba_distribution_net(self, *args, **kwargs):
        raise NotImplementedError

    def proba_distribution(self, *args, **kwargs) -> "Distribution":
        raise NotImplementedError

    def log_prob(self, x: th.Tensor) -> th.Tensor:
        raise NotImplementedError

    def entropy(self) -> Optional[th.Tensor]:
        raise NotImplementedError

    def sample(self) -> th.Tensor:
        raise NotImplementedError

    def mode(self) -> th.Tensor:
        raise NotImplementedError

    def get_actions(self, deterministic: bool = False) -> th.Tensor:
        return self.mode() if deterministic else self.sample()

    def actions_from_params(self, *args, deterministic: bool = False, **kwargs) -> th.Tensor:
        self.proba_distribution(*args, **kwargs)
        return self.get_actions(deterministic=deterministic)

    def log_prob_from_params(self, *args, **kwargs) -> Tuple[th.Tensor, th.Tensor]:
        actions = self.actions_from_params(*args, **kwargs)
        return actions, self.log_prob(actions)

    def detach_(self) -> "Distribution":
        """Detach the stored parameters from their autograd graph.

        The policy keeps ONE distribution object that every ``get_distribution`` call
        re-parametrises, so its tensors keep the last forward's graph -- and through it the
        parameters' AccumulateGrad nodes -- alive. Graph capture needs those nodes created
        on the capture stream (``utils.graphs.GraphedTrainStep`` calls this first)."""
        for k, v in vars(self).items():
            if isinstance(v, th.Tensor) and v.grad_fn is not None:
                setattr(self, k, v.detach())
            elif isinstance(v, list):
                for d in v:
                    if isinstance(d, Distribution):
                        d.detach_()
        return self


class DiagGaussianDistribution(Distribution):
    """Gaussian with diagonal covariance; ``log_std`` is a free parameter."""

    def __init__(self, action_dim: int):
        self.action_dim = action_dim
        self.mean_actions: Optional[th.Tensor] = None
        self.log_std: Optional[th.Tensor] = None

    def proba_distribution_net(self, latent_dim: int, log_std_init: float = 0.0) -> Tuple[nn.Module, nn.Parameter]:
        mean_actions = nn.Linear(latent_dim, self.action_dim)
        log_std = nn.Parameter(th.ones(self.action_dim) * log_std_init, requires_grad=True)
        return mean_actions, log_std

    def proba_distribution(self, mean_actions: th.Tensor, log_std: th.Tensor) -> "DiagGaussianDistribution":
        self.mean_actions = mean_actions
        self.log_std = log_std.expand_as(mean_actions) if log_std.dim() < mean_actions.dim() else log_std
        return self

    @property
    def distribution(self):
        return th.distributions.Normal(self.mean_actions, th.exp(self.log_std))

    def log_prob(self, actions: th.Tensor) -> th.Tensor:
        std = th.exp(self.log_std)
        z = (actions - self.mean_actions) / std
        lp = -0.5 * z * z - self.log_std - 0.5 * _LOG_2PI
        return sum_independent_dims(lp)

    def entropy(self) -> th.Tensor:
        ent = 0.5 + 0.5 * _LOG_2PI + self.log_std
        return sum_independent_dims(ent)

    def sample(self) -> th.Tensor:
        return self.mean_actions + th.exp(self.log_std) * th.randn_like(self.mean_actions)

    def mode(self) -> th.Tensor:
        return self.mean_actions


class SquashedDiagGaussianDistribution(DiagGaussianDistribution):
    """tanh-squashed Gaussian (SAC actor)."""

    def __init__(self, action_dim: int, epsilon: float = 1e-6):
        super().__init__(action_dim)
        self.epsilon = epsilon
        self.gaussian_actions: Optional[th.Tensor] = None

    def log_prob(self, actions: th.Tensor, gaussian_actions: Optional[th.Tensor] = None) -> th.Tensor:
        if gaussian_actions is None:
            a = actions.clamp(-1.0 + 1e-6, 1.0 - 1e-6)
            gaussian_actions = 0.5 * (a.log1p() - (-a).log1p())
        lp = super().log_prob(gaussian_actions)
        lp -= th.sum(th.log(1 - actions**2 + self.epsilon), dim=1)
        return lp

    def entropy(self) -> Optional[th.Tensor]:
        return None

    def sample(self) -> th.Tensor:
        self.gaussian_actions = super().sample()
        return th.tanh(self.gaussian_actions)

    def mode(self) -> th.Tensor:
        self.gaussian_actions = super().mode()
        return th.tanh(self.gaussian_actions)

    def log_prob_from_params(self, mean_actions, log_std) -> Tuple[th.Tensor, th.Tensor]:
        action = self.actions_from_params(mean_actions, log_std)
        return action, self.log_prob(action, self.gaussian_actions)


class CategoricalDistribution(Distribution):
    def __init__(self, action_dim: int):
        self.action_dim = action_dim
        self.raw_logits: Optional[th.Tensor] = None
        self._logits: Optional[th.Tensor] = None

    def proba_distribution_net(self, latent_dim: int) -> nn.Module:
        return nn.Linear(latent_dim, self.action_dim)

    def proba_distribution(self, action_logits: th.Tensor) -> "CategoricalDistribution":
        self.raw_logits = action_logits
        self._logits = None
        return self

    @property
    def logits(self) -> Optional[th.Tensor]:
        """Normalised log-probabilities, computed on first use (the fused BC / evaluation
        paths read only ``raw_logits`` and never pay for the logsumexp)."""
        if self._logits is None and self.raw_logits is not None:
            z = self.raw_logits
            self._logits = z - z.logsumexp(dim=-1, keepdim=True)
        return self._logits

    def log_prob_entropy(self, actions: th.Tensor) -> Tuple[th.Tensor, th.Tensor]:
        """``(log_prob(actions), entropy())`` in one fused pass over the raw logits (HIP
        ``cat_eval`` on the GPU, identical formulas on the CPU)."""
        from imitation_amd.ops.rl import categorical_eval

        return categorical_eval(self.raw_logits, actions)

    @property
    def probs(self) -> th.Tensor:
        return self.logits.exp()

    @property
    def distribution(self):
        return th.distributions.Categorical(logits=self.logits)

    def log_prob(self, actions: th.Tensor) -> th.Tensor:
        a = actions.long().reshape(-1, 1)
        return self.logits.gather(-1, a).squeeze(-1)

    def entropy(self) -> th.Tensor:
        p = self.probs
        return -(p * self.logits).sum(-1)

    def sample(self) -> th.Tensor:
        return th.multinomial(self.probs, 1).squeeze(-1)

    def mode(self) -> th.Tensor:
        return th.argmax(self.logits, dim=1)


class MultiCategoricalDistribution(Distribution):
    def __init__(self, action_dims: List[int]):
        self.action_dims = list(action_dims)
        self.dists: List[CategoricalDistribution] = []

    def proba_distribution_net(self, latent_dim: int) -> nn.Module:
        return nn.Linear(latent_dim, sum(self.action_dims))

    def proba_distribution(self, action_logits: th.Tensor) -> "MultiCategoricalDistribution":
        self.dists = [CategoricalDistribution(n).proba_distribution(s) for n, s in zip(self.action_dims, th.split(action_logits, self.action_dims, dim=1))]
        return self

    def log_prob(self, actions: th.Tensor) -> th.Tensor:
        return th.stack([d.log_prob(a) for d, a in zip(self.dists, th.unbind(actions, dim=1))], dim=1).sum(dim=1)

    def entropy(self) -> th.Tensor:
        return th.stack([d.entropy() for d in self.dists], dim=1).sum(dim=1)

    def sample(self) -> th.Tensor:
        return th.stack([d.sample() for d in self.dists], dim=1)

    def mode(self) -> th.Tensor:
        return th.stack([d.mode() for d in self.dists], dim=1)


class BernoulliDistribution(Distribution):
    def __init__(self, action_dims: int):
        self.action_dims = action_dims
        self.logits: Optional[th.Tensor] = None

    def proba_distribution_net(self, latent_dim: int) -> nn.Module:
        return nn.Linear(latent_dim, self.action_dims)

    def proba_distribution(self, action_logits: th.Tensor) -> "BernoulliDistribution":
        self.logits = action_logits
        return self

    def log_prob(self, actions: th.Tensor) -> th.Tensor:
        return -F.binary_cross_entropy_with_logits(self.logits, actions.float(), reduction="none").sum(dim=1)

    def entropy(self) -> th.Tensor:
        p = th.sigmoid(self.logits)
        return F.binary_cross_entropy_with_logits(self.logits, p, reduction="none").sum(dim=1)

    def sample(self) -> th.Tensor:
        return th.bernoulli(th.sigmoid(self.logits))

    def mode(self) -> th.Tensor:
        return (self.logits > 0).float()


def make_proba_distribution(action_space: spaces.Space, use_sde: bool = False, dist_kwargs: Optional[dict] = None) -> Distribution:
    dist_kwargs = dist_kwargs or {}
    if use_sde:
        raise NotImplementedError("gSDE is not supported")
    if isinstance(action_space, spaces.Box):
        return DiagGaussianDistribution(int(np.prod(action_space.shape)), **dist_kwargs)
    if isinstance(action_space, spaces.Discrete):
        return CategoricalDistribution(int(action_space.n), **dist_kwargs)
    if isinstance(action_space, spaces.MultiDiscrete):
        return MultiCategoricalDistribution([int(n) for n in action_space.nvec], **dist_kwargs)
    if isinstance(action_space, spaces.MultiBinary):
        return BernoulliDistribution(int(np.prod(action_space.shape)), **dist_kwargs)
    raise NotImplementedError(f"Unsupported action space {action_space}")


def kl_divergence(dist_true: Distribution, dist_pred: Distribution) -> th.Tensor:
    if isinstance(dist_true, DiagGaussianDistribution):
        return th.distributions.kl_divergence(dist_true.distribution, dist_pred.distribution).sum(dim=1)
    if isinstance(dist_true, CategoricalDistribution):
        return (dist_true.probs * (dist_true.logits - dist_pred.logits)).sum(-1)
    raise NotImplementedError

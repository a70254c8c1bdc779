"""Custom policies and feature extractors (reference: ``src/imitation/policies/base.py``).

* :class:`HomogenousActorCriticPolicy` (fork addition, ``base.py:20-130``): one
  parameter-shared actor-critic evaluated for ``num_agents`` agents whose
  observations are sliced by ``observation_overide(i, obs)``; actions are
  ``hstack``-ed. MI355X design: the agents are folded into the batch (M)
  dimension -- ONE fused forward for all agents instead of ``num_agents``
  sequential launches (SURVEY §2.4 "multi-agent parameter sharing").
  Fork quirk kept on purpose: ``_predict`` passed its kwargs as the positional
  ``deterministic`` argument, so predictions were always deterministic
  (``base.py:36-39``). That stays the default; pass
  ``respect_deterministic=True`` to honour the flag instead.
* :class:`NonTrainablePolicy`, :class:`RandomPolicy`, :class:`ZeroPolicy`;
* :class:`FeedForward32Policy` (``net_arch=[32, 32]``),
  :class:`HomogenousFeedForward32Policy` (``[256, 256, 128]`` despite the name),
  :class:`SAC1024Policy` (``[1024, 1024]``);
* :class:`NormalizeFeaturesExtractor` (flatten + RunningNorm).
"""

from __future__ import annotations

import abc
from typing import Any, Dict, Optional, Tuple, Type, Union

import numpy as np
import torch as th
from torch import nn

from imitation_amd.data import types
from imitation_amd.envs import spaces
from imitation_amd.rl import policies
from imitation_amd.rl.policies import get_device, obs_as_tensor
from imitation_amd.rl.sac import SACPolicy
from imitation_amd.rl.torch_layers import FlattenExtractor
from imitation_amd.util import networks


class HomogenousActorCriticPolicy(policies.ActorCriticPolicy):
    """Parameter-shared actor-critic over ``num_agents`` homogeneous agents."""

    def __init__(self, observation_overide, action_overide, num_agents, respect_deterministic: bool = False, **acp_kwargs):
        super().__init__(**acp_kwargs)
        self.observation_overide = observation_overide
        self.action_overide = action_overide
        self.num_agents = num_agents
        self.respect_deterministic = respect_deterministic

    def _agent_batch(self, observation):
        """Stack every agent's sub-observation along the batch axis (one forward for all agents)."""
        per_agent = [self.observation_overide(i, observation) for i in range(self.num_agents)]
        per_agent = [p if isinstance(p, th.Tensor) else th.as_tensor(np.asarray(p), device=self.device) for p in per_agent]
        sizes = [p.shape[0] for p in per_agent]
        return th.cat(per_agent, dim=0), sizes

    def _predict(self, observation, deterministic: bool = False, **predict_kwargs):
        det = deterministic if self.respect_deterministic else True
        stacked, sizes = self._agent_batch(observation)
        acts = super()._predict(stacked, deterministic=det)
        acts = acts.reshape(sum(sizes), -1) if acts.dim() > 1 else acts.reshape(-1, 1)
        return th.hstack(list(th.split(acts, sizes, dim=0)))

    def predict(self, observation, state: Optional[Tuple[np.ndarray, ...]] = None, episode_start: Optional[np.ndarray] = None,
                deterministic: bool = False) -> Tuple[np.ndarray, Optional[Tuple[np.ndarray, ...]]]:
        self.set_training_mode(False)
        if isinstance(observation, tuple) and len(observation) == 2 and isinstance(observation[1], dict):
            raise ValueError(
                "You have passed a tuple to the predict() function instead of a Numpy array or a Dict. "
                "You are probably mixing Gym API with SB3 VecEnv API: `obs, info = env.reset()` (Gym) "
                "vs `obs = vec_env.reset()` (SB3 VecEnv)."
            )
        obs_tensor = obs_as_tensor(observation, self.device)
        with th.no_grad():
            actions = self._predict(obs_tensor, deterministic=deterministic)
        actions = actions.cpu().numpy()
        if isinstance(self.action_space, spaces.Box):
            if self.squash_output:
                actions = self.unscale_action(actions)
            else:
                actions = np.clip(actions, np.concatenate([self.action_space.low] * self.num_agents),
                                  np.concatenate([self.action_space.high] * self.num_agents))
        return actions, state

    @classmethod
    def load(cls, observation_overide, action_overide, num_agents, path: str, device: Union[th.device, str] = "auto"):
        import json

        from imitation_amd.rl import save_util

        device = get_device(device)
        saved = th.load(path, map_location=device, weights_only=True)
        data = save_util._decode(json.loads(saved["data"])) if isinstance(saved.get("data"), str) else saved["data"]
        for k in ("observation_overide", "action_overide", "num_agents"):
            data.pop(k, None)
        data["lr_schedule"] = lambda _: 0.0
        data = {k: v for k, v in data.items() if v is not None}
        model = cls(observation_overide, action_overide, num_agents, **data)
        model.load_state_dict(saved["state_dict"])
        model.to(device)
        return model


class NonTrainablePolicy(policies.BasePolicy, abc.ABC):
    """Abstract policy for non-trainable policies."""

    def __init__(self, observation_space: spaces.Space, action_space: spaces.Space):
        super().__init__(observation_space=observation_space, action_space=action_space)

    def _predict(self, obs, deterministic: bool = False):
        if isinstance(obs, dict):
            np_obs = types.DictObs({k: v.detach().cpu().numpy() for k, v in obs.items()})
        else:
            np_obs = obs.detach().cpu().numpy()
        actions = []
        for ob in np_obs:
            ob_u = types.maybe_unwrap_dictobs(ob)
            assert self.observation_space.contains(ob_u)
            actions.append(self._choose_action(ob_u))
        return th.as_tensor(np.stack(actions, axis=0), device=self.device)

    @abc.abstractmethod
    def _choose_action(self, obs) -> np.ndarray:
        """Choose an action for a single observation."""

    def forward(self, *args):
        raise NotImplementedError  # pragma: no cover


class RandomPolicy(NonTrainablePolicy):
    """Returns random actions."""

    def _choose_action(self, obs) -> np.ndarray:
        return self.action_space.sample()


class ZeroPolicy(NonTrainablePolicy):
    """Returns constant zero action."""

    def __init__(self, observation_space: spaces.Space, action_space: spaces.Space):
        super().__init__(observation_space, action_space)
        self._zero_action = np.zeros_like(action_space.sample(), dtype=action_space.dtype)
        if self._zero_action not in action_space:
            raise ValueError(f"Zero action {self._zero_action} not in action space {action_space}")

    def _choose_action(self, obs) -> np.ndarray:
        return self._zero_action


class FeedForward32Policy(policies.ActorCriticPolicy):
    """Actor-critic with two 32-unit hidden layers for both pi and vf (fused MFMA heads on GPU)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs, net_arch=[32, 32])


class HomogenousFeedForward32Policy(HomogenousActorCriticPolicy):
    """Homogeneous multi-agent actor-critic with ``net_arch=[256, 256, 128]`` (fork addition)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs, net_arch=[256, 256, 128])


class SAC1024Policy(SACPolicy):
    """SAC actor-critic with two 1024-unit hidden layers."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs, net_arch=[1024, 1024])


class NormalizeFeaturesExtractor(FlattenExtractor):
    """Flatten then normalise features (RunningNorm by default); folded into the fused MLP on GPU."""

    def __init__(self, observation_space: spaces.Space, normalize_class: Type[nn.Module] = networks.RunningNorm):
        super().__init__(observation_space)
        self.normalize = normalize_class(self.features_dim)  # type: ignore[call-arg]

    def forward(self, observations: th.Tensor) -> th.Tensor:
        return self.normalize(super().forward(observations))

"""Observation/action preprocessing (the SB3 ``preprocessing`` surface the reference uses).

``preprocess_obs`` (one-hot Discrete, /255 images), ``get_flattened_obs_dim``,
``is_image_space``, ``get_action_dim`` -- used by the reference at
``src/imitation/rewards/reward_nets.py:88-111, 416-424, 508``.
"""

from __future__ import annotations

from typing import Dict, Union

import numpy as np
import torch as th
import torch.nn.functional as F

from imitation_amd.envs import spaces
from imitation_amd.envs.spaces import (  # noqa: F401  (re-exported)
    get_action_dim,
    get_flattened_obs_dim,
    get_obs_shape,
    is_image_space,
    is_image_space_channels_first,
)


def maybe_transpose(observation: np.ndarray, observation_space: spaces.Space) -> np.ndarray:
    """HWC -> CHW for image observations that are channel-last."""
    if is_image_space(observation_space):
        if not (observation.shape == observation_space.shape or observation.shape[1:] == observation_space.shape):
            transpose_obs = np.transpose(observation, (0, 3, 1, 2)) if observation.ndim == 4 else np.transpose(
                observation, (2, 0, 1)
            )
            return transpose_obs
    return observation


def preprocess_obs(
    obs: Union[th.Tensor, Dict[str, th.Tensor]],
    observation_space: spaces.Space,
    normalize_images: bool = True,
) -> Union[th.Tensor, Dict[str, th.Tensor]]:
    if isinstance(observation_space, spaces.Dict):
        assert isinstance(obs, dict)
        return {k: preprocess_obs(obs[k], sub, normalize_images) for k, sub in observation_space.spaces.items()}
    assert isinstance(obs, th.Tensor)
    if isinstance(observation_space, spaces.Box):
        if normalize_images and is_image_space(observation_space):
            return obs.float() / 255.0
        return obs.float()
    if isinstance(observation_space, spaces.Discrete):
        return F.one_hot(obs.long().reshape(-1), num_classes=int(observation_space.n)).float()
    if isinstance(observation_space, spaces.MultiDiscrete):
        nvec = [int(n) for n in observation_space.nvec]
        o = obs.long().reshape(-1, len(nvec))
        return th.cat([F.one_hot(o[:, i], num_classes=n).float() for i, n in enumerate(nvec)], dim=-1)
    if isinstance(observation_space, spaces.MultiBinary):
        return obs.float()
    raise NotImplementedError(f"Preprocessing not implemented for {observation_space}")


def check_for_nested_spaces(obs_space: spaces.Space) -> None:
    if isinstance(obs_space, spaces.Dict):
        for sub in obs_space.spaces.values():
            if isinstance(sub, (spaces.Dict, spaces.Tuple)):
                raise NotImplementedError("Nested observation spaces are not supported")

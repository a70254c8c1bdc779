"""Human-in-the-loop discrete policies (reference: src/imitation/policies/interactive.py).

Each query renders the observation and reads an action key from stdin; used with
DAgger's ``InteractiveTrajectoryCollector`` for interactive demonstrations.
"""

from __future__ import annotations

import abc
import collections
from typing import Dict, Optional, Union

import numpy as np

from imitation_amd.envs import spaces
from imitation_amd.policies import base as base_policies
from imitation_amd.util import util


class DiscreteInteractivePolicy(base_policies.NonTrainablePolicy, abc.ABC):
    """Renders each observation and maps a typed key to a discrete action index."""

    def __init__(self, observation_space: spaces.Space, action_space: spaces.Space,
                 action_keys_names: "collections.OrderedDict[str, str]", clear_screen_on_query: bool = True):
        super().__init__(observation_space=observation_space, action_space=action_space)
        assert isinstance(action_space, spaces.Discrete)
        assert len(action_keys_names) == len(set(action_keys_names.values())) == action_space.n
        self.action_keys_names = action_keys_names
        self.action_key_to_index = {k: i for i, k in enumerate(action_keys_names.keys())}
        self.clear_screen_on_query = clear_screen_on_query

    def _choose_action(self, obs: Union[np.ndarray, Dict[str, np.ndarray]]) -> np.ndarray:
        if self.clear_screen_on_query:
            util.clear_screen()
        if isinstance(obs, dict):
            raise ValueError("Dictionary observations are not supported here")
        context = self._render(obs)
        key = self._get_input_key()
        self._clean_up(context)
        return np.array([self.action_key_to_index[key]])

    def _get_input_key(self) -> str:
        print("Please select an action. Possible choices in [ACTION_NAME:KEY] format:",
              ", ".join(f"{n}:{k}" for k, n in self.action_keys_names.items()))
        key = input("Your choice (enter key):")
        while key not in self.action_keys_names:
            key = input("Invalid key, please try again! Your choice (enter key):")
        return key

    @abc.abstractmethod
    def _render(self, obs: np.ndarray) -> Optional[object]:
        """Render ``obs``; may return a context handed to :meth:`_clean_up`."""

    def _clean_up(self, context: object) -> None:
        """Undo whatever :meth:`_render` showed."""


class ImageObsDiscreteInteractivePolicy(DiscreteInteractivePolicy):
    """Shows image observations in a matplotlib window."""

    def _render(self, obs: np.ndarray):
        import matplotlib.pyplot as plt

        fig, ax = plt.subplots()
        ax.imshow(self._prepare_obs_image(obs), cmap="gray", vmin=0, vmax=255)
        ax.axis("off")
        fig.show()
        return fig

    def _clean_up(self, context) -> None:
        import matplotlib.pyplot as plt

        plt.close(context)

    def _prepare_obs_image(self, obs: np.ndarray) -> np.ndarray:
        return obs


ATARI_ACTION_NAMES_TO_KEYS = {
    "NOOP": "1", "FIRE": "2", "UP": "w", "RIGHT": "d", "LEFT": "a", "DOWN": "x", "UPRIGHT": "e", "UPLEFT": "q",
    "DOWNRIGHT": "c", "DOWNLEFT": "z", "UPFIRE": "t", "RIGHTFIRE": "h", "LEFTFIRE": "f", "DOWNFIRE": "b",
    "UPRIGHTFIRE": "y", "UPLEFTFIRE": "r", "DOWNRIGHTFIRE": "n", "DOWNLEFTFIRE": "v",
}

# Minimal Pong action set (ALE ``get_action_meanings`` for Pong), used by the native
# synthetic Pong env which has no ALE behind it.
PONG_ACTION_MEANINGS = ["NOOP", "FIRE", "RIGHT", "LEFT", "RIGHTFIRE", "LEFTFIRE"]


class AtariInteractivePolicy(ImageObsDiscreteInteractivePolicy):
    """Interactive policy for Atari-style envs (keys from ``ATARI_ACTION_NAMES_TO_KEYS``)."""

    def __init__(self, env, *args, **kwargs):
        if hasattr(env, "get_action_meanings"):
            names = env.get_action_meanings()
        elif hasattr(env, "env_method"):
            try:
                names = env.env_method("get_action_meanings", indices=[0])[0]
            except Exception:
                names = PONG_ACTION_MEANINGS[: env.action_space.n]
        else:
            names = PONG_ACTION_MEANINGS[: env.action_space.n]
        keys = collections.OrderedDict((ATARI_ACTION_NAMES_TO_KEYS[n], n) for n in names)
        super().__init__(env.observation_space, env.action_space, keys, *args, **kwargs)

    def _prepare_obs_image(self, obs: np.ndarray) -> np.ndarray:
        # frame-stacked HWC: show the newest frame
        return obs[..., -1] if obs.ndim == 3 and obs.shape[-1] > 3 else obs

"""Partially randomised policy (reference: src/imitation/policies/exploration_wrapper.py).

Switches between the wrapped policy and uniform-random actions: after every call
the current policy is kept with probability ``1 - switch_prob``; on a switch the
random policy is chosen with probability ``random_prob``. Random actions for the
whole batch come from one vectorised space sample per env.
"""

from __future__ import annotations

from typing import Dict, Optional, Tuple, Union

import numpy as np

from imitation_amd.data import rollout
from imitation_amd.util import util


class ExplorationWrapper:
    def __init__(self, policy: rollout.AnyPolicy, venv, random_prob: float, switch_prob: float, rng: np.random.Generator,
                 deterministic_policy: bool = False):
        policy_callable = rollout.policy_to_callable(policy, venv, deterministic_policy)
        self.wrapped_policy = policy_callable
        self.random_prob = random_prob
        self.switch_prob = switch_prob
        self.venv = venv
        self.rng = rng
        self.venv.action_space.seed(util.make_seeds(self.rng))
        self.current_policy = policy_callable
        self._switch()

    def _random_policy(self, obs, state, episode_start):
        del state, episode_start
        n = len(obs) if not isinstance(obs, dict) else len(next(iter(obs.values())))
        return np.stack([self.venv.action_space.sample() for _ in range(n)], axis=0), None

    def _switch(self) -> None:
        self.current_policy = self._random_policy if self.rng.random() < self.random_prob else self.wrapped_policy

    def __call__(self, observation: Union[np.ndarray, Dict[str, np.ndarray]], input_state: Optional[Tuple[np.ndarray, ...]],
                 episode_start: Optional[np.ndarray]) -> Tuple[np.ndarray, Optional[Tuple[np.ndarray, ...]]]:
        del episode_start
        if input_state is not None:
            raise ValueError("Exploration wrapper does not support stateful policies.")
        acts, output_state = self.current_policy(observation, None, None)
        if output_state is not None:
            raise ValueError("Exploration wrapper does not support stateful policies.")
        if self.rng.random() < self.switch_prob:
            self._switch()
        return acts, None

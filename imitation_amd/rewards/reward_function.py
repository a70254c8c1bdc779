"""Reward-function protocol (reference: ``src/imitation/rewards/reward_function.py:9-34``)."""

from __future__ import annotations

import abc

import numpy as np


class RewardFn(abc.ABC):
    """``(state, action, next_state, done) -> rewards`` over a batch (shape ``(B,)``)."""

    @abc.abstractmethod
    def __call__(self, state: np.ndarray, action: np.ndarray, next_state: np.ndarray, done: np.ndarray) -> np.ndarray:
        """Compute rewards for a batch of transitions."""

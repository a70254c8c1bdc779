"""Statistical "did it learn" checks (reference: src/imitation/testing/reward_improvement.py).

The permutation test is computed exactly-enough with a vectorised Monte-Carlo over
label shuffles (numpy, one matrix op) instead of scipy's generic routine.
"""

from __future__ import annotations

from typing import Iterable

import numpy as np


def _perm_pvalue(old: np.ndarray, new: np.ndarray, n_resamples: int = 9999, seed: int = 0) -> float:
    """One-sided p-value of H0: mean(new) <= mean(old) by label permutation."""
    pooled = np.concatenate([old, new])
    n_old = len(old)
    observed = new.mean() - old.mean()
    rng = np.random.default_rng(seed)
    keys = rng.random((n_resamples, len(pooled)))
    perms = np.argsort(keys, axis=1)
    shuffled = pooled[perms]
    stat = shuffled[:, n_old:].mean(axis=1) - shuffled[:, :n_old].mean(axis=1)
    # include the observed arrangement (as scipy does) so p > 0
    return float((np.sum(stat >= observed - 1e-12) + 1) / (n_resamples + 1))


def is_significant_reward_improvement(old_rewards: Iterable[float], new_rewards: Iterable[float],
                                      p_value: float = 0.05) -> bool:
    """True if the new returns are better than the old ones with significance ``p_value``.

    >>> is_significant_reward_improvement((5, 6, 7, 4, 4), (7, 5, 9, 9, 12))
    True
    >>> is_significant_reward_improvement((5, 6, 7, 4, 4), (7, 5, 9, 7, 4))
    False
    >>> is_significant_reward_improvement((5, 6, 7, 4, 4), (7, 5, 9, 7, 4), p_value=0.3)
    True
    """
    old = np.asarray(list(old_rewards), dtype=np.float64)
    new = np.asarray(list(new_rewards), dtype=np.float64)
    return _perm_pvalue(old, new) < p_value


def mean_reward_improved_by(old_rews: Iterable[float], new_rews: Iterable[float], min_improvement: float) -> bool:
    """True if ``mean(new) - mean(old) >= min_improvement``."""
    return float(np.mean(list(new_rews)) - np.mean(list(old_rews))) >= min_improvement

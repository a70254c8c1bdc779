"""Aggregate metrics with stratified bootstrap confidence intervals (the ``rliable``
estimators the reference's benchmark summary uses, re-implemented in numpy; rliable
is not part of the image).

Score matrices are ``[n_runs, n_tasks]``. The bootstrap resamples runs independently
within each task (stratified), vectorised over all repetitions at once.
"""

from __future__ import annotations

from typing import Callable, Dict, Tuple

import numpy as np
from scipy import stats as sps


def aggregate_mean(scores: np.ndarray) -> float:
    return float(np.mean(scores))


def aggregate_median(scores: np.ndarray) -> float:
    return float(np.median(np.mean(scores, axis=0)))


def aggregate_iqm(scores: np.ndarray) -> float:
    """Interquartile mean over all run x task scores (25% trimmed mean)."""
    return float(sps.trim_mean(scores, proportiontocut=0.25, axis=None))


def aggregate_optimality_gap(scores: np.ndarray, gamma: float = 1.0) -> float:
    return float(gamma - np.mean(np.minimum(scores, gamma)))


def probability_of_improvement(scores_x: np.ndarray, scores_y: np.ndarray) -> float:
    """P(X > Y) averaged over tasks (Mann-Whitney U statistic per task, ties count half)."""
    assert scores_x.shape[1] == scores_y.shape[1]
    probs = []
    for t in range(scores_x.shape[1]):
        x = scores_x[:, t][:, None]
        y = scores_y[:, t][None, :]
        probs.append(np.mean((x > y) + 0.5 * (x == y)))
    return float(np.mean(probs))


def _stratified_resample(scores: np.ndarray, rng: np.random.Generator, reps: int) -> np.ndarray:
    n, t = scores.shape
    idx = rng.integers(0, n, size=(reps, n, t))
    return np.take_along_axis(np.broadcast_to(scores, (reps, n, t)), idx, axis=1)


def get_interval_estimates(score_dict: Dict[str, np.ndarray], func: Callable[[np.ndarray], np.ndarray],
                           reps: int = 2000, confidence_interval_size: float = 0.95,
                           seed: int = 0) -> Tuple[Dict[str, np.ndarray], Dict[str, np.ndarray]]:
    """Point estimates ``func(scores)`` and percentile-bootstrap CIs ``[2, n_metrics]`` per key.

    Values may also be ``(scores_x, scores_y)`` pairs for two-sample metrics.
    """
    rng = np.random.default_rng(seed)
    point, cis = {}, {}
    lo_q, hi_q = 100 * (1 - confidence_interval_size) / 2, 100 * (1 + confidence_interval_size) / 2
    for k, s in score_dict.items():
        if isinstance(s, tuple):
            x, y = s
            point[k] = np.atleast_1d(func(x, y))
            bx, by = _stratified_resample(x, rng, reps), _stratified_resample(y, rng, reps)
            boots = np.array([np.atleast_1d(func(bx[i], by[i])) for i in range(reps)])
        else:
            point[k] = np.atleast_1d(func(s))
            bs = _stratified_resample(s, rng, reps)
            boots = np.array([np.atleast_1d(func(bs[i])) for i in range(reps)])
        cis[k] = np.percentile(boots, [lo_q, hi_q], axis=0)
    return point, cis

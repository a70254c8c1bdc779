"""Action noise for deterministic off-policy actors (SB3 ``common/noise.py`` semantics):
Gaussian and Ornstein-Uhlenbeck processes over the scaled ``[-1, 1]`` action box, drawn on the
host (one vector per environment step, added in ``OffPolicyAlgorithm._sample_action``)."""

from __future__ import annotations

from typing import Optional

import numpy as np


class ActionNoise:
    def reset(self, indices=None) -> None:  # (indices: VectorizedActionNoise's per-env reset)
        pass

    def __call__(self) -> np.ndarray:
        raise NotImplementedError


class NormalActionNoise(ActionNoise):
    def __init__(self, mean: np.ndarray, sigma: np.ndarray, dtype=np.float32, rng: Optional[np.random.Generator] = None):
        self._mu = np.asarray(mean, dtype)
        self._sigma = np.asarray(sigma, dtype)
        self._dtype = dtype
        self._rng = rng or np.random.default_rng()

    def __call__(self) -> np.ndarray:
        return self._rng.normal(self._mu, self._sigma).astype(self._dtype)

    def __repr__(self) -> str:
        return f"NormalActionNoise(mu={self._mu}, sigma={self._sigma})"


class OrnsteinUhlenbeckActionNoise(ActionNoise):
    """Temporally correlated noise ``x += theta (mu - x) dt + sigma sqrt(dt) N(0, 1)``."""

    def __init__(self, mean: np.ndarray, sigma: np.ndarray, theta: float = 0.15, dt: float = 1e-2,
                 initial_noise: Optional[np.ndarray] = None, dtype=np.float32, rng: Optional[np.random.Generator] = None):
        self._mu = np.asarray(mean, dtype)
        self._sigma = np.asarray(sigma, dtype)
        self._theta = theta
        self._dt = dt
        self._dtype = dtype
        self._rng = rng or np.random.default_rng()
        self.initial_noise = initial_noise
        self.reset()

    def __call__(self) -> np.ndarray:
        x = (self.noise_prev + self._theta * (self._mu - self.noise_prev) * self._dt
             + self._sigma * np.sqrt(self._dt) * self._rng.normal(size=self._mu.shape))
        self.noise_prev = x
        return x.astype(self._dtype)

    def reset(self, indices=None) -> None:
        self.noise_prev = self.initial_noise if self.initial_noise is not None else np.zeros_like(self._mu)

    def __repr__(self) -> str:
        return f"OrnsteinUhlenbeckActionNoise(mu={self._mu}, sigma={self._sigma})"


class VectorizedActionNoise(ActionNoise):
    """One independent copy of ``base_noise`` per environment: returns ``[n_envs, action_dim]``."""

    def __init__(self, base_noise: ActionNoise, n_envs: int):
        import copy

        self.n_envs = int(n_envs)
        self.noises = [copy.deepcopy(base_noise) for _ in range(self.n_envs)]

    def reset(self, indices=None) -> None:
        for i in (range(self.n_envs) if indices is None else indices):
            self.noises[i].reset()

    def __call__(self) -> np.ndarray:
        return np.stack([n() for n in self.noises])

"""Observation / action spaces.

The reference delegates spaces to ``gymnasium.spaces`` (used everywhere, e.g.
``src/imitation/data/rollout.py:345-378`` space checks,
``src/imitation/rewards/reward_nets.py:416-424`` flattening). gymnasium is not
available here, so this module provides a self-contained, numpy-backed
implementation with the subset of behaviour the framework relies on:
``shape``/``dtype``/``sample``/``contains``/``seed`` plus ``flatdim``/``flatten``
helpers and ``is_image_space`` (SB3 ``preprocessing`` semantics).
"""

from __future__ import annotations

import collections
from typing import Any, Dict, Mapping, Optional, Sequence, Tuple, Union

import numpy as np


class Space:
    """Base class for spaces."""

    def __init__(self, shape: Optional[Tuple[int, ...]] = None, dtype=None, seed=None):
        self._shape = None if shape is None else tuple(int(s) for s in shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self._np_random: Optional[np.random.Generator] = None
        if seed is not None:
            self.seed(seed)

    @property
    def shape(self) -> Optional[Tuple[int, ...]]:
        return self._shape

    @property
    def np_random(self) -> np.random.Generator:
        if self._np_random is None:
            self._np_random = np.random.default_rng()
        return self._np_random

    def seed(self, seed: Optional[int] = None):
        self._np_random = np.random.default_rng(seed)
        return [seed]

    def sample(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def contains(self, x) -> bool:  # pragma: no cover - abstract
        raise NotImplementedError

    def __contains__(self, x) -> bool:
        return self.contains(x)

    def __getstate__(self):
        state = dict(self.__dict__)
        state["_np_random"] = None
        return state


class Box(Space):
    """A (possibly unbounded) box in R^n."""

    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        dtype = np.dtype(dtype)
        if shape is None:
            low_a = np.asarray(low)
            high_a = np.asarray(high)
            shape = low_a.shape if low_a.shape else high_a.shape
        shape = tuple(int(s) for s in shape)
        super().__init__(shape, dtype, seed)

        def _cast(v, fill):
            v = np.asarray(v, dtype=np.float64) if not np.issubdtype(np.asarray(v).dtype, np.integer) else np.asarray(v)
            if np.issubdtype(dtype, np.integer) and v.dtype.kind == "f":
                info = np.iinfo(dtype)  # unbounded integer boxes clamp to the dtype range (as gymnasium)
                v = np.broadcast_to(v, shape)
                out = np.zeros(shape, dtype=dtype)
                fin = np.isfinite(v)
                out[fin] = v[fin].astype(dtype)
                out[np.isposinf(v)] = info.max
                out[np.isneginf(v)] = info.min
                return out
            return np.broadcast_to(v.astype(dtype), shape).copy()

        self.low = _cast(low, -np.inf)
        self.high = _cast(high, np.inf)

    @property
    def bounded_below(self):
        return self.low > -np.inf

    @property
    def bounded_above(self):
        return self.high < np.inf

    def is_bounded(self, manner: str = "both") -> bool:
        below = bool(np.all(self.bounded_below))
        above = bool(np.all(self.bounded_above))
        return {"both": below and above, "below": below, "above": above}[manner]

    def sample(self):
        rng = self.np_random
        if np.issubdtype(self.dtype, np.integer):
            return rng.integers(self.low, self.high.astype(np.int64) + 1, size=self.shape).astype(self.dtype)
        low = np.where(np.isfinite(self.low), self.low, -1.0)
        high = np.where(np.isfinite(self.high), self.high, 1.0)
        unb_l = ~np.isfinite(self.low)
        unb_h = ~np.isfinite(self.high)
        x = rng.uniform(low, high, size=self.shape)
        both = unb_l & unb_h
        if both.any():
            x[both] = rng.normal(size=both.sum())
        lo_only = unb_l & ~unb_h
        if lo_only.any():
            x[lo_only] = self.high[lo_only] - rng.exponential(size=lo_only.sum())
        hi_only = unb_h & ~unb_l
        if hi_only.any():
            x[hi_only] = self.low[hi_only] + rng.exponential(size=hi_only.sum())
        return x.astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        if x.shape != self.shape:
            return False
        if np.issubdtype(self.dtype, np.integer) and not np.issubdtype(x.dtype, np.integer):
            return False
        return bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"

    def __eq__(self, other):
        return (
            isinstance(other, Box)
            and self.shape == other.shape
            and self.dtype == other.dtype
            and np.allclose(self.low, other.low)
            and np.allclose(self.high, other.high)
        )

    __hash__ = object.__hash__


class Discrete(Space):
    """Integers in ``[start, start + n)``."""

    def __init__(self, n: int, seed=None, start: int = 0):
        super().__init__((), np.int64, seed)
        self.n = int(n)
        self.start = int(start)

    def sample(self):
        return np.int64(self.start + self.np_random.integers(self.n))

    def contains(self, x) -> bool:
        if isinstance(x, (int, np.integer)):
            v = int(x)
        elif isinstance(x, np.ndarray) and x.shape == () and np.issubdtype(x.dtype, np.integer):
            v = int(x)
        else:
            return False
        return self.start <= v < self.start + self.n

    def __repr__(self):
        return f"Discrete({self.n})" if self.start == 0 else f"Discrete({self.n}, start={self.start})"

    def __eq__(self, other):
        return isinstance(other, Discrete) and self.n == other.n and self.start == other.start

    __hash__ = object.__hash__


class MultiDiscrete(Space):
    """A vector of discrete variables with per-entry cardinality ``nvec``."""

    def __init__(self, nvec, dtype=np.int64, seed=None):
        self.nvec = np.asarray(nvec, dtype=np.int64)
        super().__init__(self.nvec.shape, dtype, seed)

    def sample(self):
        return (self.np_random.random(self.nvec.shape) * self.nvec).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= 0) and np.all(x < self.nvec))

    def __repr__(self):
        return f"MultiDiscrete({self.nvec})"

    def __eq__(self, other):
        return isinstance(other, MultiDiscrete) and np.array_equal(self.nvec, other.nvec)

    __hash__ = object.__hash__


class MultiBinary(Space):
    def __init__(self, n, seed=None):
        self.n = n
        shape = (int(n),) if np.isscalar(n) else tuple(int(v) for v in n)
        super().__init__(shape, np.int8, seed)

    def sample(self):
        return self.np_random.integers(0, 2, size=self.shape, dtype=np.int8)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all((x == 0) | (x == 1)))

    def __eq__(self, other):
        return isinstance(other, MultiBinary) and self.shape == other.shape

    __hash__ = object.__hash__


class Dict(Space, Mapping):
    """An ordered dictionary of sub-spaces."""

    def __init__(self, spaces: Union[None, Mapping[str, Space], Sequence[Tuple[str, Space]]] = None, seed=None, **kwargs):
        if spaces is None:
            spaces = {}
        if not isinstance(spaces, Mapping):
            spaces = collections.OrderedDict(spaces)
        spaces = dict(spaces)
        spaces.update(kwargs)
        self.spaces: Dict[str, Space] = dict(spaces)
        super().__init__(None, None, seed)

    def seed(self, seed=None):
        super().seed(seed)
        for i, sp in enumerate(self.spaces.values()):
            sp.seed(None if seed is None else seed + i)
        return [seed]

    def sample(self):
        return {k: sp.sample() for k, sp in self.spaces.items()}

    def contains(self, x) -> bool:
        if not isinstance(x, Mapping) or set(x.keys()) != set(self.spaces.keys()):
            return False
        return all(sp.contains(x[k]) for k, sp in self.spaces.items())

    def __getitem__(self, key):
        return self.spaces[key]

    def __iter__(self):
        return iter(self.spaces)

    def __len__(self):
        return len(self.spaces)

    def keys(self):
        return self.spaces.keys()

    def items(self):
        return self.spaces.items()

    def values(self):
        return self.spaces.values()

    def __repr__(self):
        return "Dict(" + ", ".join(f"{k!r}: {v}" for k, v in self.spaces.items()) + ")"

    def __eq__(self, other):
        return isinstance(other, Dict) and self.spaces == other.spaces

    __hash__ = object.__hash__


class Tuple(Space):
    def __init__(self, spaces: Sequence[Space], seed=None):
        self.spaces = tuple(spaces)
        super().__init__(None, None, seed)

    def sample(self):
        return tuple(sp.sample() for sp in self.spaces)

    def contains(self, x) -> bool:
        return isinstance(x, (tuple, list)) and len(x) == len(self.spaces) and all(
            sp.contains(v) for sp, v in zip(self.spaces, x)
        )

    def __getitem__(self, i):
        return self.spaces[i]

    def __len__(self):
        return len(self.spaces)

    def __eq__(self, other):
        return isinstance(other, Tuple) and self.spaces == other.spaces

    __hash__ = object.__hash__


# --------------------------------------------------------------------------- helpers
def flatdim(space: Space) -> int:
    """Number of features after ``flatten`` (Discrete → one-hot)."""
    if isinstance(space, Box):
        return int(np.prod(space.shape))
    if isinstance(space, Discrete):
        return space.n
    if isinstance(space, MultiDiscrete):
        return int(space.nvec.sum())
    if isinstance(space, MultiBinary):
        return int(np.prod(space.shape))
    if isinstance(space, Dict):
        return sum(flatdim(s) for s in space.spaces.values())
    if isinstance(space, Tuple):
        return sum(flatdim(s) for s in space.spaces)
    raise NotImplementedError(f"flatdim not supported for {space}")


def flatten(space: Space, x) -> np.ndarray:
    if isinstance(space, Box):
        return np.asarray(x, dtype=space.dtype).reshape(-1)
    if isinstance(space, Discrete):
        out = np.zeros(space.n, dtype=np.float32)
        out[int(x) - space.start] = 1
        return out
    if isinstance(space, MultiDiscrete):
        parts = []
        for v, n in zip(np.asarray(x).reshape(-1), space.nvec.reshape(-1)):
            o = np.zeros(n, dtype=np.float32)
            o[int(v)] = 1
            parts.append(o)
        return np.concatenate(parts)
    if isinstance(space, MultiBinary):
        return np.asarray(x, dtype=np.float32).reshape(-1)
    if isinstance(space, Dict):
        return np.concatenate([flatten(s, x[k]) for k, s in space.spaces.items()])
    if isinstance(space, Tuple):
        return np.concatenate([flatten(s, v) for s, v in zip(space.spaces, x)])
    raise NotImplementedError


def get_obs_shape(space: Space):
    """SB3 ``preprocessing.get_obs_shape`` semantics."""
    if isinstance(space, Box):
        return space.shape
    if isinstance(space, Discrete):
        return (1,)
    if isinstance(space, MultiDiscrete):
        return (int(len(space.nvec)),)
    if isinstance(space, MultiBinary):
        return space.shape
    if isinstance(space, Dict):
        return {k: get_obs_shape(s) for k, s in space.spaces.items()}
    raise NotImplementedError(space)


def get_flattened_obs_dim(space: Space) -> int:
    """Feature dimension after ``preprocess_obs`` + flatten."""
    if isinstance(space, MultiDiscrete):
        return int(space.nvec.sum())
    return flatdim(space)


def get_action_dim(space: Space) -> int:
    if isinstance(space, Box):
        return int(np.prod(space.shape))
    if isinstance(space, Discrete):
        return 1
    if isinstance(space, MultiDiscrete):
        return int(len(space.nvec))
    if isinstance(space, MultiBinary):
        return int(np.prod(space.shape))
    raise NotImplementedError(space)


def is_image_space(space: Space, check_channels: bool = False, normalized_image: bool = False) -> bool:
    """True for uint8 Box spaces of rank 3 in [0, 255] (SB3 convention)."""
    if isinstance(space, Box) and len(space.shape) == 3:
        if normalized_image:
            return True
        if space.dtype != np.uint8:
            return False
        if np.any(space.low != 0) or np.any(space.high != 255):
            return False
        if not check_channels:
            return True
        n_channels = space.shape[0] if is_image_space_channels_first(space) else space.shape[-1]
        return n_channels in (1, 3, 4)
    return False


def is_image_space_channels_first(space: Box) -> bool:
    smallest = int(np.argmin(space.shape))
    return smallest == 0


__all__ = [
    "Space",
    "Box",
    "Discrete",
    "MultiDiscrete",
    "MultiBinary",
    "Dict",
    "Tuple",
    "flatdim",
    "flatten",
    "get_obs_shape",
    "get_flattened_obs_dim",
    "get_action_dim",
    "is_image_space",
    "is_image_space_channels_first",
]

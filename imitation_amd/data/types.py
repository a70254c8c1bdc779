"""Trajectory / transition containers (reference: ``src/imitation/data/types.py``).

Frozen dataclasses with the reference's validation rules:

* :class:`DictObs` (``types.py:38-202``) -- dict-of-arrays observation with
  array-like len/index/iter and stack/concatenate helpers;
* :class:`Trajectory` (``:336-416``): ``len(obs) == len(acts) + 1``, optional
  per-step ``infos``, ``terminal`` flag, ``__setstate__`` back-compat;
* :class:`TrajectoryWithRew` (``:430-439``);
* :class:`TransitionsMinimal` / :class:`Transitions` / :class:`TransitionsWithRew`
  (``:481-638``): torch ``Dataset``s, read-only arrays, int index -> dict,
  slice -> same dataclass;
* :func:`transitions_collate_fn` (``:447-474``), :func:`dataclass_quick_asdict`.

Extra on this framework: :meth:`TransitionsMinimal.to_device` packs the numeric
fields into device tensors once, so training loops can keep demonstrations
resident in HBM instead of re-copying every minibatch (the reference converts per
batch, ``algorithms/bc.py:490-494``).
"""

from __future__ import annotations

import collections
import dataclasses
import itertools
import numbers
import os
import warnings
from typing import Any, Callable, Dict, Iterable, Iterator, List, Mapping, Optional, Sequence, Tuple, TypeVar, Union

import numpy as np
import torch as th
from torch.utils import data as th_data

try:  # TypedDict is in typing for py>=3.8
    from typing import TypedDict
except ImportError:  # pragma: no cover
    from typing_extensions import TypedDict

T = TypeVar("T")
AnyPath = Union[str, bytes, os.PathLike]
AnyTensor = Union[np.ndarray, th.Tensor]
TensorVar = TypeVar("TensorVar", np.ndarray, th.Tensor)


@dataclasses.dataclass(frozen=True)
class DictObs:
    """Observations of a ``Dict`` observation space, indexed like one array."""

    _d: Dict[str, np.ndarray]

    @classmethod
    def from_obs_list(cls, obs_list: List[Dict[str, np.ndarray]]) -> "DictObs":
        return cls.stack(map(cls, obs_list))

    def __post_init__(self):
        if not all(isinstance(v, (np.ndarray, numbers.Number)) for v in self._d.values()):
            raise TypeError("Values must be NumPy arrays")

    def __len__(self):
        lens = {len(v) for v in self._d.values()}
        if len(lens) == 1:
            return lens.pop()
        if not lens:
            raise RuntimeError("Length not defined as DictObs is empty")
        raise RuntimeError(f"Length not defined; arrays have conflicting first dimensions: {lens}")

    @property
    def dict_len(self):
        return len(self._d)

    def __getitem__(self, key) -> "DictObs":
        return self.__class__({k: np.asarray(v[key]) for k, v in self._d.items()})

    def __iter__(self) -> Iterator["DictObs"]:
        return (self[i] for i in range(len(self)))

    def __eq__(self, other):
        if not isinstance(other, self.__class__):
            return False
        if self.keys() != other.keys():
            return False
        return all(np.array_equal(self.get(k), other.get(k)) for k in self.keys())

    @property
    def shape(self) -> Dict[str, Tuple[int, ...]]:
        return {k: v.shape for k, v in self.items()}

    @property
    def dtype(self) -> Dict[str, np.dtype]:
        return {k: v.dtype for k, v in self.items()}

    def keys(self):
        return self._d.keys()

    def values(self):
        return self._d.values()

    def items(self):
        return self._d.items()

    def __contains__(self, key):
        return key in self._d

    def get(self, key: str) -> np.ndarray:
        return self._d[key]

    def unwrap(self) -> Dict[str, np.ndarray]:
        return dict(self._d)

    def map_arrays(self, fn: Callable[[np.ndarray], np.ndarray]) -> "DictObs":
        return self.__class__({k: fn(v) for k, v in self.items()})

    @staticmethod
    def _unravel(dictobs_list: Iterable["DictObs"]) -> Dict[str, List[np.ndarray]]:
        it1, it2 = itertools.tee(dictobs_list)
        key_set = {frozenset(obs.keys()) for obs in it1}
        if not key_set:
            raise ValueError("Empty list of DictObs")
        if len(key_set) != 1:
            raise ValueError(f"Inconsistent keys: {key_set}")
        out: Dict[str, List[np.ndarray]] = collections.defaultdict(list)
        for ob in it2:
            for k, arr in ob._d.items():
                out[k].append(arr)
        return out

    @classmethod
    def stack(cls, dictobs_list: Iterable["DictObs"], axis=0) -> "DictObs":
        return cls({k: np.stack(v, axis=axis) for k, v in cls._unravel(dictobs_list).items()})

    @classmethod
    def concatenate(cls, dictobs_list: Iterable["DictObs"], axis=0) -> "DictObs":
        return cls({k: np.concatenate(v, axis=axis) for k, v in cls._unravel(dictobs_list).items()})


Observation = Union[np.ndarray, DictObs]
ObsVar = TypeVar("ObsVar", np.ndarray, DictObs)


def assert_not_dictobs(x: Observation) -> np.ndarray:
    assert not isinstance(x, DictObs), "Dictionary observations are not supported here."
    return x


def concatenate_maybe_dictobs(arrs: List[ObsVar]) -> ObsVar:
    assert len(arrs) > 0
    if isinstance(arrs[0], DictObs):
        return DictObs.concatenate(arrs)
    return np.concatenate(arrs)


def stack_maybe_dictobs(arrs: List[ObsVar]) -> ObsVar:
    assert len(arrs) > 0
    if isinstance(arrs[0], DictObs):
        return DictObs.stack(arrs)
    return np.stack(arrs)


def maybe_unwrap_dictobs(maybe_dictobs):
    if isinstance(maybe_dictobs, DictObs):
        return maybe_dictobs.unwrap()
    if not isinstance(maybe_dictobs, (np.ndarray, th.Tensor, int)):
        warnings.warn(f"trying to unwrap object of type {type(maybe_dictobs)}")
    return maybe_dictobs


def maybe_wrap_in_dictobs(obs):
    if isinstance(obs, dict):
        return DictObs(obs)
    if not isinstance(obs, (np.ndarray, DictObs, float, int)):
        warnings.warn(f"tried to wrap {type(obs)} as an observation")
    return obs


def map_maybe_dict(fn, maybe_dict):
    if isinstance(maybe_dict, dict):
        return {k: fn(v) for k, v in maybe_dict.items()}
    return fn(maybe_dict)


class TransitionMappingNoNextObs(TypedDict):
    obs: Union[Observation, th.Tensor]
    acts: AnyTensor


class TransitionMapping(TransitionMappingNoNextObs, total=False):
    next_obs: Union[Observation, th.Tensor]
    dones: AnyTensor
    rew: AnyTensor


def dataclass_quick_asdict(obj) -> Dict[str, Any]:
    """Shallow ``dataclasses.asdict`` (no deep copies; keeps DictObs intact)."""
    return {f.name: getattr(obj, f.name) for f in dataclasses.fields(obj)}


@dataclasses.dataclass(frozen=True)
class Trajectory:
    """One episode (or fragment): ``obs`` has one more entry than ``acts``."""

    obs: Observation
    acts: np.ndarray
    infos: Optional[np.ndarray]
    terminal: bool

    def __len__(self) -> int:
        return len(self.acts)

    def __eq__(self, other) -> bool:
        if not isinstance(other, Trajectory):
            return False
        a, b = dataclass_quick_asdict(self), dataclass_quick_asdict(other)
        if a.keys() != b.keys() or len(self) != len(other):
            return False
        for k, va in a.items():
            vb = b[k]
            if k == "infos":
                va = [{}] * len(self) if va is None else va
                vb = [{}] * len(other) if vb is None else vb
            if isinstance(va, DictObs):
                if not va == vb:
                    return False
                continue
            if not np.array_equal(va, vb):
                return False
        return True

    def __post_init__(self):
        if len(self.obs) != len(self.acts) + 1:
            raise ValueError(f"expected one more observations than actions: {len(self.obs)} != {len(self.acts)} + 1")
        if self.infos is not None and len(self.infos) != len(self.acts):
            raise ValueError(
                f"infos when present must be present for each action: {len(self.infos)} != {len(self.acts)}"
            )
        if len(self.acts) == 0:
            raise ValueError("Degenerate trajectory: must have at least one action.")

    def __setstate__(self, state):
        if "terminal" not in state:
            warnings.warn(
                "Loading old version of Trajectory.Support for this will be removed in future versions.",
                DeprecationWarning,
            )
            state["terminal"] = True
        self.__dict__.update(state)


def _rews_validation(rews: np.ndarray, acts: np.ndarray):
    if rews.shape != (len(acts),):
        raise ValueError(f"rewards must be 1D array, one entry for each action: {rews.shape} != ({len(acts)},)")
    if not np.issubdtype(rews.dtype, np.floating):
        raise ValueError(f"rewards dtype {rews.dtype} not a float")


@dataclasses.dataclass(frozen=True, eq=False)
class TrajectoryWithRew(Trajectory):
    """A :class:`Trajectory` with per-step rewards ``rews`` (float, shape ``(T,)``)."""

    rews: np.ndarray

    def __post_init__(self):
        super().__post_init__()
        _rews_validation(self.rews, self.acts)


Pair = Tuple[T, T]
TrajectoryPair = Pair[Trajectory]
TrajectoryWithRewPair = Pair[TrajectoryWithRew]


def transitions_collate_fn(batch: Sequence[Mapping[str, np.ndarray]]) -> Mapping[str, AnyTensor]:
    """DataLoader collate for transitions: default collate except ``infos`` (list) and obs (stacked)."""
    acts_dones = [{k: np.array(v) for k, v in s.items() if k in ("acts", "dones")} for s in batch]
    result = th_data.dataloader.default_collate(acts_dones)
    assert isinstance(result, dict)
    result["infos"] = [s["infos"] for s in batch]
    result["obs"] = stack_maybe_dictobs([s["obs"] for s in batch])
    result["next_obs"] = stack_maybe_dictobs([s["next_obs"] for s in batch])
    return result


TransitionsMinimalSelf = TypeVar("TransitionsMinimalSelf", bound="TransitionsMinimal")


@dataclasses.dataclass(frozen=True)
class TransitionsMinimal(th_data.Dataset, Sequence[Mapping[str, np.ndarray]]):
    """Flat batch of (obs, act, info); int index -> dict sample, slice -> same class."""

    obs: Observation
    acts: np.ndarray
    infos: np.ndarray

    def __len__(self) -> int:
        return len(self.obs)

    def __post_init__(self):
        for val in vars(self).values():
            if isinstance(val, np.ndarray):
                val.setflags(write=False)
        if len(self.obs) != len(self.acts):
            raise ValueError(f"obs and acts must have same number of timesteps: {len(self.obs)} != {len(self.acts)}")
        if len(self.infos) != len(self.obs):
            raise ValueError(f"obs and infos must have same number of timesteps: {len(self.obs)} != {len(self.infos)}")

    def __getitem__(self, key):
        d = dataclass_quick_asdict(self)
        item = {k: v[key] for k, v in d.items()}
        if isinstance(key, slice):
            return dataclasses.replace(self, **item)
        assert isinstance(key, (int, np.integer))
        return item

    def to_device(self, device, dtype=th.float32) -> Dict[str, th.Tensor]:
        """All numeric fields as contiguous device tensors (one H2D copy each)."""
        out: Dict[str, th.Tensor] = {}
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if f.name == "infos" or isinstance(v, DictObs):
                continue
            arr = np.asarray(v)
            t = th.as_tensor(np.ascontiguousarray(arr))
            if t.dtype == th.bool:
                t = t.to(dtype)
            elif t.is_floating_point():
                t = t.to(dtype)
            out[f.name] = t.to(device, non_blocking=True)
        return out


@dataclasses.dataclass(frozen=True)
class Transitions(TransitionsMinimal):
    """Batch of (obs, act, next_obs, done) transitions."""

    next_obs: Observation
    dones: np.ndarray

    def __post_init__(self):
        super().__post_init__()
        if self.obs.shape != self.next_obs.shape:
            raise ValueError(f"obs and next_obs must have same shape: {self.obs.shape} != {self.next_obs.shape}")
        if self.obs.dtype != self.next_obs.dtype:
            raise ValueError(f"obs and next_obs must have the same dtype: {self.obs.dtype} != {self.next_obs.dtype}")
        if self.dones.shape != (len(self.acts),):
            raise ValueError(
                f"dones must be 1D array, one entry for each timestep: {self.dones.shape} != ({len(self.acts)},)"
            )
        if self.dones.dtype != bool:
            raise ValueError(f"dones must be boolean, not {self.dones.dtype}")


@dataclasses.dataclass(frozen=True)
class TransitionsWithRew(Transitions):
    """Transitions with rewards."""

    rews: np.ndarray

    def __post_init__(self):
        super().__post_init__()
        _rews_validation(self.rews, self.acts)

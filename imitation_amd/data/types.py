"""Trajectory / transition containers (reference: ``src/imitation/data/types.py``).

Behaviour (validation rules, error messages, indexing semantics) follows the reference, which
users and the parity tests depend on; the implementation is this framework's own:

* :class:`DictObs` (reference ``types.py:38-202``) -- a dict of equally long arrays that
  indexes, iterates and stacks like one array. Stored as a read-only mapping behind
  ``__slots__``; stacking checks the key sets in one pass over a materialised list.
* :class:`Trajectory` / :class:`TrajectoryWithRew` (``:336-439``) -- one episode or fragment:
  ``len(obs) == len(acts) + 1``; every check is one row of the class's ``_RULES`` table.
* :class:`TransitionsMinimal` / :class:`Transitions` / :class:`TransitionsWithRew`
  (``:481-638``) -- flat torch ``Dataset`` s with read-only arrays; int index -> dict,
  slice -> same class.
* :func:`transitions_collate_fn` (``:447-474``), :func:`dataclass_quick_asdict`.

Extra on this framework: :meth:`TransitionsMinimal.to_device` packs the numeric fields into
device tensors once, so training loops keep demonstrations resident in HBM instead of
re-copying every minibatch (the reference converts per batch, ``algorithms/bc.py:490-494``).
"""

from __future__ import annotations

import dataclasses
import numbers
import os
import types as _pytypes
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


class DictObs:
    """Observations of a ``Dict`` observation space, indexed like one array: ``len`` is the shared
    leading dimension, ``obs[i]`` / ``obs[a:b]`` index every array, iteration yields rows."""

    __slots__ = ("_arrays",)

    def __init__(self, arrays: Mapping[str, np.ndarray]):
        for v in arrays.values():
            if not isinstance(v, (np.ndarray, numbers.Number)):
                raise TypeError("Values must be NumPy arrays")
        object.__setattr__(self, "_arrays", _pytypes.MappingProxyType(dict(arrays)))

    def __setattr__(self, name, value):
        raise dataclasses.FrozenInstanceError(f"cannot assign to field {name!r}")

    def __getstate__(self):
        return dict(self._arrays)

    def __setstate__(self, state):
        object.__setattr__(self, "_arrays", _pytypes.MappingProxyType(dict(state)))

    def __repr__(self) -> str:
        return f"DictObs({dict(self._arrays)!r})"

    @property
    def _d(self) -> Mapping[str, np.ndarray]:  # read-only view (name kept for code written against the reference)
        return self._arrays

    @classmethod
    def from_obs_list(cls, obs_list: List[Dict[str, np.ndarray]]) -> "DictObs":
        return cls.stack([cls(o) for o in obs_list])

    def __len__(self) -> int:
        firsts = {len(v) for v in self._arrays.values()}
        if not firsts:
            raise RuntimeError("Length not defined as DictObs is empty")
        if len(firsts) > 1:
            raise RuntimeError(f"Length not defined; arrays have conflicting first dimensions: {firsts}")
        (n,) = firsts
        return n

    @property
    def dict_len(self) -> int:
        return len(self._arrays)

    def __getitem__(self, key) -> "DictObs":
        return type(self)({k: np.asarray(v[key]) for k, v in self._arrays.items()})

    def __iter__(self) -> Iterator["DictObs"]:
        for i in range(len(self)):
            yield self[i]

    def __eq__(self, other) -> bool:
        return (isinstance(other, type(self)) and self._arrays.keys() == other._arrays.keys()
                and all(np.array_equal(v, other._arrays[k]) for k, v in self._arrays.items()))

    __hash__ = None  # mutable-array contents: not hashable (as a dataclass with eq would be)

    @property
    def shape(self) -> Dict[str, Tuple[int, ...]]:
        return {k: v.shape for k, v in self._arrays.items()}

    @property
    def dtype(self) -> Dict[str, np.dtype]:
        return {k: v.dtype for k, v in self._arrays.items()}

    def keys(self):
        return self._arrays.keys()

    def values(self):
        return self._arrays.values()

    def items(self):
        return self._arrays.items()

    def __contains__(self, key) -> bool:
        return key in self._arrays

    def get(self, key: str) -> np.ndarray:
        return self._arrays[key]

    def unwrap(self) -> Dict[str, np.ndarray]:
        return dict(self._arrays)

    def map_arrays(self, fn: Callable[[np.ndarray], np.ndarray]) -> "DictObs":
        return type(self)({k: fn(v) for k, v in self._arrays.items()})

    @classmethod
    def _join(cls, parts: Iterable["DictObs"], fn, axis: int) -> "DictObs":
        parts = list(parts)
        if not parts:
            raise ValueError("Empty list of DictObs")
        keys = frozenset(parts[0].keys())
        if any(frozenset(p.keys()) != keys for p in parts[1:]):
            raise ValueError(f"Inconsistent keys: {set(frozenset(p.keys()) for p in parts)}")
        return cls({k: fn([p._arrays[k] for p in parts], axis=axis) for k in parts[0].keys()})

    @classmethod
    def stack(cls, dictobs_list: Iterable["DictObs"], axis=0) -> "DictObs":
        return cls._join(dictobs_list, np.stack, axis)

    @classmethod
    def concatenate(cls, dictobs_list: Iterable["DictObs"], axis=0) -> "DictObs":
        return cls._join(dictobs_list, np.concatenate, axis)


Observation = Union[np.ndarray, DictObs]
ObsVar = TypeVar("ObsVar", np.ndarray, DictObs)


def assert_not_dictobs(x: Observation) -> np.ndarray:
    assert not isinstance(x, DictObs), "Dictionary observations are not supported here."
    return x


def concatenate_maybe_dictobs(arrs: List[ObsVar]) -> ObsVar:
    assert len(arrs) > 0
    return DictObs.concatenate(arrs) if isinstance(arrs[0], DictObs) else np.concatenate(arrs)


def stack_maybe_dictobs(arrs: List[ObsVar]) -> ObsVar:
    assert len(arrs) > 0
    return DictObs.stack(arrs) if isinstance(arrs[0], DictObs) else np.stack(arrs)


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
    return {k: fn(v) for k, v in maybe_dict.items()} if isinstance(maybe_dict, dict) else fn(maybe_dict)


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


# A validation rule: (predicate on the instance -> True when it is violated, message builder).
_Rule = Tuple[Callable[[Any], bool], Callable[[Any], str]]


def _enforce(obj, rules: Sequence[_Rule]) -> None:
    for violated, message in rules:
        if violated(obj):
            raise ValueError(message(obj))


_REW_RULES: Tuple[_Rule, ...] = (
    (lambda s: s.rews.shape != (len(s.acts),),
     lambda s: f"rewards must be 1D array, one entry for each action: {s.rews.shape} != ({len(s.acts)},)"),
    (lambda s: not np.issubdtype(s.rews.dtype, np.floating), lambda s: f"rewards dtype {s.rews.dtype} not a float"),
)


def _same_field(name: str, a, b, n: int) -> bool:
    if name == "infos":  # absent infos compare equal to empty per-step dicts
        a = [{}] * n if a is None else a
        b = [{}] * n if b is None else b
    if isinstance(a, DictObs) or isinstance(b, DictObs):
        return a == b
    return bool(np.array_equal(a, b))


@dataclasses.dataclass(frozen=True)
class Trajectory:
    """One episode (or fragment): ``obs`` has one more entry than ``acts``."""

    obs: Observation
    acts: np.ndarray
    infos: Optional[np.ndarray]
    terminal: bool

    _RULES = (
        (lambda s: len(s.obs) != len(s.acts) + 1,
         lambda s: f"expected one more observations than actions: {len(s.obs)} != {len(s.acts)} + 1"),
        (lambda s: s.infos is not None and len(s.infos) != len(s.acts),
         lambda s: f"infos when present must be present for each action: {len(s.infos)} != {len(s.acts)}"),
        (lambda s: len(s.acts) == 0, lambda s: "Degenerate trajectory: must have at least one action."),
    )

    def __len__(self) -> int:
        return len(self.acts)

    def __post_init__(self):
        _enforce(self, Trajectory._RULES)

    def __eq__(self, other) -> bool:
        if not isinstance(other, Trajectory) or len(self) != len(other):
            return False
        mine, theirs = dataclass_quick_asdict(self), dataclass_quick_asdict(other)
        if mine.keys() != theirs.keys():
            return False
        return all(_same_field(k, v, theirs[k], len(self)) for k, v in mine.items())

    def __setstate__(self, state):
        if "terminal" not in state:  # pickles written before the field existed ended whole episodes
            warnings.warn("Trajectory pickled without its `terminal` field (old format): assuming terminal=True. "
                          "Reading this format will be removed in a future version.", DeprecationWarning)
            state = dict(state, terminal=True)
        for k, v in state.items():
            object.__setattr__(self, k, v)


@dataclasses.dataclass(frozen=True, eq=False)
class TrajectoryWithRew(Trajectory):
    """A :class:`Trajectory` with per-step rewards ``rews`` (float, shape ``(T,)``)."""

    rews: np.ndarray

    def __post_init__(self):
        super().__post_init__()
        _enforce(self, _REW_RULES)


Pair = Tuple[T, T]
TrajectoryPair = Pair[Trajectory]
TrajectoryWithRewPair = Pair[TrajectoryWithRew]


def transitions_collate_fn(batch: Sequence[Mapping[str, np.ndarray]]) -> Mapping[str, AnyTensor]:
    """DataLoader collate for transitions: ``acts`` / ``dones`` through torch's default collate,
    ``infos`` kept as a list, observations stacked (dict observations as one :class:`DictObs`)."""
    out = dict(th_data.dataloader.default_collate(
        [{k: np.array(s[k]) for k in ("acts", "dones") if k in s} for s in batch]))
    out["infos"] = [s["infos"] for s in batch]
    for k in ("obs", "next_obs"):
        out[k] = stack_maybe_dictobs([s[k] for s in batch])
    return out


TransitionsMinimalSelf = TypeVar("TransitionsMinimalSelf", bound="TransitionsMinimal")


@dataclasses.dataclass(frozen=True)
class TransitionsMinimal(th_data.Dataset, Sequence[Mapping[str, np.ndarray]]):
    """Flat batch of (obs, act, info); int index -> dict sample, slice -> same class. Array fields
    are made read-only on construction (the batch may be shared by loaders and replay buffers)."""

    obs: Observation
    acts: np.ndarray
    infos: np.ndarray

    _RULES = (
        (lambda s: len(s.obs) != len(s.acts),
         lambda s: f"obs and acts must have same number of timesteps: {len(s.obs)} != {len(s.acts)}"),
        (lambda s: len(s.infos) != len(s.obs),
         lambda s: f"obs and infos must have same number of timesteps: {len(s.obs)} != {len(s.infos)}"),
    )

    def __len__(self) -> int:
        return len(self.obs)

    def __post_init__(self):
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if isinstance(v, np.ndarray):
                v.flags.writeable = False
        _enforce(self, TransitionsMinimal._RULES)

    def __getitem__(self, key):
        fields = dataclass_quick_asdict(self)
        if isinstance(key, slice):
            return dataclasses.replace(self, **{k: v[key] for k, v in fields.items()})
        assert isinstance(key, (int, np.integer))
        return {k: v[key] for k, v in fields.items()}

    def to_device(self, device, dtype=th.float32) -> Dict[str, th.Tensor]:
        """All numeric fields as contiguous device tensors (one H2D copy each); floats and bools
        become ``dtype``, integers keep their type."""
        out: Dict[str, th.Tensor] = {}
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if f.name == "infos" or isinstance(v, DictObs):
                continue
            t = th.as_tensor(np.ascontiguousarray(np.asarray(v)))
            if t.dtype == th.bool or t.is_floating_point():
                t = t.to(dtype)
            out[f.name] = t.to(device, non_blocking=True)
        return out


@dataclasses.dataclass(frozen=True)
class Transitions(TransitionsMinimal):
    """Batch of (obs, act, next_obs, done) transitions."""

    next_obs: Observation
    dones: np.ndarray

    _RULES = (
        (lambda s: s.obs.shape != s.next_obs.shape,
         lambda s: f"obs and next_obs must have same shape: {s.obs.shape} != {s.next_obs.shape}"),
        (lambda s: s.obs.dtype != s.next_obs.dtype,
         lambda s: f"obs and next_obs must have the same dtype: {s.obs.dtype} != {s.next_obs.dtype}"),
        (lambda s: s.dones.shape != (len(s.acts),),
         lambda s: f"dones must be 1D array, one entry for each timestep: {s.dones.shape} != ({len(s.acts)},)"),
        (lambda s: s.dones.dtype != bool, lambda s: f"dones must be boolean, not {s.dones.dtype}"),
    )

    def __post_init__(self):
        super().__post_init__()
        _enforce(self, Transitions._RULES)


@dataclasses.dataclass(frozen=True)
class TransitionsWithRew(Transitions):
    """Transitions with rewards."""

    rews: np.ndarray

    def __post_init__(self):
        super().__post_init__()
        _enforce(self, _REW_RULES)

"""Search-space primitives for ``parallel`` / ``tuning`` (the subset of ``ray.tune``'s
sampling API the reference's configs use; Ray is not part of the MI355X image).

``grid_search([...])`` expands to one trial per value (cartesian over all grids);
``choice / uniform / loguniform / randint / sample_from`` are sampled per trial.
"""

from __future__ import annotations

import copy
import itertools
import math
from typing import Any, Callable, Dict, List, Mapping, Sequence, Tuple

import numpy as np


class Domain:
    def sample(self, rng: np.random.Generator, spec: Mapping) -> Any:  # pragma: no cover - interface
        raise NotImplementedError


class _Choice(Domain):
    def __init__(self, values: Sequence[Any]):
        self.values = list(values)

    def sample(self, rng, spec):
        return copy.deepcopy(self.values[int(rng.integers(len(self.values)))])


class _Uniform(Domain):
    def __init__(self, lo: float, hi: float, log: bool = False):
        self.lo, self.hi, self.log = lo, hi, log

    def sample(self, rng, spec):
        if self.log:
            return float(math.exp(rng.uniform(math.log(self.lo), math.log(self.hi))))
        return float(rng.uniform(self.lo, self.hi))


class _RandInt(Domain):
    def __init__(self, lo: int, hi: int):
        self.lo, self.hi = lo, hi

    def sample(self, rng, spec):
        return int(rng.integers(self.lo, self.hi))


class _SampleFrom(Domain):
    def __init__(self, fn: Callable[[Mapping], Any]):
        self.fn = fn

    def sample(self, rng, spec):
        return self.fn(spec)


def choice(values: Sequence[Any]) -> Domain:
    return _Choice(values)


def uniform(lo: float, hi: float) -> Domain:
    return _Uniform(lo, hi)


def loguniform(lo: float, hi: float) -> Domain:
    return _Uniform(lo, hi, log=True)


def randint(lo: int, hi: int) -> Domain:
    return _RandInt(lo, hi)


def sample_from(fn: Callable[[Mapping], Any]) -> Domain:
    return _SampleFrom(fn)


def grid_search(values: Sequence[Any]) -> Dict[str, List[Any]]:
    return {"grid_search": list(values)}


def _walk(space: Any, path: Tuple = ()):
    if isinstance(space, Mapping):
        if set(space) == {"grid_search"}:
            yield path, space
            return
        for k, v in space.items():
            yield from _walk(v, path + (k,))
    elif isinstance(space, Domain):
        yield path, space


def _set(d: Any, path: Tuple, value: Any) -> None:
    for p in path[:-1]:
        d = d[p]
    d[path[-1]] = value


def generate_trials(space: Mapping, num_samples: int, rng: np.random.Generator) -> List[Dict[str, Any]]:
    """Expand grids (cartesian product) x ``num_samples`` random draws of the other domains."""
    leaves = list(_walk(space))
    grids = [(p, v["grid_search"]) for p, v in leaves if isinstance(v, Mapping)]
    domains = [(p, v) for p, v in leaves if isinstance(v, Domain)]
    trials = []
    for combo in itertools.product(*[vals for _, vals in grids]) if grids else [()]:
        for _ in range(num_samples):
            t = copy.deepcopy(_strip_domains(space))
            for (p, _), val in zip(grids, combo):
                _set(t, p, copy.deepcopy(val))
            for p, dom in domains:
                _set(t, p, dom.sample(rng, t))
            trials.append(t)
    return trials


def _strip_domains(space: Any) -> Any:
    if isinstance(space, Mapping):
        if set(space) == {"grid_search"}:
            return None
        return {k: _strip_domains(v) for k, v in space.items()}
    if isinstance(space, Domain):
        return None
    return space

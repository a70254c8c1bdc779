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


# --------------------------------------------------------------------------- model-based search
class TPESearch:
    """Tree-structured Parzen Estimator search over a ``tune`` space (the reference runs Optuna's
    default TPE through ``OptunaSearch`` wrapped in ``search.Repeater``:
    ``src/imitation/scripts/parallel.py:114-125``, ``tuning.py:43-46``; neither library is in
    this image). Univariate TPE as Optuna's default sampler does it:

    * the first ``n_startup`` suggestions are random draws of the space;
    * then the completed trials are split into the best ``gamma(n) = min(ceil(0.1 n), 25)``
      ("good", metric maximised) and the rest; per leaf, a Parzen estimator l(x) is fit to the
      good values and g(x) to the rest -- truncated Gaussian mixtures in the leaf's own scale
      (log for ``loguniform``, integer-rounded for ``randint``) with a prior component and
      neighbour-distance bandwidths, or smoothed category counts for ``choice`` / grids;
    * ``n_candidates`` draws from l(x) are scored by log l(x) - log g(x), the best one is taken.

    ``sample_from`` leaves are resolved after the others (they may read the sampled spec), as in
    :func:`generate_trials`. Use :meth:`suggest` / :meth:`observe` (a batch of suggestions may be
    run in parallel before observing them)."""

    def __init__(self, space: Mapping, rng: np.random.Generator, n_startup: int = 10, n_candidates: int = 24,
                 prior_weight: float = 1.0):
        self.space = space
        self.rng = rng
        self.n_startup = int(n_startup)
        self.n_candidates = int(n_candidates)
        self.prior_weight = float(prior_weight)
        leaves = list(_walk(space))
        self.params = [(p, v) for p, v in leaves if not isinstance(v, _SampleFrom)]
        self.derived = [(p, v) for p, v in leaves if isinstance(v, _SampleFrom)]
        self.history: List[Tuple[Dict[Tuple, Any], float]] = []

    # -- leaf encodings
    @staticmethod
    def _kind(dom: Any) -> str:
        if isinstance(dom, Mapping):
            return "cat"
        if isinstance(dom, _Choice):
            return "cat"
        if isinstance(dom, _RandInt):
            return "int"
        return "float"

    @staticmethod
    def _cats(dom: Any) -> List[Any]:
        return list(dom["grid_search"]) if isinstance(dom, Mapping) else list(dom.values)

    @staticmethod
    def _bounds(dom: Any) -> Tuple[float, float]:
        if isinstance(dom, _RandInt):
            return dom.lo - 0.5, dom.hi - 0.5
        if dom.log:
            return math.log(dom.lo), math.log(dom.hi)
        return float(dom.lo), float(dom.hi)

    def _encode(self, dom: Any, value: Any) -> float:
        kind = self._kind(dom)
        if kind == "cat":
            cats = self._cats(dom)
            for i, c in enumerate(cats):
                if c == value:
                    return float(i)
            return 0.0
        if kind == "float" and dom.log:
            return math.log(value)
        return float(value)

    def _decode(self, dom: Any, x: float) -> Any:
        kind = self._kind(dom)
        if kind == "cat":
            return copy.deepcopy(self._cats(dom)[int(x)])
        if kind == "int":
            return int(min(max(round(x), dom.lo), dom.hi - 1))
        if dom.log:
            return float(min(max(math.exp(x), dom.lo), dom.hi))
        return float(min(max(x, dom.lo), dom.hi))

    # -- Parzen estimators
    def _numeric_mixture(self, obs: Sequence[float], lo: float, hi: float):
        span = hi - lo
        mus = np.asarray(list(obs) + [0.5 * (lo + hi)], dtype=np.float64)
        w = np.ones(len(mus))
        w[-1] = self.prior_weight
        order = np.argsort(mus)
        srt = mus[order]
        left = np.diff(np.concatenate(([lo], srt)))
        right = np.diff(np.concatenate((srt, [hi])))
        sig_sorted = np.maximum(left, right)
        sig = np.empty_like(sig_sorted)
        sig[order] = sig_sorted
        sig[-1] = span  # prior: wide
        n = len(obs)
        sig = np.clip(sig, span / min(100.0, 1.0 + n), span)
        return mus, sig, w / w.sum()

    @staticmethod
    def _trunc_logpdf(x: np.ndarray, mus, sig, w, lo, hi) -> np.ndarray:
        from scipy.special import logsumexp
        from scipy.stats import norm

        z = (x[:, None] - mus[None, :]) / sig[None, :]
        mass = norm.cdf((hi - mus) / sig) - norm.cdf((lo - mus) / sig)
        lp = norm.logpdf(z) - np.log(sig)[None, :] - np.log(np.maximum(mass, 1e-300))[None, :] + np.log(w)[None, :]
        return logsumexp(lp, axis=1)

    def _sample_mixture(self, mus, sig, w, lo, hi, k: int) -> np.ndarray:
        comp = self.rng.choice(len(mus), size=k, p=w)
        out = np.empty(k)
        for i, c in enumerate(comp):
            for _ in range(100):
                v = self.rng.normal(mus[c], sig[c])
                if lo <= v <= hi:
                    break
            else:
                v = min(max(mus[c], lo), hi)
            out[i] = v
        return out

    def _cat_probs(self, obs: Sequence[float], n_cat: int) -> np.ndarray:
        p = np.full(n_cat, self.prior_weight / n_cat)
        for o in obs:
            p[int(o)] += 1.0
        return p / p.sum()

    def _suggest_leaf(self, dom: Any, good: List[float], bad: List[float]) -> float:
        kind = self._kind(dom)
        if kind == "cat":
            n_cat = len(self._cats(dom))
            pl, pg = self._cat_probs(good, n_cat), self._cat_probs(bad, n_cat)
            cand = self.rng.choice(n_cat, size=self.n_candidates, p=pl)
            score = np.log(pl[cand]) - np.log(pg[cand])
            return float(cand[int(np.argmax(score))])
        lo, hi = self._bounds(dom)
        ml = self._numeric_mixture(good, lo, hi)
        mg = self._numeric_mixture(bad, lo, hi)
        cand = self._sample_mixture(*ml, lo, hi, self.n_candidates)
        if kind == "int":
            cand = np.clip(np.round(cand), dom.lo, dom.hi - 1).astype(np.float64)
        score = self._trunc_logpdf(cand, *ml, lo, hi) - self._trunc_logpdf(cand, *mg, lo, hi)
        return float(cand[int(np.argmax(score))])

    # -- public API
    def suggest(self) -> Dict[str, Any]:
        """One resolved sample of the space (a dict shaped like the space)."""
        t = copy.deepcopy(_strip_domains(self.space))
        done = [(x, m) for x, m in self.history if m == m]  # finite metrics only
        if len(done) < self.n_startup:
            for p, dom in self.params:
                if isinstance(dom, Mapping):
                    vals = dom["grid_search"]
                    _set(t, p, copy.deepcopy(vals[int(self.rng.integers(len(vals)))]))
                else:
                    _set(t, p, dom.sample(self.rng, t))
        else:
            ranked = sorted(done, key=lambda xm: -xm[1])
            n_good = max(1, min(int(math.ceil(0.1 * len(ranked))), 25))
            good, bad = ranked[:n_good], ranked[n_good:]
            for p, dom in self.params:
                x = self._suggest_leaf(dom, [self._encode(dom, g[0][p]) for g in good],
                                       [self._encode(dom, b[0][p]) for b in bad])
                _set(t, p, self._decode(dom, x))
        for p, dom in self.derived:
            _set(t, p, dom.sample(self.rng, t))
        return t

    def observe(self, sample: Mapping, metric: float) -> None:
        """Record a completed trial (``metric`` maximised; NaN = failed, ignored by the model)."""
        vals = {}
        for p, _ in self.params:
            d = sample
            for k in p:
                d = d[k]
            vals[p] = d
        self.history.append((vals, float(metric)))

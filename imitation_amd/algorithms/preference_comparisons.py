"""Learning a reward model from pairwise preferences (DRLHP)
(reference: ``src/imitation/algorithms/preference_comparisons.py``).

Components keep the reference's names and semantics: trajectory generators
(:class:`AgentTrainer`, :class:`TrajectoryDataset`), fragmenters
(:class:`RandomFragmenter`, :class:`ActiveSelectionFragmenter`), the synthetic
gatherer, the FIFO :class:`PreferenceDataset`, the Bradley-Terry
:class:`PreferenceModel` + :class:`CrossEntropyRewardLoss`, the basic / ensemble
reward trainers (bagging, gradient accumulation, regularizers) and the
:class:`PreferenceComparisons` loop with its query schedule.

MI355X design. The reference scores a minibatch pair by pair: for every pair it
flattens both fragments, runs the reward net twice and does a few scalar torch ops
(``preference_comparisons.py:441-455``) -- 2P tiny launches plus host syncs per
minibatch. Here a minibatch is packed once on the host (all 2P fragments
concatenated), the reward net runs ONCE over all 2·P·L transitions (one fused MLP
launch on the device), rewards are scattered into a padded ``[2, P, L]`` tile, and
the segment sums + Bradley-Terry probability + BCE run in one HIP kernel
(``ops.preference.bradley_terry``, ``csrc/kernels/pref.hip``) with a matching
backward kernel. Ensemble members are scored in the same batched way.
"""

from __future__ import annotations

import abc
import os
import math
import re
from collections import defaultdict
from typing import Any, Callable, Dict, List, Mapping, NamedTuple, NoReturn, Optional, Sequence, Tuple, Union, cast

import numpy as np
import torch as th

from imitation_amd.utils import graphs
from scipy import special
from torch import nn
from torch.utils import data as data_th

from imitation_amd.algorithms import base
from imitation_amd.data import rollout, types, wrappers
from imitation_amd.data.types import AnyPath, TrajectoryPair, TrajectoryWithRew, TrajectoryWithRewPair, Transitions
from imitation_amd.ops import rl as rl_ops
from imitation_amd.ops import optim as optim_ops
from imitation_amd.ops import preference as pref_ops
from imitation_amd.parallel import dist as pdist
from imitation_amd.policies import exploration_wrapper
from imitation_amd.regularization import regularizers
from imitation_amd.rewards import reward_function, reward_nets, reward_wrapper
from imitation_amd.rl.base import check_for_correct_spaces
from imitation_amd.util import logger as imit_logger
from imitation_amd.utils import gcfreeze, profiling
from imitation_amd.util import networks, util

try:  # progress bars are optional
    from tqdm.auto import tqdm as _tqdm
except ImportError:  # pragma: no cover
    def _tqdm(x, **kwargs):
        return x


# --------------------------------------------------------------------------- generators
class TrajectoryGenerator(abc.ABC):
    """Generator of trajectories with optional training logic."""

    _logger: imit_logger.HierarchicalLogger

    def __init__(self, custom_logger: Optional[imit_logger.HierarchicalLogger] = None):
        self.logger = custom_logger or imit_logger.configure()

    @abc.abstractmethod
    def sample(self, steps: int) -> Sequence[TrajectoryWithRew]:
        """Trajectories with at least ``steps`` transitions in total (env rewards)."""

    def train(self, steps: int, **kwargs: Any) -> None:
        """Train the underlying agent, if any (default: nothing)."""

    @property
    def logger(self) -> imit_logger.HierarchicalLogger:
        return self._logger

    @logger.setter
    def logger(self, value: imit_logger.HierarchicalLogger) -> None:
        self._logger = value


class TrajectoryDataset(TrajectoryGenerator):
    """A fixed dataset of trajectories, shuffled on every ``sample``."""

    def __init__(self, trajectories: Sequence[TrajectoryWithRew], rng: np.random.Generator,
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None):
        super().__init__(custom_logger=custom_logger)
        self._trajectories = trajectories
        self.rng = rng

    def sample(self, steps: int) -> Sequence[TrajectoryWithRew]:
        trajectories = list(self._trajectories)
        self.rng.shuffle(trajectories)  # type: ignore[arg-type]
        return _get_trajectories(trajectories, steps)


class AgentTrainer(TrajectoryGenerator):
    """Trains an RL algorithm on a (learned) reward function and samples its rollouts."""

    def __init__(self, algorithm, reward_fn: Union[reward_function.RewardFn, reward_nets.RewardNet], venv,
                 rng: np.random.Generator, exploration_frac: float = 0.0, switch_prob: float = 0.5,
                 random_prob: float = 0.5, custom_logger: Optional[imit_logger.HierarchicalLogger] = None) -> None:
        self.algorithm = algorithm
        super().__init__(custom_logger)
        if isinstance(reward_fn, reward_nets.RewardNet):
            check_for_correct_spaces(venv, reward_fn.observation_space, reward_fn.action_space)
            reward_fn = reward_fn.predict_processed
        self.reward_fn = reward_fn
        self.exploration_frac = exploration_frac
        self.rng = rng
        self.buffering_wrapper = wrappers.BufferingWrapper(venv)
        self.venv = self.reward_venv_wrapper = reward_wrapper.RewardVecEnvWrapper(self.buffering_wrapper, reward_fn=self.reward_fn)
        self.log_callback = self.reward_venv_wrapper.make_log_callback()
        self.algorithm.set_env(self.venv)
        algo_venv = self.algorithm.get_env()
        assert algo_venv is not None
        self.exploration_wrapper = exploration_wrapper.ExplorationWrapper(
            policy=self.algorithm, venv=algo_venv, random_prob=random_prob, switch_prob=switch_prob, rng=self.rng)

    def train(self, steps: int, **kwargs) -> None:
        n_transitions = self.buffering_wrapper.n_transitions
        if n_transitions:
            raise RuntimeError(f"There are {n_transitions} transitions left in the buffer. "
                               "Call AgentTrainer.sample() first to clear them.")
        self.algorithm.learn(total_timesteps=steps, reset_num_timesteps=False, callback=self.log_callback, **kwargs)

    def sample(self, steps: int) -> Sequence[TrajectoryWithRew]:
        agent_trajs, _ = self.buffering_wrapper.pop_finished_trajectories()
        agent_trajs = list(agent_trajs)[::-1]  # newest first
        avail_steps = sum(len(t) for t in agent_trajs)
        exploration_steps = int(self.exploration_frac * steps)
        if self.exploration_frac > 0 and exploration_steps == 0:
            self.logger.warn(f"No exploration steps included: exploration_frac = {self.exploration_frac} > 0 "
                             f"but steps={steps} is too small.")
        agent_steps = steps - exploration_steps
        algo_venv = self.algorithm.get_env()
        assert algo_venv is not None
        if avail_steps < agent_steps:
            self.logger.log(f"Requested {agent_steps} transitions but only {avail_steps} in buffer. "
                            f"Sampling {agent_steps - avail_steps} additional transitions.")
            rollout.generate_trajectories(self.algorithm, algo_venv,
                                          sample_until=rollout.make_sample_until(min_timesteps=agent_steps - avail_steps,
                                                                                 min_episodes=None),
                                          deterministic_policy=False, rng=self.rng)
            additional, _ = self.buffering_wrapper.pop_finished_trajectories()
            agent_trajs = agent_trajs + list(additional)
        trajectories = list(_get_trajectories(agent_trajs, agent_steps))
        if exploration_steps > 0:
            self.logger.log(f"Sampling {exploration_steps} exploratory transitions.")
            rollout.generate_trajectories(policy=self.exploration_wrapper, venv=algo_venv,
                                          sample_until=rollout.make_sample_until(min_timesteps=exploration_steps,
                                                                                 min_episodes=None),
                                          deterministic_policy=False, rng=self.rng)
            exploration_trajs, _ = self.buffering_wrapper.pop_finished_trajectories()
            trajectories.extend(_get_trajectories(exploration_trajs, exploration_steps))
        return trajectories

    @property
    def logger(self) -> imit_logger.HierarchicalLogger:
        return super().logger

    @logger.setter
    def logger(self, value: imit_logger.HierarchicalLogger) -> None:
        self._logger = value
        self.algorithm.set_logger(self.logger)


def _get_trajectories(trajectories: Sequence[TrajectoryWithRew], steps: int) -> Sequence[TrajectoryWithRew]:
    """Shortest prefix of ``trajectories`` with at least ``steps`` transitions."""
    if steps == 0:
        return []
    available = sum(len(t) for t in trajectories)
    if available < steps:
        raise RuntimeError(f"Asked for {steps} transitions but only {available} available")
    cums = np.cumsum([len(t) for t in trajectories])
    idx = int((cums >= steps).argmax())
    return trajectories[: idx + 1]


# --------------------------------------------------------------------------- batched fragment scoring
class _PackedPairs(NamedTuple):
    state: np.ndarray
    action: np.ndarray
    next_state: np.ndarray
    done: np.ndarray
    rows: np.ndarray  # fragment index (0..2P-1, frag1 of pair i = 2i, frag2 = 2i+1) of every transition
    cols: np.ndarray  # position of every transition inside its fragment
    n_frags: int
    max_len: int


def _pack_pairs(fragment_pairs: Sequence[TrajectoryPair]) -> _PackedPairs:
    """Concatenate the transitions of all 2P fragments (one host pass, one device copy later)."""
    frags = [f for pair in fragment_pairs for f in pair]
    lens = np.array([len(f) for f in frags], dtype=np.int64)
    obs = [types.assert_not_dictobs(f.obs) for f in frags]
    state = np.concatenate([o[:-1] for o in obs])
    next_state = np.concatenate([o[1:] for o in obs])
    action = np.concatenate([np.asarray(f.acts) for f in frags])
    done = np.zeros(int(lens.sum()), dtype=bool)
    ends = np.cumsum(lens) - 1
    done[ends] = [bool(f.terminal) for f in frags]
    rows = np.repeat(np.arange(len(frags)), lens)
    starts = np.cumsum(lens) - lens
    cols = np.arange(int(lens.sum())) - np.repeat(starts, lens)
    return _PackedPairs(state, action, next_state, done, rows, cols, len(frags), int(lens.max()))


def _to_tiles(rews: th.Tensor, packed: _PackedPairs) -> Tuple[th.Tensor, th.Tensor]:
    """Per-transition rewards ``[N(, M)]`` -> padded fragment tiles ``r1, r2`` of ``[P, L(, M)]`` (zero padding
    does not change the discounted return differences)."""
    shape = (packed.n_frags, packed.max_len) + tuple(rews.shape[1:])
    rows = th.as_tensor(packed.rows, device=rews.device)
    cols = th.as_tensor(packed.cols, device=rews.device)
    tile = th.zeros(shape, dtype=rews.dtype, device=rews.device).index_put((rows, cols), rews)
    return tile[0::2], tile[1::2]


class PreferenceModel(nn.Module):
    """Bradley-Terry model of preferring fragment 1, from (discounted) reward sums."""

    def __init__(self, model: reward_nets.RewardNet, noise_prob: float = 0.0, discount_factor: float = 1.0,
                 threshold: float = 50) -> None:
        super().__init__()
        self.model = model
        self.noise_prob = noise_prob
        self.discount_factor = discount_factor
        self.threshold = threshold
        base_model = get_base_model(model)
        self.ensemble_model = None
        if isinstance(base_model, reward_nets.RewardEnsemble):
            is_base = model is base_model
            is_std_wrapper = isinstance(model, reward_nets.AddSTDRewardWrapper) and model.base is base_model
            if not (is_base or is_std_wrapper):
                raise ValueError(f"RewardEnsemble can only be wrapped by AddSTDRewardWrapper but found {type(model).__name__}.")
            self.ensemble_model = base_model
            self.member_pref_models = [PreferenceModel(cast(reward_nets.RewardNet, m), self.noise_prob,
                                                       self.discount_factor, self.threshold)
                                       for m in self.ensemble_model.members]

    # ---- batched path
    def packed_rewards(self, packed: _PackedPairs) -> th.Tensor:
        """Rewards of every packed transition: ``[N]`` (or ``[N, M]`` for an ensemble)."""
        if self.ensemble_model is not None:
            ens = self.ensemble_model
            s, a, ns, d = ens.members[0].preprocess(packed.state, packed.action, packed.next_state, packed.done)
            return th.stack([m(s, a, ns, d) for m in ens.members], dim=-1)
        s, a, ns, d = self.model.preprocess(packed.state, packed.action, packed.next_state, packed.done)
        rews = self.model(s, a, ns, d)
        assert rews.shape == (len(packed.state),)
        return rews

    def pair_rewards(self, fragment_pairs: Sequence[TrajectoryPair]) -> Tuple[th.Tensor, th.Tensor]:
        packed = _pack_pairs(fragment_pairs)
        return _to_tiles(self.packed_rewards(packed), packed)

    def loss_and_probs(self, fragment_pairs: Sequence[TrajectoryPair], preferences) -> Tuple[th.Tensor, th.Tensor]:
        """Mean BCE and model probabilities for a minibatch, fused (non-ensemble models)."""
        r1, r2 = self.pair_rewards(fragment_pairs)
        prefs = th.as_tensor(np.asarray(preferences, dtype=np.float32), device=r1.device)
        return pref_ops.bradley_terry(r1, r2, prefs, self.discount_factor, self.threshold, self.noise_prob)

    # ---- reference API
    def forward(self, fragment_pairs: Sequence[TrajectoryPair]) -> Tuple[th.Tensor, Optional[th.Tensor]]:
        """Probability that fragment 1 is preferred, for all pairs (``[P]`` or ``[P, M]``), plus the
        ground-truth-reward probabilities when both fragments carry rewards."""
        r1, r2 = self.pair_rewards(fragment_pairs)
        if self.ensemble_model is not None:
            probs = self.probability(r1.transpose(0, 1), r2.transpose(0, 1))  # [L, P, M] -> sum over L
        else:
            probs = pref_ops.bradley_terry_probs_reference(r1, r2, self.discount_factor, self.threshold, self.noise_prob)
        gt_probs = None
        if _trajectory_pair_includes_reward(fragment_pairs[0]):
            g1 = th.as_tensor(np.stack([_pad(f.rews, r1.shape[1]) for f, _ in fragment_pairs]), dtype=th.float32)
            g2 = th.as_tensor(np.stack([_pad(f.rews, r1.shape[1]) for _, f in fragment_pairs]), dtype=th.float32)
            gt_probs = pref_ops.bradley_terry_probs_reference(g1, g2, self.discount_factor, self.threshold,
                                                              self.noise_prob).to(probs.device)
        return probs, gt_probs

    def rewards(self, transitions: Transitions) -> th.Tensor:
        state = types.assert_not_dictobs(transitions.obs)
        next_state = types.assert_not_dictobs(transitions.next_obs)
        if self.ensemble_model is not None:
            rews_np = self.ensemble_model.predict_processed_all(state, transitions.acts, next_state, transitions.dones)
            assert rews_np.shape == (len(state), self.ensemble_model.num_members)
            return util.safe_to_tensor(rews_np).to(self.ensemble_model.device)
        pre = self.model.preprocess(state, transitions.acts, next_state, transitions.dones)
        rews = self.model(*pre)
        assert rews.shape == (len(state),)
        return rews

    def probability(self, rews1: th.Tensor, rews2: th.Tensor) -> th.Tensor:
        """Boltzmann-rational probability that fragment 1 is best (time is axis 0)."""
        if self.discount_factor == 1:
            returns_diff = (rews2 - rews1).sum(axis=0)
        else:
            disc = self.discount_factor ** th.arange(len(rews1), device=rews1.device, dtype=rews1.dtype)
            disc = disc.reshape((-1,) + (1,) * (rews1.ndim - 1))
            returns_diff = (disc * (rews2 - rews1)).sum(axis=0)
        returns_diff = th.clip(returns_diff, -self.threshold, self.threshold)
        model_probability = 1 / (1 + returns_diff.exp())
        return self.noise_prob * 0.5 + (1 - self.noise_prob) * model_probability


def _pad(x: np.ndarray, n: int) -> np.ndarray:
    return np.pad(np.asarray(x, dtype=np.float32), (0, n - len(x)))


# --------------------------------------------------------------------------- fragmenters
class Fragmenter(abc.ABC):
    """Creates pairs of trajectory fragments."""

    def __init__(self, custom_logger: Optional[imit_logger.HierarchicalLogger] = None):
        self.logger = custom_logger or imit_logger.configure()

    @abc.abstractmethod
    def __call__(self, trajectories: Sequence[TrajectoryWithRew], fragment_length: int,
                 num_pairs: int) -> Sequence[TrajectoryWithRewPair]:
        """Sample ``num_pairs`` fragment pairs of length ``fragment_length``."""


def _fragment(traj: TrajectoryWithRew, start: int, end: int, terminal: bool) -> TrajectoryWithRew:
    """``traj[start:end]`` as a TrajectoryWithRew without re-running the dataclass validation:
    slices of a validated trajectory with ``0 <= start < end <= len(traj)`` are valid by
    construction (obs one longer than acts / rews / infos)."""
    frag = object.__new__(TrajectoryWithRew)
    object.__setattr__(frag, "obs", traj.obs[start: end + 1])
    object.__setattr__(frag, "acts", traj.acts[start:end])
    object.__setattr__(frag, "infos", traj.infos[start:end] if traj.infos is not None else None)
    object.__setattr__(frag, "terminal", terminal)
    object.__setattr__(frag, "rews", traj.rews[start:end])
    return frag


def _batched_discounted_sums(fragment_pairs, gamma: float) -> Optional[Tuple[np.ndarray, np.ndarray]]:
    """``rollout.discounted_sum`` (numpy ``polyval``'s Horner loop, in the rewards' dtype) of every
    fragment at once, when they all have the same length and 1-D rewards of one dtype: the same
    operations per fragment, so the same bits, without ~2K Python Horner loops (DRLHP labels ~2K
    fragments per iteration; the per-fragment loop cost ~50 ms). None when not applicable."""
    if not fragment_pairs:
        return None
    frags = [f for pair in fragment_pairs for f in pair]
    L = len(frags[0].rews)
    dt = frags[0].rews.dtype
    if L == 0 or any(f.rews.ndim != 1 or len(f.rews) != L or f.rews.dtype != dt for f in frags):
        return None
    c = np.stack([f.rews for f in frags])  # [2P, L]
    if c.dtype.char in "?bBhHiIlLqQpP":
        c = c + 0.0
    if gamma == 1.0:
        out = c.sum(axis=1)
    else:
        acc = c[:, -1] + gamma * 0
        for i in range(2, L + 1):
            acc = c[:, -i] + acc * gamma
        out = acc
    out = np.asarray(out, dtype=np.float32)
    return out[0::2].copy(), out[1::2].copy()


class RandomFragmenter(Fragmenter):
    """Fragments sampled uniformly (trajectories weighted by length), with replacement."""

    def __init__(self, rng: np.random.Generator, warning_threshold: int = 10,
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None) -> None:
        super().__init__(custom_logger)
        self.rng = rng
        self.warning_threshold = warning_threshold

    def __call__(self, trajectories, fragment_length: int, num_pairs: int) -> Sequence[TrajectoryWithRewPair]:
        prev = len(trajectories)
        trajectories = [t for t in trajectories if len(t) >= fragment_length]
        if len(trajectories) == 0:
            raise ValueError(f"No trajectories are long enough for the desired fragment length of {fragment_length}.")
        if prev - len(trajectories):
            self.logger.log(f"Discarded {prev - len(trajectories)} out of {prev} trajectories because they are shorter "
                            f"than the desired length of {fragment_length}.")
        weights = np.array([len(t) for t in trajectories], dtype=np.float64)
        num_transitions = 2 * num_pairs * fragment_length
        if weights.sum() < num_transitions:
            self.logger.warn("Fewer transitions available than needed for desired number of fragment pairs. "
                             "Some transitions will appear multiple times.")
        elif self.warning_threshold and weights.sum() < self.warning_threshold * num_transitions:
            self.logger.warn(f"Samples will contain {num_transitions} transitions in total and only {int(weights.sum())} "
                             "are available. Because we sample with replacement, a significant number of transitions "
                             "are likely to appear multiple times.")
        fragments = []
        p = weights / weights.sum()
        # ``rng.choice(len, p=p)`` draws exactly this: one ``random()`` double searched in the
        # normalised CDF (numpy Generator.choice) -- same index, same RNG stream, without
        # choice's per-call validation and cumsum (~17 of the ~28 us per fragment; DRLHP samples
        # ~2K fragments per iteration)
        cdf = p.cumsum()
        cdf /= cdf[-1]
        for _ in range(2 * num_pairs):
            traj = trajectories[int(cdf.searchsorted(self.rng.random(), side="right"))]
            n = len(traj)
            start = int(self.rng.integers(0, n - fragment_length, endpoint=True))
            end = start + fragment_length
            fragments.append(_fragment(traj, start, end, (end == n) and traj.terminal))
        it = iter(fragments)
        return list(zip(it, it))


class ActiveSelectionFragmenter(Fragmenter):
    """Keeps the fragment pairs on which an ensemble disagrees most (logit / probability / label variance)."""

    def __init__(self, preference_model: PreferenceModel, base_fragmenter: Fragmenter, fragment_sample_factor: float,
                 uncertainty_on: str = "logit", custom_logger: Optional[imit_logger.HierarchicalLogger] = None) -> None:
        super().__init__(custom_logger=custom_logger)
        if preference_model.ensemble_model is None:
            raise ValueError("PreferenceModel not wrapped over an ensemble of networks.")
        self.preference_model = preference_model
        self.base_fragmenter = base_fragmenter
        self.fragment_sample_factor = fragment_sample_factor
        self._uncertainty_on = uncertainty_on
        if uncertainty_on not in ("logit", "probability", "label"):
            self.raise_uncertainty_on_not_supported()

    @property
    def uncertainty_on(self) -> str:
        return self._uncertainty_on

    def raise_uncertainty_on_not_supported(self) -> NoReturn:
        raise ValueError(f"""{self.uncertainty_on} not supported.
            `uncertainty_on` should be from `logit`, `probability`, or `label`""")

    def __call__(self, trajectories, fragment_length: int, num_pairs: int) -> Sequence[TrajectoryWithRewPair]:
        fragment_pairs = self.base_fragmenter(trajectories=trajectories, fragment_length=fragment_length,
                                              num_pairs=int(self.fragment_sample_factor * num_pairs))
        # all candidate pairs scored by all members in one batched pass
        with th.no_grad():
            r1, r2 = self.preference_model.pair_rewards(fragment_pairs)  # [P, L, M]
        var_estimates = self.variance_estimates(r1, r2)
        order = np.argsort(var_estimates, kind="stable")[::-1]
        return [fragment_pairs[i] for i in order[:num_pairs]]

    def variance_estimates(self, r1: th.Tensor, r2: th.Tensor) -> np.ndarray:
        """Per-pair variance across ensemble members; ``r1, r2``: ``[P, L, M]``."""
        if self.uncertainty_on == "logit":
            return (r1.sum(1) - r2.sum(1)).var(dim=-1).cpu().numpy()
        probs = self.preference_model.probability(r1.transpose(0, 1), r2.transpose(0, 1)).cpu().numpy()  # [P, M]
        if self.uncertainty_on == "probability":
            return probs.var(axis=-1)
        if self.uncertainty_on == "label":
            pe = (probs > 0.5).astype(np.float32).mean(-1)
            return pe * (1 - pe)
        self.raise_uncertainty_on_not_supported()

    def variance_estimate(self, rews1: th.Tensor, rews2: th.Tensor) -> float:
        """Single-pair variant (``[L, M]`` rewards), reference API."""
        return float(self.variance_estimates(rews1[None], rews2[None])[0])


# --------------------------------------------------------------------------- preference gathering
class PreferenceGatherer(abc.ABC):
    def __init__(self, rng: Optional[np.random.Generator] = None,
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None) -> None:
        del rng
        self.logger = custom_logger or imit_logger.configure()

    @abc.abstractmethod
    def __call__(self, fragment_pairs: Sequence[TrajectoryWithRewPair]) -> np.ndarray:
        """Probability that fragment 1 is preferred, shape ``(len(fragment_pairs),)``."""


class SyntheticGatherer(PreferenceGatherer):
    """Preferences from ground-truth returns under a Boltzmann-rational model."""

    def __init__(self, temperature: float = 1, discount_factor: float = 1, sample: bool = True,
                 rng: Optional[np.random.Generator] = None, threshold: float = 50,
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None) -> None:
        super().__init__(custom_logger=custom_logger)
        self.temperature = temperature
        self.discount_factor = discount_factor
        self.sample = sample
        self.rng = rng
        self.threshold = threshold
        if self.sample and self.rng is None:
            raise ValueError("If `sample` is True, then `rng` must be provided.")

    def __call__(self, fragment_pairs: Sequence[TrajectoryWithRewPair]) -> np.ndarray:
        returns1, returns2 = self._reward_sums(fragment_pairs)
        if self.temperature == 0:
            return (np.sign(returns1 - returns2) + 1) / 2
        returns1 /= self.temperature
        returns2 /= self.temperature
        returns_diff = np.clip(returns2 - returns1, -self.threshold, self.threshold)
        model_probs = 1 / (1 + np.exp(returns_diff))
        entropy = -(special.xlogy(model_probs, model_probs) + special.xlogy(1 - model_probs, 1 - model_probs)).mean()
        self.logger.record("entropy", entropy)
        if self.sample:
            assert self.rng is not None
            return self.rng.binomial(n=1, p=model_probs).astype(np.float32)
        return model_probs

    def _reward_sums(self, fragment_pairs) -> Tuple[np.ndarray, np.ndarray]:
        fast = _batched_discounted_sums(fragment_pairs, self.discount_factor)
        if fast is not None:
            return fast
        r1, r2 = zip(*[(rollout.discounted_sum(f1.rews, self.discount_factor),
                        rollout.discounted_sum(f2.rews, self.discount_factor)) for f1, f2 in fragment_pairs])
        return np.array(r1, dtype=np.float32), np.array(r2, dtype=np.float32)


class PreferenceDataset(data_th.Dataset):
    """FIFO dataset of (fragment pair, preference) items grown with :meth:`push`."""

    def __init__(self, max_size: Optional[int] = None) -> None:
        self.fragments1: List[TrajectoryWithRew] = []
        self.fragments2: List[TrajectoryWithRew] = []
        self.max_size = max_size
        self.preferences: np.ndarray = np.array([], dtype=np.float32)

    def push(self, fragments: Sequence[TrajectoryWithRewPair], preferences: np.ndarray) -> None:
        fragments1, fragments2 = zip(*fragments)
        if preferences.shape != (len(fragments),):
            raise ValueError(f"Unexpected preferences shape {preferences.shape}, expected {(len(fragments),)}")
        if preferences.dtype != np.float32:
            raise ValueError("preferences should have dtype float32")
        self.fragments1.extend(fragments1)
        self.fragments2.extend(fragments2)
        self.preferences = np.concatenate((self.preferences, preferences)).astype(np.float32)
        if self.max_size is not None:
            extra = len(self.preferences) - self.max_size
            if extra > 0:
                self.fragments1 = self.fragments1[extra:]
                self.fragments2 = self.fragments2[extra:]
                self.preferences = self.preferences[extra:]

    def __getitem__(self, key):
        return (self.fragments1[key], self.fragments2[key]), self.preferences[key]

    def __len__(self) -> int:
        assert len(self.fragments1) == len(self.fragments2) == len(self.preferences)
        return len(self.fragments1)

    def save(self, path: AnyPath) -> None:
        """Write the dataset as one ``.npz`` of packed arrays (no pickle; infos as JSON)."""
        from imitation_amd.data import huggingface_utils as hfu

        frags = self.fragments1 + self.fragments2
        arrays: Dict[str, np.ndarray] = {
            "preferences": self.preferences.astype(np.float32),
            "max_size": np.array(-1 if self.max_size is None else self.max_size),
            "lengths": np.array([len(f) for f in frags], dtype=np.int64),
            "terminal": np.array([bool(f.terminal) for f in frags]),
            "obs": np.concatenate([types.assert_not_dictobs(f.obs) for f in frags]) if frags else np.zeros((0,)),
            "acts": np.concatenate([np.asarray(f.acts) for f in frags]) if frags else np.zeros((0,)),
            "rews": np.concatenate([np.asarray(f.rews, dtype=np.float32) for f in frags]) if frags else np.zeros((0,)),
            "infos": np.array([hfu.encode_info(i) for f in frags for i in (f.infos if f.infos is not None else [])],
                              dtype=np.str_),
            "has_infos": np.array([f.infos is not None for f in frags]),
        }
        with open(path, "wb") as fh:
            np.savez_compressed(fh, **arrays)

    @staticmethod
    def load(path: AnyPath) -> "PreferenceDataset":
        from imitation_amd.data import huggingface_utils as hfu

        z = np.load(path, allow_pickle=False)
        max_size = int(z["max_size"])
        ds = PreferenceDataset(max_size=None if max_size < 0 else max_size)
        lens, term, has_inf = z["lengths"], z["terminal"], z["has_infos"]
        obs, acts, rews, infos = z["obs"], z["acts"], z["rews"], z["infos"]
        frags, o, a, k = [], 0, 0, 0
        for n, t, hi in zip(lens, term, has_inf):
            n = int(n)
            inf = None
            if hi:
                inf = np.array([hfu.decode_info(s) for s in infos[k:k + n]], dtype=object)
                k += n
            frags.append(TrajectoryWithRew(obs=obs[o: o + n + 1], acts=acts[a: a + n], infos=inf, rews=rews[a: a + n],
                                           terminal=bool(t)))
            o += n + 1
            a += n
        half = len(frags) // 2
        ds.fragments1, ds.fragments2 = frags[:half], frags[half:]
        ds.preferences = z["preferences"].astype(np.float32)
        return ds


def preference_collate_fn(batch: Sequence[Tuple[TrajectoryWithRewPair, float]]) -> Tuple[Sequence[TrajectoryWithRewPair], np.ndarray]:
    fragment_pairs, preferences = zip(*batch)
    return list(fragment_pairs), np.array(preferences)


# --------------------------------------------------------------------------- losses / reward trainers
class LossAndMetrics(NamedTuple):
    loss: th.Tensor
    metrics: Mapping[str, th.Tensor]


class RewardLoss(nn.Module, abc.ABC):
    @abc.abstractmethod
    def forward(self, fragment_pairs: Sequence[TrajectoryPair], preferences: np.ndarray,
                preference_model: PreferenceModel) -> LossAndMetrics:
        """Loss and metrics over a minibatch of pairs."""


def _trajectory_pair_includes_reward(fragment_pair: TrajectoryPair) -> bool:
    f1, f2 = fragment_pair
    return isinstance(f1, TrajectoryWithRew) and isinstance(f2, TrajectoryWithRew)


class CrossEntropyRewardLoss(RewardLoss):
    """BCE between the modelled preference probability and the gathered preference."""

    def forward(self, fragment_pairs, preferences, preference_model: PreferenceModel) -> LossAndMetrics:
        prefs_np = np.asarray(preferences, dtype=np.float32)
        if preference_model.ensemble_model is None:
            loss, probs = preference_model.loss_and_probs(fragment_pairs, prefs_np)
        else:  # scoring only (ensembles are trained member by member)
            probs, _ = preference_model(fragment_pairs)
            loss = th.nn.functional.binary_cross_entropy(pref_ops._finite_probs(probs), th.as_tensor(prefs_np, device=probs.device)[:, None]
                                                         .expand_as(probs))
        preferences_th = th.as_tensor(prefs_np, device=probs.device)
        metrics = {"accuracy": ((probs.detach() > 0.5) == (preferences_th > 0.5).reshape((-1,) + (1,) * (probs.ndim - 1)))
                   .float().mean()}
        if _trajectory_pair_includes_reward(fragment_pairs[0]):
            g1 = np.stack([_pad(f.rews, max(len(f) for p in fragment_pairs for f in p)) for f, _ in fragment_pairs])
            g2 = np.stack([_pad(f.rews, g1.shape[1]) for _, f in fragment_pairs])
            gt_probs = pref_ops.bradley_terry_probs_reference(th.as_tensor(g1), th.as_tensor(g2),
                                                              preference_model.discount_factor,
                                                              preference_model.threshold, preference_model.noise_prob)
            metrics["gt_reward_loss"] = th.nn.functional.binary_cross_entropy(gt_probs, th.as_tensor(prefs_np))
        return LossAndMetrics(loss=loss, metrics={k: v.detach().cpu() for k, v in metrics.items()})


class RewardTrainer(abc.ABC):
    """Trains the reward model of a :class:`PreferenceModel` on a preference dataset."""

    def __init__(self, preference_model: PreferenceModel, custom_logger: Optional[imit_logger.HierarchicalLogger] = None):
        self._preference_model = preference_model
        self._logger = custom_logger or imit_logger.configure()

    @property
    def logger(self) -> imit_logger.HierarchicalLogger:
        return self._logger

    @logger.setter
    def logger(self, custom_logger: imit_logger.HierarchicalLogger) -> None:
        self._logger = custom_logger

    def train(self, dataset: PreferenceDataset, epoch_multiplier: float = 1.0) -> None:
        with networks.training(self._preference_model.model):
            self._train(dataset, epoch_multiplier)

    @abc.abstractmethod
    def _train(self, dataset: PreferenceDataset, epoch_multiplier: float) -> None:
        """Train for ``round(epochs * epoch_multiplier)`` epochs."""


class BasicRewardTrainer(RewardTrainer):
    """AdamW on the reward net; gradient accumulation over minibatches; optional regularizer with
    a validation split driving λ."""

    regularizer: Optional[regularizers.Regularizer]

    def __init__(self, preference_model: PreferenceModel, loss: RewardLoss, rng: np.random.Generator, batch_size: int = 32,
                 minibatch_size: Optional[int] = None, epochs: int = 1, lr: float = 1e-3,
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None,
                 regularizer_factory: Optional[regularizers.RegularizerFactory] = None) -> None:
        super().__init__(preference_model, custom_logger)
        self.loss = loss
        self.batch_size = batch_size
        self.minibatch_size = minibatch_size or batch_size
        if self.batch_size % self.minibatch_size != 0:
            raise ValueError("Batch size must be a multiple of minibatch size.")
        self.epochs = epochs
        params = list(self._preference_model.parameters())
        # AdamW on a GPU -> one-launch flat-buffer step (ops/optim.py); its gradient buffer is
        # also the DP all-reduce bucket
        opt_cls = (optim_ops.fused_for(th.optim.AdamW, params[0].device) if params else None) or th.optim.AdamW
        self.optim = opt_cls(params, lr=lr)
        self.rng = rng
        self.regularizer = regularizer_factory(optimizer=self.optim, logger=self.logger) if regularizer_factory else None

    def _make_data_loader(self, dataset: data_th.Dataset) -> data_th.DataLoader:
        return data_th.DataLoader(dataset, batch_size=self.minibatch_size, shuffle=True, collate_fn=preference_collate_fn,
                                  generator=th.Generator().manual_seed(self._shuffle_seed()))

    def _optimizer_step(self) -> None:
        """``optim.step()`` after averaging the gradients over DP ranks (one collective)."""
        if pdist.world_size() > 1:
            if isinstance(self.optim, optim_ops.FusedAdam):
                for flat in self.optim.flat_grads:
                    pdist.allreduce_grads_flat(flat)
            else:
                pdist.allreduce_grads(self._preference_model.parameters())
        self.optim.step()

    def _dp_graph_ok(self) -> bool:
        """Under DP the graphed minibatch holds its gradient mean (and the RunningNorm
        moments) only on the capturable one-shot all-reduce: FusedAdam's flat buckets must
        fit its staging slot (RCCL / gloo collectives cannot be captured)."""
        if not (pdist.oneshot_active() and isinstance(self.optim, optim_ops.FusedAdam)):
            return False
        from imitation_amd.parallel import oneshot

        return all(oneshot._COMM.fits(f) for f in self.optim.flat_grads)

    def _shuffle_seed(self) -> int:
        """Seed of this epoch set's minibatch order; rank 0's under DP, so every replica walks
        the (identical, all-gathered) dataset in the same order."""
        seed = util.make_seeds(self.rng)
        return int(pdist.broadcast_object(seed)) if pdist.world_size() > 1 else seed

    @property
    def requires_regularizer_update(self) -> bool:
        return self.regularizer is not None and self.regularizer.val_split is not None

    def _fast_path_ok(self, dataset) -> bool:
        """Device-resident minibatching applies: BCE loss on a single reward net, no
        validation split, a plain PreferenceDataset of equal-length array fragments."""
        pm = self._preference_model
        if os.environ.get("IMITATION_AMD_PREF_FAST", "1") == "0":
            return False
        if type(self.loss) is not CrossEntropyRewardLoss or pm.ensemble_model is not None:
            return False
        if self.requires_regularizer_update or not isinstance(dataset, PreferenceDataset) or len(dataset) == 0:
            return False
        if isinstance(dataset.fragments1[0].obs, types.DictObs):
            return False
        return len({len(f) for f in dataset.fragments1} | {len(f) for f in dataset.fragments2}) == 1

    def _train_fast(self, dataset: PreferenceDataset, epoch_multiplier: float) -> int:
        """Same epochs / shuffling (a DataLoader over pair indices, generator seeded from ``self.rng`` as
        the DataLoader does) / gradient accumulation / logged means as the generic loop, but
        the whole dataset is packed and preprocessed ONCE into device tensors; a minibatch
        is a row gather, one reward-net forward over its 2*B*L transitions and the fused
        Bradley-Terry kernel. Per-minibatch metrics stay on device until the epoch ends
        (one host sync per epoch instead of three per minibatch)."""
        pm = self._preference_model
        pairs = list(zip(dataset.fragments1, dataset.fragments2))
        packed = _pack_pairs(pairs)
        s_all, a_all, ns_all, d_all = pm.model.preprocess(packed.state, packed.action, packed.next_state, packed.done)
        dev = s_all.device
        P, L = len(pairs), packed.max_len
        prefs_all = th.as_tensor(dataset.preferences, device=dev)
        gt = None
        if _trajectory_pair_includes_reward(pairs[0]):
            gt = th.as_tensor(np.stack([np.asarray(f.rews, np.float32) for pr in pairs for f in pr]), device=dev).view(P, 2, L)
        span = th.arange(2 * L, device=dev)
        # a DataLoader over the pair indices: the generator is consumed exactly as by the
        # DataLoader of the generic loop (base seed + permutation per epoch)
        index_loader = data_th.DataLoader(range(P), batch_size=self.minibatch_size, shuffle=True,
                                          generator=th.Generator().manual_seed(self._shuffle_seed()))
        epochs = round(self.epochs * epoch_multiplier)
        assert epochs > 0, "Must train for at least one epoch."
        B = self.minibatch_size
        # Data parallel: the dataset is replicated (fragments are all-gathered before push)
        # and the epoch order agreed; a GLOBAL minibatch is world x minibatch_size pairs of
        # which rank r takes slice r, and the gradients are averaged before every optimizer
        # step -- i.e. one rank training with minibatch world x B (the RunningNorm moments are
        # all-reduced inside the forward). The epoch order is cut to a multiple of world so
        # that the last global minibatch splits evenly.
        world, rank = pdist.world_size(), pdist.rank()
        G = B * world
        graph = None
        from imitation_amd.engine import reward_model

        if (dev.type == "cuda" and self.minibatch_size == self.batch_size and self.regularizer is None
                and (world == 1 or self._dp_graph_ok() or reward_model.fused_check(self)[0])
                and os.environ.get("IMITATION_AMD_PREF_GRAPH", "1") != "0"):
            graph = self._minibatch_graph(s_all, a_all, ns_all, d_all, prefs_all, gt, P, L, B)
        if (graph is not None and graph.fused is not None and graph.fused.capturable and world == 1
                and os.environ.get("IMITATION_AMD_PREF_EPOCH_GRAPH", "1") != "0"):
            with self.logger.accumulate_means("reward"):
                return self._train_fused_epochs(graph, index_loader, epochs, P, dev)
        epoch_num = 0
        with self.logger.accumulate_means("reward"):
            for epoch_num in range(epochs):
                order = th.cat(list(index_loader)).to(dev, non_blocking=True)
                if world > 1:
                    order = order[: P - P % world]
                recs = []
                accumulated = 0
                self.optim.zero_grad()
                for start in range(0, order.shape[0], G):
                    n_glob = int(min(G, order.shape[0] - start))
                    n = n_glob // world
                    idx = order[start + rank * n : start + (rank + 1) * n]
                    if graph is not None:
                        recs.append(graph.run(idx))
                        continue
                    rows = (idx[:, None] * (2 * L) + span).reshape(-1)
                    rews = pm.model(s_all.index_select(0, rows), a_all.index_select(0, rows),
                                    ns_all.index_select(0, rows), d_all.index_select(0, rows)).view(n, 2, L)
                    prefs = prefs_all.index_select(0, idx)
                    loss, probs = pref_ops.bradley_terry(rews[:, 0], rews[:, 1], prefs, pm.discount_factor, pm.threshold,
                                                         pm.noise_prob)
                    rec = [loss.detach(), ((probs.detach() > 0.5) == (prefs > 0.5)).float().mean()]
                    if gt is not None:
                        g = gt.index_select(0, idx)
                        gp = pref_ops.bradley_terry_probs_reference(g[:, 0], g[:, 1], pm.discount_factor, pm.threshold,
                                                                    pm.noise_prob)
                        rec.append(th.nn.functional.binary_cross_entropy(gp, prefs))
                    recs.append(th.stack(rec))
                    loss = loss * (n / self.batch_size)
                    if self.regularizer:
                        self.regularizer.regularize_and_backward(loss)
                    else:
                        loss.backward()
                    accumulated += n
                    if accumulated >= self.batch_size:
                        self._optimizer_step()
                        self.optim.zero_grad()
                        accumulated = 0
                if accumulated != 0:
                    self._optimizer_step()
                names = ["loss", "accuracy", "gt_reward_loss"]
                with self.logger.add_key_prefix(f"epoch-{epoch_num}"), self.logger.add_key_prefix("train"):
                    for vals in th.stack(recs).cpu().tolist():
                        for k, v in zip(names, vals):
                            self.logger.record(k, v)
        return epoch_num

    def _train_fused_epochs(self, store: "_MinibatchGraph", index_loader, epochs: int, P: int, dev) -> int:
        """All epochs on the fused minibatch kernels with ONE host sync: the epoch orders (the
        same DataLoader permutations as the minibatch loop) go to the device up front, one
        epoch -- every minibatch plus the metrics copy -- is captured as a HIP graph reading
        its pair ids at a device epoch cursor, epoch 0 runs eagerly as the capture's warm-up
        and the graph is replayed for the others; the logged per-minibatch metrics are read
        back once at the end."""
        fm = store.fused
        B = self.minibatch_size
        n_mb = -(-P // B)
        orders = th.stack(_epoch_orders(index_loader, P, epochs)).to(dev, non_blocking=True)
        cursor = th.zeros(1, dtype=th.int32, device=dev)
        ep = th.zeros(n_mb * 8, device=dev)
        allm = th.zeros(epochs, n_mb, 8, device=dev)
        merge = fm.norm is not None and fm.norm.training
        side = th.cuda.Stream()
        side.wait_stream(th.cuda.current_stream())
        with th.cuda.stream(side):  # warm-up == epoch 0
            fm.plan.epoch(orders, P, cursor, ep, allm, merge)
        th.cuda.current_stream().wait_stream(side)
        if epochs > 1:
            import os

            # a few epochs (the per-iteration schedule) launch eagerly: one C++ call per epoch
            # issues its n_mb x 4 kernels faster than the device runs them, and a capture would
            # cost a device sync + cache flush + instantiate every iteration (the dataset grows,
            # so the graph cannot be kept); long schedules (the initial x200 epochs) replay a graph
            min_ep = int(os.environ.get("IMITATION_AMD_PREF_EPOCH_GRAPH_MIN", "8"))
            if epochs - 1 < min_ep:
                for _ in range(epochs - 1):
                    fm.plan.epoch(orders, P, cursor, ep, allm, merge)
            else:
                graph = th.cuda.CUDAGraph()
                with graphs.capture(graph):
                    fm.plan.epoch(orders, P, cursor, ep, allm, merge)
                for _ in range(epochs - 1):
                    graph.replay()
        vals = allm[:, :, : fm.n_metrics].cpu().tolist()
        names = ["loss", "accuracy", "gt_reward_loss"]
        for epoch_num in range(epochs):
            with self.logger.add_key_prefix(f"epoch-{epoch_num}"), self.logger.add_key_prefix("train"):
                for rec in vals[epoch_num]:
                    for k, v in zip(names, rec):
                        self.logger.record(k, v)
        return epochs - 1

    def _minibatch_graph(self, s_all, a_all, ns_all, d_all, prefs_all, gt, P: int, L: int, B: int) -> "_MinibatchGraph":
        """The persistent HIP-graph of one full minibatch step (re-captured only when the
        dataset outgrows its device buffers or the shapes change)."""
        key = (L, B, tuple(s_all.shape[1:]), tuple(a_all.shape[1:]), tuple(ns_all.shape[1:]), tuple(d_all.shape[1:]),
               s_all.dtype, a_all.dtype, gt is not None, s_all.device)
        g = getattr(self, "_mb_graph", None)
        if g is None or g.key != key or g.capacity < P:
            # capacity doubling, capped by what fits in half of the free HBM (an MI355X holds
            # tens of millions of Walker fragment pairs): the store never overshoots into OOM
            cap = 1 << max(0, (P - 1).bit_length())
            if s_all.is_cuda:
                from imitation_amd.data.buffer import hbm_capacity

                per_pair = 2 * L * sum(t[:1].numel() * t.element_size() for t in (s_all, a_all, ns_all, d_all)) + 4
                if g is not None:  # the old store is released before the new one is allocated
                    per_free = g.capacity * per_pair
                else:
                    per_free = 0
                fits = hbm_capacity(per_pair, fraction=0.5, device=s_all.device,
                                    free_bytes=th.cuda.mem_get_info(s_all.device)[0] + per_free)
                if fits < P:
                    raise MemoryError(f"{P} preference pairs need {P * per_pair / 2**30:.1f} GiB; "
                                      f"half the free HBM holds {fits}")
                cap = max(P, min(cap, fits))
            self._mb_graph = g = None
            g = _MinibatchGraph(self, key, cap, s_all, a_all, ns_all, d_all, gt is not None, L, B)
            self._mb_graph = g
        g.load(s_all, a_all, ns_all, d_all, prefs_all, gt, P)
        return g

    def _record_final(self, epoch_num: int) -> None:
        """Record the last epoch's means under ``reward/final/...``."""
        outer_prefix = self.logger.get_accumulate_prefixes()
        base_path = f"{outer_prefix}reward/"
        pattern = re.compile(rf"mean/{re.escape(base_path)}epoch-{epoch_num}/(.+)")
        for key in list(self.logger.name_to_value.keys()):
            m = pattern.match(key)
            if m:
                self.logger.record(f"{base_path}final/{m.group(1)}", self.logger.name_to_value[key])

    def _train(self, dataset: PreferenceDataset, epoch_multiplier: float = 1.0) -> None:
        if self._fast_path_ok(dataset):
            self._record_final(self._train_fast(dataset, epoch_multiplier))
            return
        if self.regularizer is not None and self.regularizer.val_split is not None:
            val_length = int(len(dataset) * self.regularizer.val_split)
            train_length = len(dataset) - val_length
            if val_length < 1 or train_length < 1:
                raise ValueError("Not enough data samples to split into training and validation, or the validation "
                                 "split is too large/small. Make sure you've generated enough initial preference data. "
                                 "You can adjust this through initial_comparison_frac in PreferenceComparisons.")
            train_ds, val_ds = data_th.random_split(dataset, lengths=[train_length, val_length],
                                                    generator=th.Generator().manual_seed(util.make_seeds(self.rng)))
            dataloader = self._make_data_loader(train_ds)
            val_dataloader = self._make_data_loader(val_ds)
        else:
            dataloader = self._make_data_loader(dataset)
            val_dataloader = None
        epochs = round(self.epochs * epoch_multiplier)
        assert epochs > 0, "Must train for at least one epoch."
        epoch_num = 0
        with self.logger.accumulate_means("reward"):
            for epoch_num in _tqdm(range(epochs), desc="Training reward model", disable=True):
                with self.logger.add_key_prefix(f"epoch-{epoch_num}"):
                    train_loss = 0.0
                    accumulated = 0
                    self.optim.zero_grad()
                    for fragment_pairs, preferences in dataloader:
                        with self.logger.add_key_prefix("train"):
                            loss = self._training_inner_loop(fragment_pairs, preferences)
                            loss = loss * (len(fragment_pairs) / self.batch_size)
                        train_loss += loss.item()
                        if self.regularizer:
                            self.regularizer.regularize_and_backward(loss)
                        else:
                            loss.backward()
                        accumulated += len(fragment_pairs)
                        if accumulated >= self.batch_size:
                            self._optimizer_step()
                            self.optim.zero_grad()
                            accumulated = 0
                    if accumulated != 0:
                        self._optimizer_step()
                    if not self.requires_regularizer_update:
                        continue
                    assert val_dataloader is not None and self.regularizer is not None
                    val_loss = 0.0
                    with th.no_grad():
                        for fragment_pairs, preferences in val_dataloader:
                            with self.logger.add_key_prefix("val"):
                                val_loss += self._training_inner_loop(fragment_pairs, preferences).item()
                    self.regularizer.update_params(train_loss, val_loss)
        self._record_final(epoch_num)

    def _training_inner_loop(self, fragment_pairs, preferences: np.ndarray) -> th.Tensor:
        output = self.loss.forward(fragment_pairs, preferences, self._preference_model)
        self.logger.record("loss", output.loss.item())
        for name, value in output.metrics.items():
            self.logger.record(name, value.item())
        return output.loss


def _epoch_orders(index_loader: data_th.DataLoader, P: int, epochs: int) -> List[th.Tensor]:
    """The pair order of each of ``epochs`` passes of a shuffling DataLoader over range(P).

    An epoch of that loader draws one int64 from its generator (the iterator's base seed),
    one ``randperm(P)`` (RandomSampler) and, when the sampler is drained, a second one for its
    empty remainder; replaying exactly those draws costs ~20 us per epoch instead of ~0.5 ms
    of DataLoader iteration. The first two epochs are checked against the loader itself (on
    the restored generator state); any mismatch falls back to iterating it."""
    g = index_loader.generator
    def draw(gen: th.Generator) -> th.Tensor:
        th.empty((), dtype=th.int64).random_(generator=gen)
        perm = th.randperm(P, generator=gen)
        th.randperm(P, generator=gen)
        return perm

    if g is not None and isinstance(index_loader.sampler, data_th.RandomSampler) and not index_loader.sampler.replacement:
        state = g.get_state()
        probe = th.Generator()
        probe.set_state(state)
        fast = [draw(probe) for _ in range(2)]
        ref = [th.cat(list(index_loader)) for _ in range(2)]
        g.set_state(state)
        if all(th.equal(a, b) for a, b in zip(fast, ref)):
            return [draw(g) for _ in range(epochs)]
    return [th.cat(list(index_loader)) for _ in range(epochs)]


class _MinibatchGraph:
    """One reward-model minibatch step (row gather -> reward net fwd (incl. RunningNorm
    update) -> fused Bradley-Terry loss -> backward -> AdamW step, plus the logged
    metrics) captured as a HIP graph over device-resident dataset buffers, one graph per
    minibatch size (full, and the epoch's last partial one); a minibatch is then an index
    copy and a graph replay instead of ~100 eager launches. The first minibatch of each
    size runs eagerly on a side stream (the warm-up IS that minibatch's step), the capture
    follows. Semantics are the eager loop's with minibatch == batch and no regulariser: a
    partial minibatch's loss is scaled by n / batch and stepped at the epoch end, which is
    the same single step. The optimiser runs in ``capturable`` mode; gradients live in the
    graphs' pools."""

    def __init__(self, trainer: "BasicRewardTrainer", key, capacity: int, s_all, a_all, ns_all, d_all, has_gt: bool,
                 L: int, B: int):
        self.key, self.capacity, self.L, self.B = key, capacity, L, B
        self.trainer = trainer
        dev = s_all.device
        rows = capacity * 2 * L
        mk = lambda t: th.zeros((rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
        self.s, self.a, self.ns, self.d = mk(s_all), mk(a_all), mk(ns_all), mk(d_all)
        self.prefs = th.zeros(capacity, device=dev)
        self.gt = th.zeros(capacity, 2, L, device=dev) if has_gt else None
        self.span = th.arange(2 * L, device=dev)
        self.graphs: Dict[int, Tuple[th.Tensor, Any, Any]] = {}  # n -> (idx buffer, graph, metrics out)
        # the fused four-launch minibatch (engine/reward_model.py) when the reward net and
        # optimizer qualify; it reads these buffers (dones as float32)
        from imitation_amd.engine import reward_model

        self.d_f = self.d.float() if self.d.dtype != th.float32 else self.d
        self.fused = reward_model.maybe_fused(trainer, self, L, B)

    def load(self, s_all, a_all, ns_all, d_all, prefs_all, gt, P: int) -> None:
        n = s_all.shape[0]
        self.s[:n].copy_(s_all)
        self.a[:n].copy_(a_all)
        self.ns[:n].copy_(ns_all)
        self.d[:n].copy_(d_all)
        if self.d_f is not self.d:
            self.d_f[:n].copy_(d_all)
        self.prefs[:P].copy_(prefs_all)
        if gt is not None:
            self.gt[:P].copy_(gt)

    def _step(self, idx: th.Tensor) -> th.Tensor:
        if self.fused is not None:
            return self.fused.step(idx)
        tr = self.trainer
        pm = tr._preference_model
        n, L = idx.shape[0], self.L
        rows = (idx[:, None] * (2 * L) + self.span).reshape(-1)
        # the four transition fields in ONE gather launch, preferences (+ ground truth) in another
        s_, a_, ns_, d_ = rl_ops.gather_rows([self.s, self.a, self.ns, self.d], rows)
        rews = pm.model(s_, a_, ns_, d_).view(n, 2, L)
        per_pair = rl_ops.gather_rows([self.prefs] + ([self.gt] if self.gt is not None else []), idx)
        prefs = per_pair[0]
        loss, probs = pref_ops.bradley_terry(rews[:, 0], rews[:, 1], prefs, pm.discount_factor, pm.threshold,
                                             pm.noise_prob)
        rec = [loss.detach(), ((probs.detach() > 0.5) == (prefs > 0.5)).float().mean()]
        if self.gt is not None:
            g = per_pair[1]
            gp = pref_ops.bradley_terry_probs_reference(g[:, 0], g[:, 1], pm.discount_factor, pm.threshold, pm.noise_prob)
            rec.append(th.nn.functional.binary_cross_entropy(gp, prefs))
        (loss * (n / tr.batch_size)).backward()
        tr._optimizer_step()  # under DP: the one-shot gradient mean, captured with the step
        return th.stack(rec)

    def run(self, idx: th.Tensor) -> th.Tensor:
        """One minibatch step; returns its metrics (a fresh device tensor)."""
        n = int(idx.shape[0])
        opt = self.trainer.optim
        if self.fused is not None and not self.fused.capturable:  # DP fused step: collectives, eager
            return self.fused.step(idx).clone()
        if n in self.graphs:
            buf, graph, out = self.graphs[n]
            buf.copy_(idx)
            graph.replay()
            return out.clone()
        for grp in opt.param_groups:
            grp["capturable"] = True
        for st in opt.state.values():
            if "step" in st and not st["step"].is_cuda:
                st["step"] = st["step"].to(idx.device, th.float32)
        buf = idx.clone()
        side = th.cuda.Stream()
        side.wait_stream(th.cuda.current_stream())
        with th.cuda.stream(side):  # warm-up == this minibatch's real step
            opt.zero_grad(set_to_none=True)
            rec = self._step(buf).clone()  # (the fused step returns a view of its metrics buffer)
        th.cuda.current_stream().wait_stream(side)
        opt.zero_grad(set_to_none=True)
        graph = th.cuda.CUDAGraph()
        with graphs.capture(graph):
            out = self._step(buf)
        self.graphs[n] = (buf, graph, out)
        return rec


class EnsembleTrainer(BasicRewardTrainer):
    """Trains every ensemble member on its own bootstrap resample of the dataset."""

    def __init__(self, preference_model: PreferenceModel, loss: RewardLoss, rng: np.random.Generator, batch_size: int = 32,
                 minibatch_size: Optional[int] = None, epochs: int = 1, lr: float = 1e-3,
                 custom_logger: Optional[imit_logger.HierarchicalLogger] = None,
                 regularizer_factory: Optional[regularizers.RegularizerFactory] = None) -> None:
        if preference_model.ensemble_model is None:
            raise TypeError("PreferenceModel of a RewardEnsemble expected by EnsembleTrainer.")
        super().__init__(preference_model, loss=loss, batch_size=batch_size, minibatch_size=minibatch_size, epochs=epochs,
                         lr=lr, custom_logger=custom_logger, rng=rng, regularizer_factory=regularizer_factory)
        self.member_trainers = [
            BasicRewardTrainer(m, loss=loss, batch_size=batch_size, minibatch_size=minibatch_size, epochs=epochs, lr=lr,
                               custom_logger=self.logger, regularizer_factory=regularizer_factory, rng=self.rng)
            for m in self._preference_model.member_pref_models
        ]

    @property
    def logger(self) -> imit_logger.HierarchicalLogger:
        return super().logger

    @logger.setter
    def logger(self, custom_logger: imit_logger.HierarchicalLogger) -> None:
        self._logger = custom_logger
        for t in getattr(self, "member_trainers", []):
            t.logger = custom_logger

    def _batched_ok(self, dataset) -> bool:
        """All members train in one grouped step when they stack (identical BasicRewardNet
        MLPs) and the member trainers would take their fast path; ``IMITATION_AMD_ENSEMBLE_BATCHED=0``
        keeps the reference's member-by-member loop."""
        if os.environ.get("IMITATION_AMD_ENSEMBLE_BATCHED", "1") == "0":
            return False
        ens = self._preference_model.ensemble_model
        if ens is None or ens.stack() is None or type(self.loss) is not CrossEntropyRewardLoss:
            return False
        if self.regularizer is not None or not isinstance(dataset, PreferenceDataset) or len(dataset) == 0:
            return False
        if isinstance(dataset.fragments1[0].obs, types.DictObs):
            return False
        return len({len(f) for f in dataset.fragments1} | {len(f) for f in dataset.fragments2}) == 1

    def _stack_optimizer(self, stack):
        """One (Fused)AdamW over the stacked member parameters (== M independent AdamWs)."""
        if getattr(self, "_stack_opt", None) is None:
            params = [t.clone().requires_grad_(True) for t in stack.gather_params()]
            lr = self.member_trainers[0].optim.defaults["lr"]
            cls = optim_ops.fused_for(th.optim.AdamW, params[0].device) or th.optim.AdamW
            self._stack_params = params
            self._stack_opt = cls(params, lr=lr)
        return self._stack_params, self._stack_opt

    def _train_batched(self, dataset: PreferenceDataset, epoch_multiplier: float) -> None:
        """The reference's bagged member training (same bootstrap bags, per-member epoch
        orders and accumulation, from the same rng draws) with every minibatch of ALL members
        as one grouped forward/backward (``ops.tmlp_grouped``) and one optimizer step."""
        pm = self._preference_model
        ens = pm.ensemble_model
        st = ens.stack()
        M = ens.num_members
        params, opt = self._stack_optimizer(st)
        with th.no_grad():
            for t, g in zip(params, st.gather_params()):
                t.copy_(g)  # members may have changed since the last call (e.g. a checkpoint load)
        norm = st.gather_norm()
        pairs = list(zip(dataset.fragments1, dataset.fragments2))
        packed = _pack_pairs(pairs)
        s_all, a_all, ns_all, d_all = ens.preprocess(packed.state, packed.action, packed.next_state, packed.done)
        x_all = st.features(s_all, a_all, ns_all, d_all)
        dev = x_all.device
        P, L = len(pairs), packed.max_len
        prefs_all = th.as_tensor(dataset.preferences, device=dev)
        gt = None
        if _trajectory_pair_includes_reward(pairs[0]):
            gt = th.as_tensor(np.stack([np.asarray(f.rews, np.float32) for pr in pairs for f in pr]), device=dev).view(P, 2, L)
        # rng draws in the reference's order: the bagging sampler, then each member trainer's
        # DataLoader seed
        sampler = data_th.RandomSampler(range(P), replacement=True, num_samples=P,
                                        generator=th.Generator().manual_seed(util.make_seeds(self.rng)))
        bags = th.as_tensor([list(sampler) for _ in range(M)], device=dev)  # [M, P]
        loaders = [data_th.DataLoader(range(P), batch_size=self.minibatch_size, shuffle=True,
                                      generator=th.Generator().manual_seed(t._shuffle_seed())) for t in self.member_trainers]
        epochs = round(self.epochs * epoch_multiplier)
        assert epochs > 0, "Must train for at least one epoch."
        B = self.minibatch_size
        span = th.arange(2 * L, device=dev)
        recs_by_epoch = []
        import contextlib

        sync = pdist.no_norm_sync() if pdist.world_size() > 1 else contextlib.nullcontext()  # replicated compute
        with sync:
            for _ in range(epochs):
                orders = th.stack([th.cat(list(ld)) for ld in loaders]).to(dev)  # [M, P] positions in each bag
                recs = []
                accumulated = 0
                opt.zero_grad()
                for start in range(0, P, B):
                    n = int(min(B, P - start))
                    idx = bags.gather(1, orders[:, start : start + n])  # [M, n] pair indices
                    rows = (idx[..., None] * (2 * L) + span).reshape(M, -1)
                    x = x_all[rows]  # [M, n*2L, din]
                    if norm is not None:
                        st.update_norm(norm, x)
                    rews = st.forward(x, params, norm).view(M * n, 2, L)
                    prefs = prefs_all[idx].reshape(-1)
                    loss, probs = pref_ops.bradley_terry(rews[:, 0], rews[:, 1], prefs, pm.discount_factor, pm.threshold,
                                                         pm.noise_prob)
                    # sum of the members' minibatch means, each scaled like its own trainer's
                    (loss * M * (n / self.batch_size)).backward()
                    with th.no_grad():
                        p2 = probs.detach().view(M, n).clamp(1e-7, 1 - 1e-7)
                        y = prefs.view(M, n)
                        rec = [-(y * p2.log() + (1 - y) * (1 - p2).log()).mean(1), ((p2 > 0.5) == (y > 0.5)).float().mean(1)]
                        if gt is not None:
                            g = gt[idx.reshape(-1)]
                            gp = pref_ops.bradley_terry_probs_reference(g[:, 0], g[:, 1], pm.discount_factor, pm.threshold,
                                                                        pm.noise_prob).view(M, n).clamp(1e-7, 1 - 1e-7)
                            rec.append(-(y * gp.log() + (1 - y) * (1 - gp).log()).mean(1))
                        recs.append(th.stack(rec, 1))  # [M, n_metrics]
                    accumulated += n
                    if accumulated >= self.batch_size:
                        opt.step()
                        opt.zero_grad()
                        accumulated = 0
                if accumulated != 0:
                    opt.step()
                recs_by_epoch.append(th.stack(recs, 1).cpu())  # [M, n_minibatches, n_metrics]
        st.scatter(params, norm)
        names = ["loss", "accuracy", "gt_reward_loss"]
        for m, trainer in enumerate(self.member_trainers):
            with self.logger.add_accumulate_prefix(f"member-{m}"):
                with self.logger.accumulate_means("reward"):
                    for e, recs in enumerate(recs_by_epoch):
                        with self.logger.add_key_prefix(f"epoch-{e}"), self.logger.add_key_prefix("train"):
                            for vals in recs[m].tolist():
                                for k, v in zip(names, vals):
                                    self.logger.record(k, v)
                trainer._record_final(epochs - 1)

    def _train(self, dataset: PreferenceDataset, epoch_multiplier: float = 1.0) -> None:
        if self._batched_ok(dataset):
            self._train_batched(dataset, epoch_multiplier)
        else:
            sampler = data_th.RandomSampler(dataset, replacement=True, num_samples=len(dataset),
                                            generator=th.Generator().manual_seed(util.make_seeds(self.rng)))
            for idx, trainer in enumerate(self.member_trainers):
                bagging = data_th.Subset(dataset, list(sampler))
                with self.logger.add_accumulate_prefix(f"member-{idx}"):
                    trainer.train(bagging, epoch_multiplier=epoch_multiplier)
        metrics = defaultdict(list)
        for key in list(self.logger.name_to_value.keys()):
            if re.match(r"member-(\d+)/reward/(.+)", key) and "final" in key:
                metrics["/".join(key.split("/")[1:])].append(self.logger.name_to_value[key])
        for k, v in metrics.items():
            self.logger.record(k, np.mean(v))
            self.logger.record(k + "_std", np.std(v))


def get_base_model(reward_model: reward_nets.RewardNet) -> reward_nets.RewardNet:
    base_model = reward_model
    while hasattr(base_model, "base"):
        base_model = cast(reward_nets.RewardNet, base_model.base)
    return base_model


def _make_reward_trainer(preference_model: PreferenceModel, loss: RewardLoss, rng: np.random.Generator,
                         reward_trainer_kwargs: Optional[Mapping[str, Any]] = None) -> RewardTrainer:
    kwargs = dict(reward_trainer_kwargs or {})
    if preference_model.ensemble_model is not None:
        return EnsembleTrainer(preference_model, loss, rng=rng, **kwargs)
    return BasicRewardTrainer(preference_model, loss=loss, rng=rng, **kwargs)


def _all_gather_pairs(fragments: Sequence[TrajectoryWithRewPair],
                      preferences: np.ndarray) -> Tuple[List[TrajectoryWithRewPair], np.ndarray]:
    """Concatenate every rank's fragment pairs and preferences in rank order."""
    parts = pdist.all_gather_object((list(fragments), np.asarray(preferences)))
    frags: List[TrajectoryWithRewPair] = []
    for f, _ in parts:
        frags.extend(f)
    return frags, np.concatenate([np.asarray(p) for _, p in parts]).astype(np.float32)


QUERY_SCHEDULES: Dict[str, Callable[[float], float]] = {
    "constant": lambda t: 1.0,
    "hyperbolic": lambda t: 1.0 / (1.0 + t),
    "inverse_quadratic": lambda t: 1.0 / (1.0 + t**2),
}


# --------------------------------------------------------------------------- main loop
class PreferenceComparisons(base.BaseImitationAlgorithm):
    """Alternate: sample trajectories -> fragment -> gather preferences -> train reward -> train agent."""

    def __init__(self, trajectory_generator: TrajectoryGenerator, reward_model: reward_nets.RewardNet, num_iterations: int,
                 fragmenter: Optional[Fragmenter] = None, preference_gatherer: Optional[PreferenceGatherer] = None,
                 reward_trainer: Optional[RewardTrainer] = None, comparison_queue_size: Optional[int] = None,
                 fragment_length: int = 100, transition_oversampling: float = 1, initial_comparison_frac: float = 0.1,
                 initial_epoch_multiplier: float = 200.0, custom_logger: Optional[imit_logger.HierarchicalLogger] = None,
                 allow_variable_horizon: bool = False, rng: Optional[np.random.Generator] = None,
                 query_schedule: Union[str, Callable[[float], float]] = "hyperbolic") -> None:
        super().__init__(custom_logger=custom_logger, allow_variable_horizon=allow_variable_horizon)
        if pdist.world_size() > 1:  # every replica starts from rank 0's reward model
            pdist.broadcast_module(reward_model)
        self._iteration = 0
        self._completed_iterations = 0  # iterations of the current train() call done (checkpoint state)
        self._resume_at = 0  # set by a checkpoint restore: the next train() skips this many iterations
        self.model = reward_model
        self.rng = rng
        any_default = None in (preference_gatherer, fragmenter, reward_trainer)
        if self.rng is None and any_default:
            raise ValueError("If you don't provide a random state, you must provide your own seeded fragmenter, "
                             "preference gatherer, and reward_trainer. You can initialize a random state with "
                             "`np.random.default_rng(seed)`.")
        if self.rng is not None and not any_default:
            raise ValueError("If you provide your own fragmenter, preference gatherer, and reward trainer, you don't "
                             "need to provide a random state.")
        if reward_trainer is None:
            assert self.rng is not None
            self.reward_trainer = _make_reward_trainer(PreferenceModel(reward_model), CrossEntropyRewardLoss(), rng=self.rng)
        else:
            self.reward_trainer = reward_trainer
        self.reward_trainer.logger = self.logger
        self.trajectory_generator = trajectory_generator
        self.trajectory_generator.logger = self.logger
        if fragmenter:
            self.fragmenter = fragmenter
        else:
            assert self.rng is not None
            self.fragmenter = RandomFragmenter(custom_logger=self.logger, rng=self.rng)
        self.fragmenter.logger = self.logger
        if preference_gatherer:
            self.preference_gatherer = preference_gatherer
        else:
            assert self.rng is not None
            self.preference_gatherer = SyntheticGatherer(custom_logger=self.logger, rng=self.rng)
        self.preference_gatherer.logger = self.logger
        self.fragment_length = fragment_length
        self.initial_comparison_frac = initial_comparison_frac
        self.initial_epoch_multiplier = initial_epoch_multiplier
        self.num_iterations = num_iterations
        self.transition_oversampling = transition_oversampling
        if callable(query_schedule):
            self.query_schedule = query_schedule
        elif query_schedule in QUERY_SCHEDULES:
            self.query_schedule = QUERY_SCHEDULES[query_schedule]
        else:
            raise ValueError(f"Unknown query schedule: {query_schedule}")
        self.dataset = PreferenceDataset(max_size=comparison_queue_size)

    def train(self, total_timesteps: int, total_comparisons: int,
              callback: Optional[Callable[[int], None]] = None) -> Mapping[str, Any]:
        """Run every iteration (reference ``preference_comparisons.py:1656-1753``)."""
        out: Mapping[str, Any] = {"reward_loss": None, "reward_accuracy": None}
        for out in self.train_iter(total_timesteps, total_comparisons, callback):
            pass
        return out

    def train_iter(self, total_timesteps: int, total_comparisons: int,
                   callback: Optional[Callable[[int], None]] = None):
        """:meth:`train` as a generator: yields ``{"reward_loss", "reward_accuracy"}`` after each
        iteration (for per-iteration timing / external control). The heap from before the loop
        is kept out of the garbage collector's full passes meanwhile (``utils/gcfreeze.py``)."""
        with gcfreeze.frozen_heap():
            yield from self._train_iter(total_timesteps, total_comparisons, callback)

    def _train_iter(self, total_timesteps: int, total_comparisons: int, callback: Optional[Callable[[int], None]]):
        initial_comparisons = int(total_comparisons * self.initial_comparison_frac)
        total_comparisons -= initial_comparisons
        probs = np.vectorize(self.query_schedule)(np.linspace(0, 1, self.num_iterations))
        probs = probs / np.sum(probs)
        shares = util.oric(probs * total_comparisons)
        schedule = [initial_comparisons] + shares.tolist()
        print(f"Query schedule: {schedule}")
        timesteps_per_iteration, extra_timesteps = divmod(total_timesteps, self.num_iterations)
        reward_loss = reward_accuracy = None
        # resumed from a checkpoint taken after iteration `start` - 1 (utils/checkpoint.py): the
        # schedule is recomputed identically and the finished iterations are skipped
        start, self._resume_at = (self._resume_at if self._resume_at < len(schedule) else 0), 0
        self._completed_iterations = start
        for i, num_pairs in enumerate(schedule):
            if i < start:
                continue
            num_steps = math.ceil(self.transition_oversampling * 2 * num_pairs * self.fragment_length)
            self.logger.log(f"Collecting {2 * num_pairs} fragments ({num_steps} transitions)")
            with profiling.range("pref/sample"):
                trajectories = self.trajectory_generator.sample(num_steps)
            self._check_fixed_horizon(len(t) for t in trajectories if t.terminal)
            self.logger.log("Creating fragment pairs")
            with profiling.range("pref/fragment"):
                fragments = self.fragmenter(trajectories, self.fragment_length, num_pairs)
            with self.logger.accumulate_means("preferences"), profiling.range("pref/gather"):
                self.logger.log("Gathering preferences")
                preferences = self.preference_gatherer(fragments)
            if pdist.world_size() > 1:
                # every rank sampled and labelled its own pairs; all replicas push the same
                # rank-ordered union, so the reward models stay identical
                fragments, preferences = _all_gather_pairs(fragments, preferences)
            self.dataset.push(fragments, preferences)
            self.logger.log(f"Dataset now contains {len(self.dataset)} comparisons")
            epoch_multiplier = self.initial_epoch_multiplier if i == 0 else 1.0
            with profiling.range("pref/reward_train"):
                self.reward_trainer.train(self.dataset, epoch_multiplier=epoch_multiplier)
            base_key = self.logger.get_accumulate_prefixes() + "reward/final/train"
            assert f"{base_key}/loss" in self.logger.name_to_value
            assert f"{base_key}/accuracy" in self.logger.name_to_value
            reward_loss = self.logger.name_to_value[f"{base_key}/loss"]
            reward_accuracy = self.logger.name_to_value[f"{base_key}/accuracy"]
            if not math.isfinite(float(reward_loss)):  # already a host float: fail fast, no extra sync
                from imitation_amd.utils.watchdog import NonFiniteError

                raise NonFiniteError(f"non-finite reward-model loss in preference iteration {i}: {reward_loss}")
            steps = timesteps_per_iteration + (extra_timesteps if i == self.num_iterations - 1 else 0)
            with self.logger.accumulate_means("agent"):
                self.logger.log(f"Training agent for {steps} timesteps")
                with profiling.range("pref/agent_train"):
                    self.trajectory_generator.train(steps=steps)
            # the last iteration's collectives are checked blocking: a NaN-poisoned one-shot
            # all-reduce there must raise, not return NaN weights
            pdist.check_comm("preference iteration", blocking=i == len(schedule) - 1)
            check = getattr(self.trajectory_generator, "check_errors", None)  # device agent (PPO kernel)
            if check is not None:
                check(blocking=i == len(schedule) - 1)
            self.logger.dump(self._iteration)
            self._completed_iterations = i + 1
            self._iteration += 1  # before the callback: a checkpoint taken there resumes at the next iteration
            if callback:
                callback(self._iteration - 1)
            yield {"reward_loss": reward_loss, "reward_accuracy": reward_accuracy}

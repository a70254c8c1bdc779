"""Algorithm base classes (reference: ``src/imitation/algorithms/base.py``).

* :class:`BaseImitationAlgorithm` -- logger plumbing, ``_check_fixed_horizon``
  (``base.py:77-110``), logger dropped on pickling (``:112-121``);
* :class:`DemonstrationAlgorithm` -- ``set_demonstrations`` + ``policy``;
* :func:`make_data_loader` (``:226-288``) -- trajectories are flattened; flat
  transitions are served shuffled with ``drop_last``.

Data path: for flat transitions the loader is a vectorised sampler (one numpy
fancy-index per batch and one collate) instead of a per-sample ``__getitem__``
+ ``default_collate`` DataLoader; it yields the exact same batch structure
(``obs``/``next_obs`` arrays, ``acts``/``dones`` tensors, ``infos`` list). Under
data parallelism each rank draws its own random order (rank-seeded), i.e. every
rank samples minibatches from the full demonstration set.
"""

from __future__ import annotations

import abc
from typing import Any, Generic, Iterable, Iterator, Mapping, Optional, TypeVar, Union, cast

import numpy as np
import torch as th
import torch.utils.data as th_data

from imitation_amd.data import rollout, types
from imitation_amd.util import logger as imit_logger
from imitation_amd.util import util


class BaseImitationAlgorithm(abc.ABC):
    """Base class for all imitation learning algorithms."""

    def __init__(self, *, custom_logger: Optional[imit_logger.HierarchicalLogger] = None, allow_variable_horizon: bool = False):
        self._logger = custom_logger or imit_logger.configure()
        self.allow_variable_horizon = allow_variable_horizon
        if allow_variable_horizon:
            self.logger.warn(
                "Running with `allow_variable_horizon` set to True. Some algorithms are biased towards shorter or longer "
                "episodes, which may significantly confound results. Additionally, even unbiased algorithms can exploit "
                "the information leak from the termination condition, producing spuriously high performance. See "
                "https://imitation.readthedocs.io/en/latest/getting-started/variable-horizon.html for more information."
            )
        self._horizon: Optional[int] = None

    @property
    def logger(self) -> imit_logger.HierarchicalLogger:
        return self._logger

    @logger.setter
    def logger(self, value: imit_logger.HierarchicalLogger) -> None:
        self._logger = value

    def _check_fixed_horizon(self, horizons: Iterable[int]) -> None:
        """Raise if episodes of different lengths were seen (unless allowed)."""
        if self.allow_variable_horizon:
            return
        horizons = set(int(h) for h in horizons)
        if self._horizon is not None:
            horizons.add(self._horizon)
        if len(horizons) > 1:
            raise ValueError(
                f"Episodes of different length detected: {horizons}. Variable horizon environments are discouraged -- "
                "termination conditions leak information about reward. See "
                "https://imitation.readthedocs.io/en/latest/getting-started/variable-horizon.html for more information. "
                "If you are SURE you want to run imitation on a variable horizon task, then please pass in the flag: "
                "`allow_variable_horizon=True`."
            )
        elif len(horizons) == 1:
            self._horizon = horizons.pop()

    def __getstate__(self):
        state = self.__dict__.copy()
        del state["_logger"]
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        self.logger = state.get("_logger") or imit_logger.configure()


TransitionKind = TypeVar("TransitionKind", bound=types.TransitionsMinimal)
AnyTransitions = Union[Iterable[types.Trajectory], Iterable[types.TransitionMapping], types.TransitionsMinimal]


class DemonstrationAlgorithm(BaseImitationAlgorithm, Generic[TransitionKind]):
    """An algorithm that learns from demonstration: BC, IRL, etc."""

    def __init__(self, *, demonstrations: Optional[AnyTransitions], custom_logger=None, allow_variable_horizon: bool = False):
        super().__init__(custom_logger=custom_logger, allow_variable_horizon=allow_variable_horizon)
        if demonstrations is not None:
            self.set_demonstrations(demonstrations)

    @abc.abstractmethod
    def set_demonstrations(self, demonstrations: AnyTransitions) -> None:
        """Set the demonstration data."""

    @property
    @abc.abstractmethod
    def policy(self):
        """Returns a policy imitating the demonstration data."""


class _WrappedDataLoader:
    """Wraps a data loader (batch iterable) and checks every batch has the expected size."""

    def __init__(self, data_loader: Iterable[types.TransitionMapping], expected_batch_size: int):
        self.data_loader = data_loader
        self.expected_batch_size = expected_batch_size

    def __iter__(self) -> Iterator[types.TransitionMapping]:
        for batch in self.data_loader:
            if len(batch["obs"]) != self.expected_batch_size:
                raise ValueError(f"Expected batch size {self.expected_batch_size} != {len(batch['obs'])} = len(batch['obs'])")
            if len(batch["acts"]) != self.expected_batch_size:
                raise ValueError(f"Expected batch size {self.expected_batch_size} != {len(batch['acts'])} = len(batch['acts'])")
            yield batch


class TransitionsBatchLoader:
    """Vectorised shuffled/drop-last minibatch loader over a flat transitions dataset.

    Batches have the same structure as ``DataLoader(..., collate_fn=transitions_collate_fn)``.
    """

    def __init__(self, dataset: types.TransitionsMinimal, batch_size: int, shuffle: bool = True, drop_last: bool = True,
                 seed: Optional[int] = None):
        self.dataset = dataset
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.drop_last = drop_last
        from imitation_amd.parallel import dist as pdist

        if seed is None:
            seed = int(np.random.randint(0, 2**31 - 1)) + 7919 * pdist.rank()
        self._rng = np.random.default_rng(seed)
        d = types.dataclass_quick_asdict(dataset)
        self._fields = d
        self._has_next = "next_obs" in d

    def __len__(self) -> int:
        n = len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _take(self, arr, idx):
        if isinstance(arr, types.DictObs):
            return arr[idx]
        return np.asarray(arr)[idx]

    def __iter__(self) -> Iterator[types.TransitionMapping]:
        n = len(self.dataset)
        order = self._rng.permutation(n) if self.shuffle else np.arange(n)
        stop = n - (n % self.batch_size) if self.drop_last else n
        for s in range(0, stop, self.batch_size):
            idx = order[s : s + self.batch_size]
            batch = {}
            for k, v in self._fields.items():
                if k == "infos":
                    batch["infos"] = list(np.asarray(v)[idx])
                elif k in ("obs", "next_obs"):
                    batch[k] = self._take(v, idx)
                else:
                    batch[k] = th.as_tensor(np.asarray(v)[idx])
            yield batch


def make_data_loader(transitions: AnyTransitions, batch_size: int, data_loader_kwargs: Optional[Mapping[str, Any]] = None) -> Iterable[types.TransitionMapping]:
    """Convert demonstrations into a minibatch iterable of the given batch size."""
    if batch_size <= 0:
        raise ValueError(f"batch_size={batch_size} must be positive.")
    if isinstance(transitions, Iterable):
        first_item, transitions = util.get_first_iter_element(transitions)  # type: ignore[assignment]
        if isinstance(first_item, types.Trajectory):
            transitions = rollout.flatten_trajectories(list(cast(Iterable[types.Trajectory], transitions)))
    if isinstance(transitions, types.TransitionsMinimal):
        if len(transitions) < batch_size:
            raise ValueError(f"Number of transitions in `demonstrations` {len(transitions)} is smaller than batch size {batch_size}.")
        kwargs = {"shuffle": True, "drop_last": True, **(data_loader_kwargs or {})}
        if set(kwargs) <= {"shuffle", "drop_last"}:
            return TransitionsBatchLoader(transitions, batch_size, shuffle=kwargs["shuffle"], drop_last=kwargs["drop_last"])
        return th_data.DataLoader(transitions, batch_size=batch_size, collate_fn=types.transitions_collate_fn, **kwargs)
    elif isinstance(transitions, Iterable):
        return _WrappedDataLoader(transitions, batch_size)  # type: ignore[arg-type]
    raise TypeError(f"`demonstrations` unexpected type {type(transitions)}")

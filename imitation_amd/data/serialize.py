"""Trajectory (de)serialisation (reference: ``src/imitation/data/serialize.py``).

* :func:`save` writes a HuggingFace ``datasets`` directory (``save_to_disk``);
* :func:`load` reads that format, or the legacy ``.npz`` layout (``obs`` with one
  extra row per trajectory, split points in ``indices``). Legacy ``.npz`` files are
  opened with ``allow_pickle=False``: their object-dtype ``infos`` column cannot be
  read without unpickling, so it is dropped (``infos=None``) unless the caller
  explicitly opts in with ``allow_pickle=True`` for a file it trusts. Legacy
  pickled trajectory lists are refused unless ``allow_pickle=True``.
"""

from __future__ import annotations

import logging
import os
import warnings
from typing import Mapping, Sequence, cast

import numpy as np

from imitation_amd.data import huggingface_utils
from imitation_amd.data.types import AnyPath, Trajectory, TrajectoryWithRew
from imitation_amd.util import util


def save(path: AnyPath, trajectories: Sequence[Trajectory]) -> None:
    """Save trajectories to a HuggingFace dataset directory at ``path``."""
    p = str(util.parse_path(path))
    import datasets

    was_enabled = datasets.utils.logging.is_progress_bar_enabled()
    datasets.utils.logging.disable_progress_bar()  # one bar per demo file otherwise
    try:
        huggingface_utils.trajectories_to_dataset(trajectories).save_to_disk(p)
    finally:
        if was_enabled:
            datasets.utils.logging.enable_progress_bar()
    logging.info(f"Dumped demonstrations to {p}.")


def _load_npz(path, allow_pickle: bool):
    data = np.load(path, allow_pickle=allow_pickle)
    if not hasattr(data, "files"):
        raise ValueError(f"{path} is not an .npz archive")
    warnings.warn("Loading old npz version of Trajectories", DeprecationWarning)
    num_trajs = len(data["indices"])
    try:
        infos = np.split(data["infos"], data["indices"])
    except ValueError:
        infos = [None] * (num_trajs + 1)
    fields = [
        np.split(data["obs"], data["indices"] + np.arange(num_trajs) + 1),
        np.split(data["acts"], data["indices"]),
        infos,
        data["terminal"],
    ]
    if "rews" in data.files:
        fields = [*fields, np.split(data["rews"], data["indices"])]
        return [TrajectoryWithRew(*args) for args in zip(*fields)]
    return [Trajectory(*args) for args in zip(*fields)]


def load(path: AnyPath, allow_pickle: bool = False) -> Sequence[Trajectory]:
    """Load trajectories from ``path`` (HF dataset dir or legacy ``.npz``)."""
    if os.path.isdir(path):
        import datasets

        dataset = datasets.load_from_disk(str(path))
        if not isinstance(dataset, datasets.Dataset):  # pragma: no cover
            raise ValueError(f"Expected to load a `datasets.Dataset` but got {type(dataset)}")
        return huggingface_utils.TrajectoryDatasetSequence(dataset)
    with open(path, "rb") as f:
        magic = f.read(4)
    if magic[:2] == b"PK":
        return _load_npz(path, allow_pickle)
    if not allow_pickle:
        raise ValueError(
            f"{path} looks like a legacy pickled trajectory list; refusing to unpickle it. "
            "Convert it with a trusted tool or pass allow_pickle=True for a file you trust."
        )
    import pickle

    with open(path, "rb") as f:  # pragma: no cover - explicit opt-in only
        data = pickle.load(f)  # noqa: pickle -- explicit allow_pickle=True opt-in
    warnings.warn("Loading old pickle version of Trajectories", DeprecationWarning)
    return data


def load_with_rewards(path: AnyPath, allow_pickle: bool = False) -> Sequence[TrajectoryWithRew]:
    data = load(path, allow_pickle=allow_pickle)
    mismatched = [type(t) for t in data if not isinstance(t, TrajectoryWithRew)]
    if mismatched:
        raise ValueError(f"Expected all trajectories to be of type `TrajectoryWithRew`, but found {mismatched[0].__name__}")
    return cast(Sequence[TrajectoryWithRew], data)

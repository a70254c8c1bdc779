"""HuggingFace ``datasets`` adapter for trajectories (reference: ``src/imitation/data/huggingface_utils.py``).

Columns: ``obs`` [T+1, ...], ``acts`` [T, ...], ``infos`` (one JSON string per
step), ``terminal``, optional ``rews``. ``jsonpickle`` is not
installed here; :func:`encode_info` / :func:`decode_info` implement the subset of
its wire format that trajectory infos use (plain JSON values, ``py/tuple``,
numpy arrays as ``py/object: numpy.ndarray``), so files are interchangeable for
plain-dict infos.
"""

from __future__ import annotations

import json
from typing import Any, Dict, Iterable, Optional, Sequence, cast

import datasets
import numpy as np

from imitation_amd.data import types


def _to_jsonable(v: Any) -> Any:
    if isinstance(v, dict):
        return {str(k): _to_jsonable(x) for k, x in v.items()}
    if isinstance(v, tuple):
        return {"py/tuple": [_to_jsonable(x) for x in v]}
    if isinstance(v, list):
        return [_to_jsonable(x) for x in v]
    if isinstance(v, np.ndarray):
        flat = v.reshape(-1)
        if flat.dtype.kind in "biu" or (flat.dtype.kind == "f" and bool(np.isfinite(flat).all())):
            values = flat.tolist()  # already plain JSON scalars: no per-element pass (84x84x4 frames)
        else:
            values = _to_jsonable(flat.tolist())
        return {"py/object": "numpy.ndarray", "dtype": str(v.dtype), "shape": list(v.shape), "values": values}
    if isinstance(v, (np.bool_,)):
        return bool(v)
    if isinstance(v, np.integer):
        return int(v)
    if isinstance(v, np.floating):
        return float(v)
    if isinstance(v, float) and (np.isnan(v) or np.isinf(v)):
        return {"py/float": repr(v)}
    return v


def _from_jsonable(v: Any) -> Any:
    if isinstance(v, dict):
        # tags are only honoured in the exact form the encoder writes them
        if len(v) == 1 and isinstance(v.get("py/tuple"), list):
            return tuple(_from_jsonable(x) for x in v["py/tuple"])
        if v.get("py/object") == "numpy.ndarray" and "values" in v:
            try:  # plain numeric lists convert in C; tagged (nan/inf) entries need the walk
                arr = np.asarray(v["values"], dtype=v.get("dtype", None))
                if arr.dtype == object:
                    raise TypeError
            except (TypeError, ValueError):
                arr = np.asarray(_from_jsonable(v["values"]), dtype=v.get("dtype", None))
            return arr.reshape(v.get("shape", arr.shape))
        if len(v) == 1 and isinstance(v.get("py/float"), str):
            return float(v["py/float"])
        return {k: _from_jsonable(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_from_jsonable(x) for x in v]
    return v


def encode_info(info: Dict[str, Any]) -> str:
    return json.dumps(_to_jsonable(info))


def decode_info(s: str) -> Any:
    return _from_jsonable(json.loads(s))


def _list_scalar_to_numpy(val) -> np.ndarray:
    """Rectangular nested Arrow list value -> ndarray straight from the Arrow buffers.

    The datasets formatters materialise nested lists as Python objects first (minutes for
    a few thousand 84x84x4 frames); flattening the child arrays level by level is a
    buffer copy."""
    import pyarrow as pa

    arr = val.values
    shape = [len(arr)]
    while pa.types.is_list(arr.type) or pa.types.is_large_list(arr.type) or pa.types.is_fixed_size_list(arr.type):
        if len(arr) == 0:
            break
        if pa.types.is_fixed_size_list(arr.type):
            n = arr.type.list_size
        else:
            lens = arr.value_lengths().to_numpy(zero_copy_only=False)
            n = int(lens[0])
            if not (lens == n).all():
                raise ValueError("ragged nested list")
        shape.append(n)
        arr = arr.flatten()
    return arr.to_numpy(zero_copy_only=False).reshape(shape)


class TrajectoryDatasetSequence(Sequence[types.Trajectory]):
    """A sequence of trajectories lazily backed by a HuggingFace dataset."""

    def __init__(self, dataset: datasets.Dataset):
        def numpy_transform(batch):
            return {key: np.asarray(val) if key != "infos" else val for key, val in batch.items()}

        self._raw = dataset
        self._dataset = dataset.with_transform(numpy_transform)
        self._trajectory_class = types.TrajectoryWithRew if "rews" in dataset.features else types.Trajectory
        # Arrow fast path for array columns (no index mapping: row i of the table == item i)
        self._table = dataset.data.table if getattr(dataset, "_indices", None) is None else None

    def __len__(self) -> int:
        return len(self._dataset)

    def _row_fast(self, idx: int) -> Dict[str, Any]:
        t = self._table
        out: Dict[str, Any] = {}
        for key in ("obs", "acts", "rews"):
            if key in t.column_names:
                out[key] = _list_scalar_to_numpy(t.column(key)[idx])
        out["terminal"] = bool(t.column("terminal")[idx].as_py())
        out["infos"] = t.column("infos")[idx].as_py()
        return out

    def __getitem__(self, idx):
        if isinstance(idx, slice):
            return [self[i] for i in range(*idx.indices(len(self)))]
        kwargs = None
        if self._table is not None:
            if idx < 0:
                idx += len(self)
            try:
                kwargs = self._row_fast(int(idx))
            except (ValueError, KeyError, TypeError):
                kwargs = None
        if kwargs is None:
            kwargs = self._dataset[idx]
        kwargs["infos"] = _LazyDecodedList(kwargs["infos"])
        return self._trajectory_class(**kwargs)

    @property
    def dataset(self):
        return self._dataset.with_transform(None)


class _LazyDecodedList(Sequence[Any]):
    """A list of JSON-encoded infos decoded on access (and cached)."""

    def __init__(self, encoded_list: Sequence[str]):
        self._encoded_list = encoded_list
        self._decoded_cache: Dict[int, Any] = {}

    def __len__(self):
        return len(self._encoded_list)

    def __getitem__(self, idx):
        if isinstance(idx, slice):
            return [self[i] for i in range(*idx.indices(len(self)))]
        if idx < 0:
            idx += len(self)
        if idx not in self._decoded_cache:
            self._decoded_cache[idx] = decode_info(self._encoded_list[idx])
        return self._decoded_cache[idx]


def trajectories_to_dict(trajectories: Sequence[types.Trajectory]) -> Dict[str, Sequence[Any]]:
    has_reward = [isinstance(t, types.TrajectoryWithRew) for t in trajectories]
    all_rew = all(has_reward)
    if not all_rew and any(has_reward):
        raise ValueError("Some trajectories have rewards but not all")
    if any(isinstance(t.obs, types.DictObs) for t in trajectories):
        raise ValueError("DictObs are not currently supported")
    d: Dict[str, Sequence[Any]] = dict(
        obs=[t.obs for t in trajectories],
        acts=[t.acts for t in trajectories],
        infos=[[encode_info(i) for i in (t.infos if t.infos is not None else [{}] * len(t))] for t in trajectories],
        terminal=[t.terminal for t in trajectories],
    )
    if all_rew:
        d["rews"] = [cast(types.TrajectoryWithRew, t).rews for t in trajectories]
    return d


def _nested_list_array(arrays: Sequence[np.ndarray]):
    """One row per array: ``[n_i, d1, ..., dk]`` ndarrays (equal trailing dims) as a nested
    Arrow ``list<list<...<dtype>>>`` built over ONE contiguous values buffer with arithmetic
    offsets -- the exact schema ``Dataset.from_dict`` infers from the arrays, without going
    through Python lists (~15x faster for image observations)."""
    import pyarrow as pa

    flat = np.concatenate([np.ascontiguousarray(a).reshape(-1) for a in arrays]) if arrays else np.zeros(0)
    values = pa.array(flat)
    n = flat.size
    for d in reversed(arrays[0].shape[1:]):
        n //= d
        values = pa.ListArray.from_arrays(pa.array(np.arange(n + 1, dtype=np.int32) * d), values)
    outer = np.zeros(len(arrays) + 1, dtype=np.int32)
    np.cumsum([a.shape[0] for a in arrays], out=outer[1:])
    return pa.ListArray.from_arrays(pa.array(outer), values)


def _fast_dataset(trajectories: Sequence[types.Trajectory], info) -> Optional[datasets.Dataset]:
    """Arrow-native build of the same dataset (None when a field needs the generic path)."""
    import pyarrow as pa
    from datasets.table import InMemoryTable

    has_rew = [isinstance(t, types.TrajectoryWithRew) for t in trajectories]
    if not trajectories or (any(has_rew) and not all(has_rew)):
        return None
    cols = {"obs": [t.obs for t in trajectories], "acts": [t.acts for t in trajectories]}
    if all(has_rew):
        cols["rews"] = [cast(types.TrajectoryWithRew, t).rews for t in trajectories]
    for k, arrs in cols.items():
        if not all(isinstance(a, np.ndarray) and a.dtype.kind in "biuf" and a.ndim >= 1 for a in arrs):
            return None
        if len({a.shape[1:] for a in arrs}) != 1 or len({a.dtype for a in arrs}) != 1:
            return None
    d = {"obs": _nested_list_array(cols["obs"]), "acts": _nested_list_array(cols["acts"]),
         "infos": pa.array([[encode_info(i) for i in (t.infos if t.infos is not None else [{}] * len(t))]
                            for t in trajectories], type=pa.list_(pa.string())),
         "terminal": pa.array([bool(t.terminal) for t in trajectories], type=pa.bool_())}
    if "rews" in cols:
        d["rews"] = _nested_list_array(cols["rews"])
    return datasets.Dataset(InMemoryTable(pa.table(d)), info=info)


def trajectories_to_dataset(trajectories: Sequence[types.Trajectory], info: Optional[datasets.DatasetInfo] = None) -> datasets.Dataset:
    if isinstance(trajectories, TrajectoryDatasetSequence):
        return trajectories.dataset
    if not any(isinstance(t.obs, types.DictObs) for t in trajectories):
        fast = _fast_dataset(trajectories, info)
        if fast is not None:
            return fast
    return datasets.Dataset.from_dict(trajectories_to_dict(trajectories), info=info)

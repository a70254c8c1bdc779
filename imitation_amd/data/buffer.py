"""Ring buffers (reference: ``src/imitation/data/buffer.py``).

* :class:`Buffer` (``buffer.py:30-237``): FIFO ring of named arrays, wrap-around
  ``store``, uniform with-replacement ``sample``. Unlike the reference (global
  ``np.random``, ``buffer.py:231``) sampling takes an optional
  injected ``rng`` for reproducibility; the global stream stays the default.
* :class:`ReplayBuffer` (``:240-416``): transitions (obs, acts, next_obs, dones, infos).
* :class:`DeviceBuffer`: the same ring held as device tensors (HBM-resident
  generator replay buffer for the adversarial trainer; sampling is a device
  index-gather).
"""

from __future__ import annotations

from typing import Any, Dict, Mapping, Optional, Tuple

import numpy as np
import torch as th

from imitation_amd.data import types


def num_samples(data: Mapping[Any, np.ndarray]) -> int:
    lens = np.unique([arr.shape[0] for arr in data.values()])
    if len(lens) > 1:
        raise ValueError("Keys map to different length values.")
    return int(lens[0])


class Buffer:
    """A FIFO ring buffer for NumPy arrays of fixed shape and dtype."""

    def __init__(self, capacity: int, sample_shapes: Mapping[str, Tuple[int, ...]], dtypes: Mapping[str, np.dtype]):
        if sample_shapes.keys() != dtypes.keys():
            raise KeyError("sample_shape and dtypes keys don't match")
        self.capacity = capacity
        self.sample_shapes = {k: tuple(s) for k, s in sample_shapes.items()}
        self._arrays = {k: np.zeros((capacity,) + s, dtype=dtypes[k]) for k, s in self.sample_shapes.items()}
        self._n_data = 0
        self._idx = 0

    @classmethod
    def from_data(cls, data: Mapping[str, np.ndarray], capacity: Optional[int] = None, truncate_ok: bool = False) -> "Buffer":
        caps = np.unique([arr.shape[0] for arr in data.values()])
        if len(data) == 0:
            raise ValueError("No keys in data.")
        if len(caps) > 1:
            raise ValueError("Keys map to different length values")
        if capacity is None:
            capacity = int(caps[0])
        buf = cls(capacity, {k: a.shape[1:] for k, a in data.items()}, {k: a.dtype for k, a in data.items()})
        buf.store(data, truncate_ok=truncate_ok)
        return buf

    def store(self, data: Mapping[str, np.ndarray], truncate_ok: bool = False) -> None:
        expected = set(self.sample_shapes)
        missing = expected.difference(data.keys())
        unexpected = set(data.keys()).difference(expected)
        if missing:
            raise ValueError(f"Missing keys {missing}")
        if unexpected:
            raise ValueError(f"Unexpected keys {unexpected}")
        n = num_samples(data)
        if n == 0:
            raise ValueError("Trying to store empty data.")
        if n > self.capacity:
            if not truncate_ok:
                raise ValueError("Not enough capacity to store data.")
            data = {k: a[-self.capacity :] for k, a in data.items()}
        for k, a in data.items():
            if a.shape[1:] != self.sample_shapes[k]:
                raise ValueError(f"Wrong data shape for {k}")
        if self._idx + num_samples(data) > self.capacity:
            n_remain = self.capacity - self._idx
            self._store_easy({k: a[:n_remain] for k, a in data.items()})
            assert self._idx == 0
            self._store_easy({k: a[n_remain:] for k, a in data.items()})
        else:
            self._store_easy(data)

    def _store_easy(self, data: Mapping[str, np.ndarray]) -> None:
        n = num_samples(data)
        assert n <= self.capacity - self._idx
        hi = self._idx + n
        for k, a in data.items():
            self._arrays[k][self._idx : hi] = a
        self._idx = hi % self.capacity
        self._n_data = min(self._n_data + n, self.capacity)

    def sample(self, n_samples: int, rng: Optional[np.random.Generator] = None) -> Mapping[str, np.ndarray]:
        if self.size() == 0:
            raise ValueError("Buffer is empty")
        ind = rng.integers(self.size(), size=n_samples) if rng is not None else np.random.randint(self.size(), size=n_samples)
        return {k: a[ind] for k, a in self._arrays.items()}

    def size(self) -> int:
        assert 0 <= self._n_data <= self.capacity
        return self._n_data


class ReplayBuffer:
    """Buffer of :class:`~imitation_amd.data.types.Transitions`."""

    def __init__(self, capacity: int, venv=None, *, obs_shape=None, act_shape=None, obs_dtype=None, act_dtype=None):
        if venv is not None:
            if venv.observation_space.shape is not None:
                if obs_shape is not None:
                    raise ValueError("Cannot specify both observation shape and also environment with an observation space that has a shape.")
                obs_shape = tuple(venv.observation_space.shape)
            if venv.observation_space.dtype is not None:
                if obs_dtype is not None:
                    raise ValueError("Cannot specify both observation dtype and also environment with an observation space that has a dtype.")
                obs_dtype = venv.observation_space.dtype
            if venv.action_space.shape is not None:
                if act_shape is not None:
                    raise ValueError("Cannot specify both action shape and also environment with an action space that has a shape.")
                act_shape = tuple(venv.action_space.shape)
            if venv.action_space.dtype is not None:
                if act_dtype is not None:
                    raise ValueError("Cannot specify both action dtype and also environment with an action space that has a dtype.")
                act_dtype = venv.action_space.dtype
        elif any(x is None for x in (obs_shape, act_shape, obs_dtype, act_dtype)):
            raise ValueError("Shape or dtype missing and no environment specified.")
        assert obs_shape is not None and act_shape is not None
        self.capacity = capacity
        sample_shapes = {"obs": obs_shape, "acts": act_shape, "next_obs": obs_shape, "dones": (), "infos": ()}
        dtypes = {"obs": obs_dtype, "acts": act_dtype, "next_obs": obs_dtype, "dones": bool, "infos": object}
        self._buffer = Buffer(capacity, sample_shapes=sample_shapes, dtypes=dtypes)

    @classmethod
    def from_data(cls, transitions: types.Transitions, capacity: Optional[int] = None, truncate_ok: bool = False) -> "ReplayBuffer":
        obs_shape = transitions.obs.shape[1:]
        act_shape = transitions.acts.shape[1:]
        if capacity is None:
            capacity = transitions.obs.shape[0]
        inst = cls(capacity=capacity, obs_shape=obs_shape, act_shape=act_shape, obs_dtype=transitions.obs.dtype,
                   act_dtype=transitions.acts.dtype)
        inst.store(transitions, truncate_ok=truncate_ok)
        return inst

    def sample(self, n_samples: int, rng: Optional[np.random.Generator] = None) -> types.Transitions:
        sample = self._buffer.sample(n_samples, rng=rng)
        assert set(sample.keys()) == {f.name for f in types.Transitions.__dataclass_fields__.values()}
        return types.Transitions(**sample)

    def store(self, transitions: types.Transitions, truncate_ok: bool = True) -> None:
        trans = types.dataclass_quick_asdict(transitions)
        trans = {k: trans[k] for k in self._buffer.sample_shapes.keys()}
        if len(trans["acts"]) > 0:
            self._buffer.store(trans, truncate_ok=truncate_ok)

    def size(self) -> Optional[int]:
        return self._buffer.size()


def hbm_capacity(bytes_per_sample: int, *, fraction: float = 0.5, device=None, reserve_bytes: int = 4 << 30,
                 free_bytes: Optional[int] = None) -> int:
    """Rows a device-resident ring can hold in ``fraction`` of the device's currently free
    memory (an MI355X has 288 GB of HBM3E: at the default half of it a Pong frame store
    holds ~5M 84x84x4 transitions), keeping ``reserve_bytes`` back for activations and the
    allocator. ``free_bytes`` overrides the query (tests, planning on the host)."""
    if bytes_per_sample <= 0:
        raise ValueError("bytes_per_sample must be positive")
    if free_bytes is None:
        dev = th.device(device if device is not None else "cuda")
        if dev.type != "cuda":
            raise ValueError("hbm_capacity sizes device buffers; pass free_bytes for a host plan")
        free_bytes, _ = th.cuda.mem_get_info(dev)
    usable = max(0, int(free_bytes * fraction) - reserve_bytes)
    return max(1, usable // int(bytes_per_sample))


class DeviceBuffer:
    """Ring buffer of named device tensors with device-side uniform sampling (one
    multi-field gather launch per draw, ``ops.rl.gather_rows``)."""

    @classmethod
    def sized_to_hbm(cls, sample_shapes: Mapping[str, Tuple[int, ...]], dtypes: Mapping[str, th.dtype], device, *,
                     fraction: float = 0.5, max_capacity: Optional[int] = None) -> "DeviceBuffer":
        """A ring whose capacity is :func:`hbm_capacity` of one sample's bytes."""
        per = sum(int(np.prod(s)) * th.empty((), dtype=dtypes[k]).element_size() for k, s in sample_shapes.items())
        cap = hbm_capacity(per, fraction=fraction, device=device)
        if max_capacity is not None:
            cap = min(cap, max_capacity)
        return cls(cap, sample_shapes, dtypes, device)

    def __init__(self, capacity: int, sample_shapes: Mapping[str, Tuple[int, ...]], dtypes: Mapping[str, th.dtype], device):
        self.capacity = capacity
        self.device = th.device(device)
        self.sample_shapes = {k: tuple(s) for k, s in sample_shapes.items()}
        self._arrays = {k: th.zeros((capacity,) + s, dtype=dtypes[k], device=self.device) for k, s in self.sample_shapes.items()}
        self._n_data = 0
        self._idx = 0

    def store(self, data: Mapping[str, th.Tensor]) -> None:
        n = next(iter(data.values())).shape[0]
        if n == 0:
            return
        if n > self.capacity:
            data = {k: v[-self.capacity :] for k, v in data.items()}
            n = self.capacity
        first = min(n, self.capacity - self._idx)
        for k, v in data.items():
            v = v.to(self.device, self._arrays[k].dtype)
            self._arrays[k][self._idx : self._idx + first] = v[:first]
            if first < n:
                self._arrays[k][: n - first] = v[first:]
        self._idx = (self._idx + n) % self.capacity
        self._n_data = min(self._n_data + n, self.capacity)

    def sample(self, n_samples: int, generator: Optional[th.Generator] = None) -> Dict[str, th.Tensor]:
        if self._n_data == 0:
            raise ValueError("Buffer is empty")
        from imitation_amd.ops.rl import gather_rows

        ind = th.randint(0, self._n_data, (n_samples,), device=self.device, generator=generator)
        keys = list(self._arrays)
        out: Dict[str, th.Tensor] = {}
        for s in range(0, len(keys), 8):  # <= 8 fields per gather launch
            ks = keys[s : s + 8]
            out.update(zip(ks, gather_rows([self._arrays[k] for k in ks], ind)))
        return out

    def size(self) -> int:
        return self._n_data

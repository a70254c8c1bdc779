"""Seeding, deterministic mode and RNG-state capture (SURVEY §5 "determinism / resume").

The reference seeds through ``util.make_vec_env(rng=...)`` and SB3's ``set_random_seed``
(``src/imitation/util/util.py:68-160``) and never captures RNG state. For exact
resume every generator that feeds training is captured here as plain tensors /
ints, so a checkpoint stays loadable with ``torch.load(weights_only=True)``.

Determinism of the HIP path: every hand-written reduction in ``csrc/kernels`` sums in
a fixed block order (no float atomics), so with :func:`set_deterministic` a rerun of
the device engine is bitwise reproducible on the same GPU and world size.
"""

from __future__ import annotations

import os
import random
from typing import Any, Dict, Optional

import numpy as np
import torch as th


def seed_everything(seed: int, rank: Optional[int] = None) -> int:
    """Seed python, numpy and torch (CPU + all GPUs); distinct per DP rank if given."""
    s = int(seed) + (0 if rank is None else 1_000_003 * int(rank))
    s &= 0xFFFFFFFF
    random.seed(s)
    np.random.seed(s)
    th.manual_seed(s)
    if th.cuda.is_available():
        th.cuda.manual_seed_all(s)
    return s


def set_deterministic(flag: bool = True) -> None:
    """Deterministic library kernels (rocBLAS/hipBLASLt atomics off, MIOpen deterministic)."""
    th.use_deterministic_algorithms(flag, warn_only=True)
    th.backends.cudnn.deterministic = flag
    th.backends.cudnn.benchmark = not flag
    if flag:
        os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
        os.environ.setdefault("ROCBLAS_DEFAULT_ATOMICS_MODE", "0")


def _np_state_to_tensors(st) -> Dict[str, Any]:
    name, keys, pos, has_gauss, cached = st
    return {"name": name, "keys": th.as_tensor(np.asarray(keys, dtype=np.int64)), "pos": int(pos),
            "has_gauss": int(has_gauss), "cached": float(cached)}


def _np_state_from_tensors(d: Dict[str, Any]):
    return (d["name"], d["keys"].numpy().astype(np.uint32), d["pos"], d["has_gauss"], d["cached"])


def generator_state(gen: np.random.Generator) -> Dict[str, Any]:
    """State of a ``numpy.random.Generator`` as JSON-able / tensor-only data."""
    st = gen.bit_generator.state
    return _jsonable(st)


def set_generator_state(gen: np.random.Generator, state: Dict[str, Any]) -> None:
    gen.bit_generator.state = _from_jsonable(state)


def _jsonable(x):
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, np.ndarray):
        return {"__ndarray__": th.as_tensor(x.astype(np.int64) if x.dtype.kind == "u" else x), "dtype": str(x.dtype)}
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, int) and x >= 2**63:
        return {"__bigint__": str(x)}
    return x


def _from_jsonable(x):
    if isinstance(x, dict):
        if "__ndarray__" in x:
            return x["__ndarray__"].numpy().astype(x["dtype"])
        if "__bigint__" in x:
            return int(x["__bigint__"])
        return {k: _from_jsonable(v) for k, v in x.items()}
    return x


def capture_rng_state() -> Dict[str, Any]:
    """Global RNG state of python / numpy / torch CPU / every visible GPU."""
    st: Dict[str, Any] = {
        "python": _jsonable({"state": list(random.getstate()[1]), "version": random.getstate()[0],
                             "gauss": random.getstate()[2]}),
        "numpy": _np_state_to_tensors(np.random.get_state()),
        "torch": th.get_rng_state(),
    }
    if th.cuda.is_available():
        st["cuda"] = [s for s in th.cuda.get_rng_state_all()]
    return st


def restore_rng_state(st: Dict[str, Any]) -> None:
    py = st["python"]
    random.setstate((py["version"], tuple(py["state"]), py["gauss"]))
    np.random.set_state(_np_state_from_tensors(st["numpy"]))
    th.set_rng_state(st["torch"])
    if "cuda" in st and th.cuda.is_available():
        cur = th.cuda.device_count()
        states = list(st["cuda"])[:cur]
        for i, s in enumerate(states):
            th.cuda.set_rng_state(s, i)

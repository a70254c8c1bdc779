"""``model.zip`` archive I/O (SB3 layout).

Archive members: ``data`` (JSON of algorithm attributes), ``policy.pth``
(state dict), ``policy.optimizer.pth``, ``pytorch_variables.pth``,
``_stable_baselines3_version``, ``system_info.txt``.

Reading: our own archives round-trip exactly. Archives written by SB3 store
spaces and classes as base64 *cloudpickle* blobs; those blobs are never
unpickled here (untrusted-code rule). Instead the plain JSON side fields SB3
writes next to each blob (``_shape``, ``dtype``, ``low_repr``/``high_repr``, ``n``)
are parsed, and ``policy.pth`` is loaded with ``torch.load(weights_only=True)``
-- enough to rebuild an SB3 ``ActorCriticPolicy`` expert by state-dict key.
"""

from __future__ import annotations

import importlib
import io
import json
import os
import pathlib
import platform
import re
import zipfile
from typing import Any, Dict, Optional, Tuple, Union

import numpy as np
import torch as th

from imitation_amd.envs import spaces

FORMAT_VERSION = "imitation_amd-2.4"


def _space_to_json(space: spaces.Space) -> Dict[str, Any]:
    if isinstance(space, spaces.Box):
        return {"__space__": "Box", "low": np.asarray(space.low).tolist(), "high": np.asarray(space.high).tolist(),
                "shape": list(space.shape), "dtype": str(np.dtype(space.dtype))}
    if isinstance(space, spaces.Discrete):
        return {"__space__": "Discrete", "n": int(space.n), "start": int(getattr(space, "start", 0))}
    if isinstance(space, spaces.MultiDiscrete):
        return {"__space__": "MultiDiscrete", "nvec": np.asarray(space.nvec).tolist()}
    if isinstance(space, spaces.MultiBinary):
        return {"__space__": "MultiBinary", "n": list(space.shape)}
    if isinstance(space, spaces.Dict):
        return {"__space__": "Dict", "spaces": {k: _space_to_json(v) for k, v in space.spaces.items()}}
    raise TypeError(f"cannot serialize space {space}")


def _space_from_json(d: Dict[str, Any]) -> spaces.Space:
    kind = d["__space__"]
    if kind == "Box":
        dt = np.dtype(d["dtype"])
        low = np.asarray(d["low"], dtype=dt)
        high = np.asarray(d["high"], dtype=dt)
        return spaces.Box(low, high, tuple(d["shape"]), dt)
    if kind == "Discrete":
        return spaces.Discrete(d["n"], start=d.get("start", 0))
    if kind == "MultiDiscrete":
        return spaces.MultiDiscrete(d["nvec"])
    if kind == "MultiBinary":
        return spaces.MultiBinary(d["n"] if len(d["n"]) > 1 else d["n"][0])
    if kind == "Dict":
        return spaces.Dict({k: _space_from_json(v) for k, v in d["spaces"].items()})
    raise ValueError(kind)


def _parse_np_repr(s: str, dtype) -> np.ndarray:
    body = s.strip().strip("[]").replace("\n", " ")
    vals = [float(x) for x in re.split(r"[\s,]+", body) if x]
    return np.asarray(vals, dtype=dtype)


def _space_from_sb3_json(d: Dict[str, Any]) -> Optional[spaces.Space]:
    """Rebuild a space from the plain-JSON side fields of an SB3 archive (no unpickling)."""
    t = d.get(":type:", "")
    if "Box" in t:
        shape = tuple(json.loads(d["_shape"])) if isinstance(d["_shape"], str) else tuple(d["_shape"])
        dt = np.dtype(d.get("dtype", "float32"))
        low = _parse_np_repr(d.get("low_repr", d.get("low")), np.float64)
        high = _parse_np_repr(d.get("high_repr", d.get("high")), np.float64)
        if low.size == 1:
            low = np.full(shape, low.item())
            high = np.full(shape, high.item())
        low = low.reshape(shape)
        high = high.reshape(shape)
        return spaces.Box(low.astype(dt), high.astype(dt), shape, dt)
    if "MultiDiscrete" in t:
        return spaces.MultiDiscrete(_parse_np_repr(d["nvec"], np.int64))
    if "Discrete" in t:
        return spaces.Discrete(int(d["n"]), start=int(d.get("start", 0)))
    return None


def _encode(v: Any) -> Any:
    if isinstance(v, spaces.Space):
        return _space_to_json(v)
    if isinstance(v, type):
        return {"__class__": f"{v.__module__}:{v.__qualname__}"}
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    if isinstance(v, np.ndarray):
        return {"__ndarray__": v.tolist(), "dtype": str(v.dtype)}
    if isinstance(v, dict):
        return {str(k): _encode(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_encode(x) for x in v]
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    return {"__unserializable__": repr(v)[:200]}


def _resolve_class(path: str):
    mod, _, qual = path.partition(":")
    # Only classes importable from installed modules are resolved (no pickle).
    obj = importlib.import_module(mod)
    for part in qual.split("."):
        obj = getattr(obj, part)
    return obj


def _decode(v: Any) -> Any:
    if isinstance(v, dict):
        if "__space__" in v:
            return _space_from_json(v)
        if "__class__" in v:
            try:
                return _resolve_class(v["__class__"])
            except Exception:
                return None
        if "__ndarray__" in v:
            return np.asarray(v["__ndarray__"], dtype=v["dtype"])
        if "__unserializable__" in v:
            return None
        if ":type:" in v or ":serialized:" in v:
            return _space_from_sb3_json(v)
        return {k: _decode(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_decode(x) for x in v]
    return v


def save_to_zip_file(path, data: Dict[str, Any], params: Dict[str, Dict[str, Any]], pytorch_variables: Optional[Dict[str, Any]] = None) -> None:
    path = pathlib.Path(path)
    if path.suffix != ".zip":
        path = path.with_suffix(".zip")
    path.parent.mkdir(parents=True, exist_ok=True)
    with zipfile.ZipFile(path, mode="w") as archive:
        archive.writestr("data", json.dumps({k: _encode(v) for k, v in data.items()}, indent=2))
        for name, state in params.items():
            buf = io.BytesIO()
            th.save(state, buf)
            archive.writestr(name + ".pth", buf.getvalue())
        if pytorch_variables is not None:
            buf = io.BytesIO()
            th.save(pytorch_variables, buf)
            archive.writestr("pytorch_variables.pth", buf.getvalue())
        archive.writestr("_stable_baselines3_version", FORMAT_VERSION)
        archive.writestr(
            "system_info.txt",
            f"- OS: {platform.platform()}\n- Python: {platform.python_version()}\n- PyTorch: {th.__version__}\n"
            f"- Framework: imitation_amd (MI355X / gfx950)\n",
        )


def load_from_zip_file(path, device: Union[str, th.device] = "cpu") -> Tuple[Dict[str, Any], Dict[str, Any], Optional[Dict[str, Any]]]:
    """Returns ``(data, params, pytorch_variables)``; tensors via ``weights_only=True`` only."""
    path = pathlib.Path(path)
    if not path.exists() and path.with_suffix(".zip").exists():
        path = path.with_suffix(".zip")
    with zipfile.ZipFile(path) as archive:
        names = archive.namelist()
        data = {}
        if "data" in names:
            raw = json.loads(archive.read("data").decode())
            data = {k: _decode(v) for k, v in raw.items()}
        params = {}
        pvars = None
        for n in names:
            if not n.endswith(".pth"):
                continue
            buf = io.BytesIO(archive.read(n))
            try:
                obj = th.load(buf, map_location=device, weights_only=True)
            except Exception:
                obj = None  # refuses non-tensor payloads (e.g. pickled optimizer param groups from SB3)
            if n == "pytorch_variables.pth":
                pvars = obj
            elif obj is not None:
                params[n[: -len(".pth")]] = obj
    return data, params, pvars

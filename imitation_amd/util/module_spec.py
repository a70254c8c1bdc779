"""Pickle-free module checkpoints: record constructor calls, rebuild, load state dict.

The reference serialises reward nets and policies with ``torch.save(module)``
(pickle; ``scripts/train_adversarial.py:save``, ``rewards/serialize.py``). Here a
module class that mixes in :class:`SpecRecorded` remembers the arguments of its
outermost constructor call; :func:`save_module` writes that call tree as JSON next
to the state dict in a tensor-only file, and :func:`load_module` rebuilds it with
``torch.load(weights_only=True)``. Constructor arguments may be spaces, classes,
importable functions, other recorded modules, and JSON-able values.
"""

from __future__ import annotations

import functools
import importlib
import inspect
import json
from typing import Any, Dict

import numpy as np
import torch as th
from torch import nn

FORMAT = "imitation_amd.module.v1"
_ALLOWED_PREFIXES = ("imitation_amd.", "torch.nn", "torch.optim", "torch:")


class SpecRecorded:
    """Mixin: wraps every subclass ``__init__`` to record the outermost call's arguments."""

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        init = cls.__dict__.get("__init__")
        if init is None or getattr(init, "_spec_wrapped", False):
            return
        sig = inspect.signature(init)

        @functools.wraps(init)
        def wrapped(self, *args, **kw):
            if "_ctor_spec" not in self.__dict__:
                try:
                    bound = sig.bind(self, *args, **kw)
                    params = dict(bound.arguments)
                    params.pop(next(iter(sig.parameters)))  # self
                    for name, p in sig.parameters.items():
                        if p.kind is inspect.Parameter.VAR_KEYWORD and name in params:
                            params.update(params.pop(name))
                        elif p.kind is inspect.Parameter.VAR_POSITIONAL and name in params:
                            if params.pop(name):
                                params = None
                                break
                except TypeError:
                    params = None
                object.__setattr__(self, "_ctor_spec", (type(self), params))
            init(self, *args, **kw)

        wrapped._spec_wrapped = True  # type: ignore[attr-defined]
        cls.__init__ = wrapped  # type: ignore[misc]


def _path(obj) -> str:
    return f"{obj.__module__}:{obj.__qualname__}"


def _resolve(path: str):
    if not path.startswith(_ALLOWED_PREFIXES):
        raise ValueError(f"refusing to import {path!r} while loading a module checkpoint")
    mod, _, qual = path.partition(":")
    obj = importlib.import_module(mod)
    for part in qual.split("."):
        obj = getattr(obj, part)
    return obj


def encode(v: Any) -> Any:
    from imitation_amd.envs import spaces
    from imitation_amd.rl import save_util

    if isinstance(v, nn.Module):
        return {"__module__": module_spec(v)}
    if isinstance(v, spaces.Space):
        return save_util._encode(v)
    if isinstance(v, type) or inspect.isfunction(v) or isinstance(v, functools.partial) is False and inspect.isbuiltin(v):
        return {"__ref__": _path(v)}
    if isinstance(v, functools.partial):
        return {"__partial__": encode(v.func), "args": encode(list(v.args)), "kwargs": encode(dict(v.keywords))}
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, np.ndarray):
        return {"__ndarray__": v.tolist(), "dtype": str(v.dtype)}
    if isinstance(v, dict):
        return {"__dict__": [[encode(k), encode(x)] for k, x in v.items()]}
    if isinstance(v, tuple):
        return {"__tuple__": [encode(x) for x in v]}
    if isinstance(v, list):
        return [encode(x) for x in v]
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    raise TypeError(f"cannot serialise constructor argument of type {type(v).__name__}")


def decode(v: Any) -> Any:
    from imitation_amd.rl import save_util

    if isinstance(v, list):
        return [decode(x) for x in v]
    if not isinstance(v, dict):
        return v
    if "__module__" in v:
        return build_module(v["__module__"])
    if "__ref__" in v:
        return _resolve(v["__ref__"])
    if "__partial__" in v:
        return functools.partial(decode(v["__partial__"]), *decode(v["args"]), **decode(v["kwargs"]))
    if "__ndarray__" in v:
        return np.asarray(v["__ndarray__"], dtype=v["dtype"])
    if "__dict__" in v:
        return {decode(k): decode(x) for k, x in v["__dict__"]}
    if "__tuple__" in v:
        return tuple(decode(x) for x in v["__tuple__"])
    if "__space__" in v:
        return save_util._decode(v)
    return {k: decode(x) for k, x in v.items()}


def module_spec(m: nn.Module) -> Dict[str, Any]:
    spec = m.__dict__.get("_ctor_spec")
    if spec is None or spec[1] is None:
        raise TypeError(f"{type(m).__name__} was not built through a recorded constructor; cannot serialise it")
    cls, params = spec
    return {"class": _path(cls), "kwargs": {k: encode(x) for k, x in params.items()}}


def build_module(spec: Dict[str, Any]) -> nn.Module:
    cls = _resolve(spec["class"])
    return cls(**{k: decode(x) for k, x in spec["kwargs"].items()})


def save_module(m: nn.Module, path) -> None:
    th.save({"format": FORMAT, "spec": json.dumps(module_spec(m)), "state_dict": m.state_dict()}, str(path))


def load_module(path, map_location=None) -> nn.Module:
    saved = th.load(str(path), map_location=map_location, weights_only=True)
    if not isinstance(saved, dict) or saved.get("format") != FORMAT:
        raise ValueError(f"{path} is not a module checkpoint written by imitation_amd")
    m = build_module(json.loads(saved["spec"]))
    m.load_state_dict(saved["state_dict"])
    if map_location is not None:
        m.to(map_location)
    return m

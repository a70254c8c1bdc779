"""Registry of lazily-loaded objects (reference: src/imitation/util/registry.py).

Keys map either to a value or to an ``"module.path:attr"`` string imported on first
use, so optional dependencies are only touched when selected.
"""

from __future__ import annotations

import importlib
from typing import Callable, Dict, Generic, Iterable, Optional, TypeVar

T = TypeVar("T")
LoaderFn = Callable[..., T]


def load_attr(name: str):
    """Import ``"path.to.module:attribute"``."""
    module_name, attr_name = name.split(":")
    return getattr(importlib.import_module(module_name), attr_name)


class Registry(Generic[T]):
    def __init__(self):
        self._values: Dict[str, T] = {}
        self._indirect: Dict[str, str] = {}

    def get(self, key: str) -> T:
        if key in self._values:
            return self._values[key]
        if key in self._indirect:
            self._values[key] = load_attr(self._indirect[key])
            return self._values[key]
        raise KeyError(f"Key '{key}' is not registered.")

    def keys(self) -> Iterable[str]:
        return set(self._values).union(self._indirect)

    def register(self, key: str, *, value: Optional[T] = None, indirect: Optional[str] = None) -> None:
        if key in self._values or key in self._indirect:
            raise KeyError(f"Duplicate registration for '{key}'")
        if (value is None) == (indirect is None):
            raise ValueError("Must provide exactly one of 'value' and 'indirect'.")
        if value is not None:
            self._values[key] = value
        else:
            self._indirect[key] = indirect


def build_loader_fn_require_space(fn: Callable, **kwargs) -> LoaderFn:
    """Adapt ``fn(observation_space, action_space)`` to a ``loader(venv)`` signature."""

    def f(venv, *args, **kw):
        del args, kw
        return fn(venv.observation_space, venv.action_space, **kwargs)

    return f


def build_loader_fn_require_env(fn: Callable, **kwargs) -> LoaderFn:
    """Adapt ``fn(venv)`` to a loader ignoring extra positional arguments."""

    def f(venv, *args, **kw):
        del args, kw
        return fn(venv, **kwargs)

    return f

"""Loader for the native extension ``imitation_amd._C``.

Policy: the extension is *required*. On a machine with a GPU every device op
dispatches to a HIP kernel from ``_C`` and raises if the extension is missing
(no silent eager fallback). CPU tensors use the PyTorch reference
implementations in :mod:`imitation_amd.ops` (those are the numerics oracles the
kernel tests compare against).
"""

from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None


def load(build_if_missing: bool = True):
    """Import (building in-tree first if needed) and return the ``_C`` module."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        import torch  # noqa: F401  (loads libc10/libtorch/libamdhip64 first)

        from imitation_amd import _build

        want_build = build_if_missing and os.environ.get("IMITATION_AMD_NO_BUILD", "0") != "1"
        if want_build and _build.is_stale():
            _build.build()
        try:
            _mod = importlib.import_module("imitation_amd._C")
        except ImportError as e:  # pragma: no cover - exercised only when the build is absent
            raise ImportError(
                "imitation_amd._C is not built. Run `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `python -m imitation_amd._build`."
            ) from e
        return _mod


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False

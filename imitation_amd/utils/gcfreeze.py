"""Keep Python's cyclic garbage collector off the heap that existed before a training loop.

After ``import torch`` the interpreter tracks ~170K container objects (module dicts, functions,
classes). A full (generation-2) collection walks all of them: ~100 ms on one core. A training
loop that keeps many small Python objects alive (trajectories, preference fragments, log
records) triggers such collections every few iterations, and each one stalls the host for as
long as a DRLHP reward-model epoch (``profiles/r5_drlhp.md`` call Z: one 95-118 ms pause every
~4 iterations, inside whichever phase happened to allocate).

:func:`frozen_heap` moves every object tracked at entry into the interpreter's permanent
generation (``gc.freeze``) and back out at exit (``gc.unfreeze``). Objects created inside are
collected as usual; objects from before are not scanned while it is active, and cyclic garbage
among them is collected after it ends. Nested uses freeze and unfreeze once, at the outermost
level. ``IMITATION_AMD_GC_FREEZE=0`` turns it into a no-op.
"""

from __future__ import annotations

import contextlib
import gc
import os
import threading
from typing import Iterator

_lock = threading.Lock()
_depth = 0


@contextlib.contextmanager
def frozen_heap() -> Iterator[None]:
    global _depth
    if os.environ.get("IMITATION_AMD_GC_FREEZE", "1") == "0":
        yield
        return
    with _lock:
        if _depth == 0:
            gc.freeze()
        _depth += 1
    try:
        yield
    finally:
        with _lock:
            _depth -= 1
            if _depth == 0:
                gc.unfreeze()


def during(fn):
    """Method / function decorator: the call runs inside :func:`frozen_heap`."""
    import functools

    @functools.wraps(fn)
    def wrapped(*args, **kwargs):
        with frozen_heap():
            return fn(*args, **kwargs)

    return wrapped

"""Tracing and throughput accounting (SURVEY §5 "tracing / profiling").

The reference has no tracing beyond SB3/HumanCompatibleAI logger timings
(``src/imitation/util/logger.py:28-120`` accumulates means; nothing marks phases).
Here every training phase can be bracketed by a ROCTX range, so a
``rocprofv3 --marker-trace --kernel-trace`` run shows rollout / reward inference /
PPO / discriminator / collective phases on the timeline next to the kernels they
launched, and :class:`StepTimer` turns wall time into env-steps/s per rank and
for the whole node (one all-reduce, only when a report is requested).

``ranges`` are off unless ``IMITATION_AMD_ROCTX=1`` (or :func:`enable_roctx`) so a
production run pays one ``if`` per phase.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Dict, Iterator, Optional

import torch as th

_ROCTX_CANDIDATES = (
    "librocprofiler-sdk-roctx.so.1",  # rocprofv3 --marker-trace listens on this one
    "librocprofiler-sdk-roctx.so",
    "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
    "libroctx64.so.4",
    "/opt/rocm/lib/libroctx64.so.4",
)

_lib = None
_enabled = os.environ.get("IMITATION_AMD_ROCTX", "0") == "1"


def _load_roctx():
    global _lib
    if _lib is not None:
        return _lib or None
    for name in _ROCTX_CANDIDATES:
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            return lib
        except (OSError, AttributeError):
            continue
    _lib = False
    return None


def roctx_available() -> bool:
    return _load_roctx() is not None


def enable_roctx(flag: bool = True) -> None:
    """Turn ROCTX phase ranges on/off for this process."""
    global _enabled
    _enabled = bool(flag)


def roctx_enabled() -> bool:
    return _enabled and roctx_available()


def mark(name: str) -> None:
    """Instant marker on the ROCTX timeline."""
    if _enabled:
        lib = _load_roctx()
        if lib is not None:
            lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name: str) -> Iterator[None]:  # noqa: A001 - mirrors roctx naming
    """ROCTX push/pop range around a phase (no-op when disabled)."""
    lib = _load_roctx() if _enabled else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def traced(name: str):
    """Decorator: run the function inside ``range(name)`` when ROCTX ranges are on (disabled:
    one flag test per call). The device engines mark their phases with it -- rollout chain,
    reward pass, PPO update, discriminator updates, replay store, collectives, host logging --
    so a ``rocprofv3 --marker-trace`` timeline attributes the host gaps to phases."""
    import functools

    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            if not _enabled:
                return fn(*args, **kwargs)
            lib = _load_roctx()
            if lib is None:
                return fn(*args, **kwargs)
            lib.roctxRangePushA(name.encode())
            try:
                return fn(*args, **kwargs)
            finally:
                lib.roctxRangePop()

        return wrapper

    return deco


class StepTimer:
    """Per-phase wall clock + env-step throughput, per rank and whole node.

    ``sync=True`` calls ``torch.cuda.synchronize`` at phase boundaries so phase times
    are device times (use for diagnosis; the bench only syncs at its brackets).

    >>> t = StepTimer()
    >>> with t.phase("rollout"):
    ...     pass
    >>> t.add_env_steps(4096)
    """

    def __init__(self, sync: bool = False, roctx: bool = True):
        self.sync = sync and th.cuda.is_available()
        self.roctx = roctx
        self.phase_s: Dict[str, float] = {}
        self.phase_n: Dict[str, int] = {}
        self.env_steps = 0
        self._t0 = time.perf_counter()

    def reset(self) -> None:
        self.phase_s.clear()
        self.phase_n.clear()
        self.env_steps = 0
        self._t0 = time.perf_counter()

    @contextlib.contextmanager
    def phase(self, name: str) -> Iterator[None]:
        if self.sync:
            th.cuda.synchronize()
        t = time.perf_counter()
        cm = range(name) if self.roctx else contextlib.nullcontext()
        with cm:
            yield
            if self.sync:
                th.cuda.synchronize()
        self.phase_s[name] = self.phase_s.get(name, 0.0) + time.perf_counter() - t
        self.phase_n[name] = self.phase_n.get(name, 0) + 1

    def add_env_steps(self, n: int) -> None:
        self.env_steps += int(n)

    def elapsed(self) -> float:
        return time.perf_counter() - self._t0

    def report(self, all_ranks: bool = True) -> Dict[str, float]:
        """Throughput summary. With ``all_ranks`` (and an initialised process group) the
        whole-node figure sums env steps over ranks and divides by the slowest rank's time."""
        from imitation_amd.parallel import dist as pdist

        el = max(self.elapsed(), 1e-12)
        out = {"rank_env_steps_per_s": self.env_steps / el, "elapsed_s": el, "env_steps": float(self.env_steps)}
        for k, v in self.phase_s.items():
            out[f"phase_s/{k}"] = v
            out[f"phase_frac/{k}"] = v / el
        if all_ranks and pdist.world_size() > 1:
            tot = pdist.allreduce_scalars([float(self.env_steps)], op="sum")[0]
            slow = pdist.allreduce_scalars([el], op="max")[0]
            out["node_env_steps_per_s"] = tot / slow
            out["world_size"] = float(pdist.world_size())
        else:
            out["node_env_steps_per_s"] = out["rank_env_steps_per_s"]
            out["world_size"] = 1.0
        return out

    def log_to(self, logger, prefix: str = "perf/") -> Dict[str, float]:
        rep = self.report()
        for k, v in rep.items():
            logger.record(prefix + k, v)
        return rep


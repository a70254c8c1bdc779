"""Failure detection: hang watchdog and NaN/Inf fail-fast (SURVEY §5 "failure detection").

The reference relies on Ray Tune retries and SLURM timeouts
(``src/imitation/scripts/parallel.py:1-290``, ``benchmarking/run_benchmark_on_slurm.sh``)
and has no in-process detection. A production multi-GPU job needs to fail fast:

* :class:`Watchdog` -- a heartbeat thread. If the training loop does not call
  :meth:`Watchdog.beat` within ``timeout_s`` (a stuck collective, a wedged kernel),
  every thread's Python stack is dumped to stderr and the process exits with
  ``exit_code`` so the launcher (torchrun) tears the job down and a restart can
  resume from the last checkpoint. Collective timeouts themselves are set at
  ``parallel.dist.init(timeout_s=...)``.
* :func:`check_finite` / :func:`assert_finite_module` -- raise :class:`NonFiniteError`
  naming the first offending tensor. Checks are batched into one device->host copy.
"""

from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Iterable, Mapping, Optional, Union

import torch as th


class NonFiniteError(FloatingPointError):
    """A loss, gradient or parameter became NaN/Inf."""


def _items(tensors) -> Iterable:
    if isinstance(tensors, th.Tensor):
        return [("tensor", tensors)]
    if isinstance(tensors, Mapping):
        return list(tensors.items())
    return [(str(i), t) for i, t in enumerate(tensors)]


def check_finite(tensors: Union[th.Tensor, Mapping[str, th.Tensor], Iterable[th.Tensor]], where: str = "") -> None:
    """Raise :class:`NonFiniteError` if any tensor holds NaN/Inf (one host sync in total)."""
    items = [(k, t) for k, t in _items(tensors) if isinstance(t, th.Tensor) and t.is_floating_point() and t.numel()]
    if not items:
        return
    flags = th.stack([th.isfinite(t.detach()).all() for _, t in items])
    ok = flags.cpu()
    if bool(ok.all()):
        return
    bad = [k for (k, _), f in zip(items, ok.tolist()) if not f]
    raise NonFiniteError(f"non-finite values{' in ' + where if where else ''}: {', '.join(bad)}")


def assert_finite_module(module: th.nn.Module, where: str = "", grads: bool = True) -> None:
    """Fail fast if any parameter (and, with ``grads``, any gradient) of ``module`` is non-finite."""
    ts = {}
    for n, p in module.named_parameters():
        ts[n] = p
        if grads and p.grad is not None:
            ts[n + ".grad"] = p.grad
    check_finite(ts, where or type(module).__name__)


class Watchdog:
    """Abort the process if :meth:`beat` is not called for ``timeout_s`` seconds.

    >>> with Watchdog(timeout_s=600) as wd:
    ...     for r in range(rounds):
    ...         trainer.train(step)
    ...         wd.beat()
    """

    def __init__(self, timeout_s: float, exit_code: int = 124, name: str = "imitation_amd", on_timeout=None,
                 poll_s: Optional[float] = None):
        if timeout_s <= 0:
            raise ValueError("timeout_s must be positive")
        self.timeout_s = float(timeout_s)
        self.exit_code = exit_code
        self.name = name
        self.on_timeout = on_timeout
        self.poll_s = poll_s if poll_s is not None else min(1.0, self.timeout_s / 4)
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.fired = False

    def beat(self) -> None:
        self._last = time.monotonic()

    def start(self) -> "Watchdog":
        self._last = time.monotonic()
        self._stop.clear()
        self._thread = threading.Thread(target=self._run, name=f"{self.name}-watchdog", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    def __enter__(self) -> "Watchdog":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            idle = time.monotonic() - self._last
            if idle > self.timeout_s:
                self.fired = True
                rank = os.environ.get("RANK", "0")
                sys.stderr.write(f"[{self.name} watchdog] rank {rank}: no heartbeat for {idle:.1f}s "
                                 f"(> {self.timeout_s:.1f}s); dumping stacks and aborting\n")
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                sys.stderr.flush()
                if self.on_timeout is not None:
                    self.on_timeout()
                    return
                os._exit(self.exit_code)


def cli_watchdog(name: str):
    """The CLIs' hang watchdog (``IMITATION_AMD_WATCHDOG_S`` seconds without a per-round beat,
    default 1800; 0 disables): a context manager yielding an object with ``beat()``."""
    import contextlib

    s = float(os.environ.get("IMITATION_AMD_WATCHDOG_S", "1800"))
    if s <= 0:
        class _Null:
            def beat(self) -> None:
                pass

        return contextlib.nullcontext(_Null())
    return Watchdog(timeout_s=s, name=name)


def rl_beat_callback(wd):
    """An RL ``BaseCallback`` beating ``wd`` at every rollout end (``train_rl`` / SQIL ``learn``)."""
    from imitation_amd.rl.callbacks import BaseCallback

    class _Beat(BaseCallback):
        def _on_step(self) -> bool:
            return True

        def _on_rollout_end(self) -> None:
            wd.beat()

    return _Beat()

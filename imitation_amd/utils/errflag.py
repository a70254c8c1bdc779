"""Host-visible error word of a device kernel (fail-fast).

The cooperating-workgroup PPO kernel (``csrc/kernels/ppo_rc.hip``) bounds every spin on a
partner workgroup; a spin that gives up ORs 1 into this word. The word persists across launches
(unlike the kernel's per-launch sync words), so a check after any later launch still sees it.

Checks are non-blocking by default, like ``OneShotComm.check``: a stream-ordered copy into
pinned memory is enqueued and the copy enqueued by the PREVIOUS check is read if it has landed,
so a per-round check never serialises pipelined rounds. ``blocking=True`` reads now (end of a
training call). Reference behaviour mirrored: broken invariants raise
(``src/imitation/algorithms/base.py:77-110``).
"""

from __future__ import annotations

import contextlib
from typing import Optional

import torch as th


class DeviceErrorFlag:
    """One int32 device word + its async host mirror."""

    def __init__(self, device: th.device, what: str):
        self.device = th.device(device)
        self.what = what
        self.word = th.zeros(1, dtype=th.int32, device=self.device)
        self._host: Optional[th.Tensor] = None
        self._ev: Optional[th.cuda.Event] = None

    def clear(self) -> None:
        self.word.zero_()

    def check(self, where: str = "", blocking: bool = False, stream: Optional[th.cuda.Stream] = None) -> None:
        """``stream``: enqueue the copy there (already ordered after the kernels that set the
        word) instead of on the current stream."""
        if blocking:
            err = int(self.word.item())
        else:
            err = 0
            if self._ev is not None and self._ev.query():
                err = int(self._host[0])
            if self._host is None:
                self._host = th.zeros(1, dtype=th.int32, pin_memory=True)
            if self._ev is None or self._ev.query():  # one copy in flight at a time
                with th.cuda.device(self.device), (th.cuda.stream(stream) if stream is not None
                                                   else contextlib.nullcontext()):
                    self._host.copy_(self.word, non_blocking=True)
                    self._ev = th.cuda.Event()
                    self._ev.record()
        if err:
            self.clear()
            self._ev = None
            raise RuntimeError(f"{self.what} timed out waiting for a cooperating workgroup"
                               f"{(' (' + where + ')') if where else ''}: the update used partial gradients; "
                               "aborting the run (a partner workgroup was not co-resident or stalled)")

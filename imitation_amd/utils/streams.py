"""Process-wide side streams, one per (device, role).

HIP maps every new stream onto one of the device's ``GPU_MAX_HW_QUEUES`` (4) hardware queues in
creation order. An engine that creates its side streams per instance therefore lands them on
different hardware queues in successive instances of one process; in round 6 every second GAIL
trainer instance had its discriminator side stream on the hardware queue of the main stream, so
the 8 discriminator updates (~0.7 ms) no longer ran under the PPO kernel and ``hipLaunchKernel``
took 22.7 instead of 7.8 us (2.74 -> 3.4-3.5 ms per round, ``profiles/r6_bench_quality.md``).
Creating each role's stream once per process keeps the first instance's mapping for all of them.
Sharing a stream between two live trainers only adds ordering between their side work; each
trainer still orders its own work with events.
"""

from __future__ import annotations

import threading
from typing import Dict, Tuple

import torch as th

_lock = threading.Lock()
_streams: Dict[Tuple[int, str], "th.cuda.Stream"] = {}


def shared_stream(device, role: str) -> "th.cuda.Stream":
    """The process-wide side stream of ``role`` on ``device`` (created on first use)."""
    dev = th.device(device)
    idx = dev.index if dev.index is not None else th.cuda.current_device()
    key = (idx, role)
    with _lock:
        s = _streams.get(key)
        if s is None:
            s = _streams[key] = th.cuda.Stream(device=th.device("cuda", idx))
        return s

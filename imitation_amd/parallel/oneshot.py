"""One-shot all-reduce for small data-parallel buckets (kernel: ``csrc/kernels/comm.hip``).

The DP runtime reduces KB-sized buckets several times per round (discriminator gradients,
normaliser moment sums; reference hook points ``algorithms/adversarial/common.py:371-372``,
``util/networks.py:80-134``).  RCCL's ring all-reduce pays 2(W-1) hops of xGMI latency per
message; here every rank maps every peer's staging region through a ``hipIpc`` handle
(exchanged once over the process group), and ONE kernel stages, signals, waits and sums in
rank order -- one xGMI hop, no host involvement, graph-capture safe (the generation counter
lives on the device), bitwise identical on every rank.

Selection (``IMITATION_AMD_ONESHOT``):

* ``auto`` (default) -- on when the backend is RCCL, every rank has its own GPU on this node
  (``LOCAL_WORLD_SIZE == WORLD_SIZE``) and the start-up self-test passes;
* ``1`` -- also on under gloo with ranks sharing one GPU (the one-card rehearsal path);
* ``0`` -- off (every collective goes to torch.distributed).

Buckets larger than ``IMITATION_AMD_ONESHOT_MAX_BYTES`` (default 1 MiB) keep RCCL, whose
pipelined ring wins once the message is bandwidth bound.
"""

from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as tdist

_COMM: Optional["OneShotComm"] = None
_TRIED = False


class OneShotComm:
    """IPC-mapped staging regions of all ranks + the one-shot all-reduce launch."""

    def __init__(self, native, rank: int, world: int, device: torch.device, stage_bytes: int, timeout_s: float):
        if world > 8:
            raise ValueError("one-shot all-reduce supports up to 8 ranks")
        self._C = native
        self.rank, self.world, self.device = rank, world, device
        self.stage_bytes = int(stage_bytes)
        self.timeout_s = float(timeout_s)
        self.bases: List[int] = []
        self._opened: List[int] = []
        self.local = None
        handle = None
        try:
            with torch.cuda.device(device):
                self.local, handle = native.oneshot_alloc(self.stage_bytes)
        except Exception:
            handle = None
        handles = [None] * world
        tdist.all_gather_object(handles, handle)  # every rank learns whether every rank allocated
        if any(h is None for h in handles):
            self.close()
            raise RuntimeError("one-shot all-reduce: staging allocation failed on some rank")
        opened = True
        try:
            with torch.cuda.device(device):
                for r, h in enumerate(handles):
                    if r == rank:
                        self.bases.append(self.local)
                    else:
                        p = native.oneshot_open(h)
                        self._opened.append(p)
                        self.bases.append(p)
        except Exception:
            opened = False
        if not _agree(opened, device):
            self.close()
            raise RuntimeError("one-shot all-reduce: IPC mapping failed on some rank")
        self.calls = 0

    def fits(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.device == self.device and t.dtype in (torch.float32, torch.float64) and t.is_contiguous()
                and t.numel() * t.element_size() <= self.stage_bytes and t.data_ptr() % 16 == 0)

    def allreduce_(self, t: torch.Tensor, scale: float = 1.0) -> None:
        """``t <- sum_r scale * t_r`` in place (rank-order sum, identical on all ranks)."""
        flat = t.view(-1)
        self._C.oneshot_allreduce(self.bases, self.rank, flat, flat, float(scale), self.stage_bytes, self.timeout_s)
        self.calls += 1

    def error(self) -> int:
        return int(self._C.oneshot_error(self.local))

    def clear_error(self) -> None:
        self._C.oneshot_clear_error(self.local)

    def check(self, where: str = "", blocking: bool = False) -> None:
        """Raise if a bounded wait of this communicator timed out (a lost or stalled peer:
        the kernel wrote NaN into that reduction's output). Called once per round / epoch by
        the training loops, so a lost peer stops the run instead of training on NaN.

        Non-blocking by default: a stream-ordered copy of the error word into pinned memory
        is enqueued, and the copy enqueued by the PREVIOUS check is read if it has landed
        (a synchronous read would wait for every stream -- including a next round the loop
        has already enqueued -- and serialise the pipelined rounds). ``blocking``: read now."""
        if blocking:
            err = self.error()
        else:
            err = 0
            ev = getattr(self, "_err_ev", None)
            if ev is not None and ev.query():
                err = int(self._err_host[0])
            if not hasattr(self, "_err_host"):
                self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            if ev is None or ev.query():  # one copy in flight at a time
                with torch.cuda.device(self.device):
                    self._C.oneshot_error_async(self.local, self._err_host)
                    self._err_ev = torch.cuda.Event()
                    self._err_ev.record()
        if err:
            self.clear_error()
            raise RuntimeError(f"one-shot all-reduce timed out waiting for a peer{(' (' + where + ')') if where else ''}: "
                               "its output was poisoned with NaN; aborting the run")

    def block_floats(self) -> int:
        """Floats per block slice (a bucket of n floats runs ceil(n / block_floats) blocks)."""
        return 4 * max(256, -(-(self.stage_bytes // 16) // 64))

    def blocks(self, n: int) -> int:
        return int(self._C.oneshot_blocks(int(n), self.stage_bytes))

    def self_test(self) -> bool:
        return self.self_test_report()[0]

    def self_test_report(self):
        """Start-up check before any gradient goes through this communicator: ``(ok, reason)``,
        agreed over ranks (every rank returns the same verdict).

        1. closed form: rank-dependent buckets (odd sizes, both staging parities) against
           ``sum_r``, with the device error word clear;
        2. cross-check against the process group (RCCL): the same rank-distinct buckets reduced
           by ``torch.distributed.all_reduce``. Exactly representable values (small integers +
           halves) make every summation order exact, so the two must be BITWISE equal; a second,
           non-dyadic bucket must agree to rounding (a wrong row / rank mapping shows as O(1)
           differences).
        The bounded waits use a 5 s timeout here, so a broken peer mapping fails fast (the kernel
        then poisons its output and sets the error word)."""
        reasons = []
        saved, self.timeout_s = self.timeout_s, min(self.timeout_s, 5.0)
        # Every rank issues every process-group collective below whatever happened before it (each
        # step has its own try): a rank whose one-shot call raised must not skip to the verdict's
        # MIN all-reduce while the others issue the RCCL cross-check -- mismatched collectives hang
        # or pair wrongly. (One-shot calls only wait on peers, boundedly.)
        w = self.world
        try:
            for n in (1, 5, 1027, min(self.stage_bytes // 4, 16384 + 3)):
                for rep in range(2):
                    try:
                        x = torch.arange(n, dtype=torch.float32, device=self.device) * (self.rank + 1) + rep
                        self.allreduce_(x)
                        exp = torch.arange(n, dtype=torch.float32, device=self.device) * (w * (w + 1) / 2) + rep * w
                        if not bool(torch.allclose(x, exp, rtol=1e-6, atol=1e-3)) and not reasons:
                            reasons.append(f"closed-form mismatch at n={n}")
                    except Exception as e:  # noqa: BLE001 -- any failure disables the path
                        reasons.append(f"closed form n={n} raised {e!r}")
            n = min(self.stage_bytes // 4, 4099)
            g = torch.Generator().manual_seed(1234 + self.rank)
            exact = (torch.randint(-512, 512, (n,), generator=g).float() + 0.5 * (self.rank % 2)).to(self.device)
            fuzzy = torch.randn(n, generator=g).to(self.device)
            for name, t in (("exact", exact), ("fuzzy", fuzzy)):
                mine = None
                try:
                    mine = t.clone()
                    self.allreduce_(mine)
                except Exception as e:  # noqa: BLE001
                    reasons.append(f"{name} one-shot call raised {e!r}")
                    mine = None
                ref = self._reference_allreduce(t)  # (issued on every rank)
                if mine is None:
                    continue
                if name == "exact" and not torch.equal(mine, ref):
                    reasons.append("not bitwise equal to the process-group all-reduce on exactly representable data")
                if name == "fuzzy" and not bool(torch.allclose(mine, ref, rtol=1e-5, atol=1e-5 * w)):
                    reasons.append("differs from the process-group all-reduce beyond rounding")
        finally:
            self.timeout_s = saved
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        try:
            if self.error() != 0:
                reasons.append("a bounded peer wait timed out (error word set)")
        except Exception as e:  # noqa: BLE001
            reasons.append(f"error word unreadable: {e!r}")
        ok = _agree(not reasons, self.device)
        if not ok and not reasons:
            reasons.append("failed on another rank")
        return ok, "; ".join(reasons)

    def _reference_allreduce(self, t: torch.Tensor) -> torch.Tensor:
        ref = t.clone() if tdist.get_backend() == "nccl" else t.detach().cpu().clone()
        tdist.all_reduce(ref)
        return ref.to(self.device)

    def close(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        for p in self._opened:
            self._C.oneshot_close(p)
        self._opened = []
        if self.local is not None:
            self._C.oneshot_free(self.local)
            self.local = None


def _agree(ok: bool, device: torch.device) -> bool:
    """Logical AND of ``ok`` over ranks (one tiny collective)."""
    flag = torch.tensor([1.0 if ok else 0.0])
    if tdist.get_backend() == "nccl":
        flag = flag.to(device)
    tdist.all_reduce(flag, op=tdist.ReduceOp.MIN)
    return bool(flag.item() > 0.5)


def _mode() -> str:
    return os.environ.get("IMITATION_AMD_ONESHOT", "auto").strip().lower()


def get() -> Optional[OneShotComm]:
    """The process-wide communicator, created (and self-tested) on first use; None when the
    one-shot path is off or unavailable. Every rank must call this at the same point (the
    first call is collective)."""
    global _COMM, _TRIED
    if _TRIED:
        return _COMM
    _TRIED = True
    mode = _mode()
    if mode in ("0", "off", "false") or not (tdist.is_available() and tdist.is_initialized()):
        return None
    world = tdist.get_world_size()
    if world <= 1 or world > 8 or not torch.cuda.is_available():
        return None
    backend = tdist.get_backend()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if mode == "auto" and (backend != "nccl" or local_world != world):
        return None
    from imitation_amd import _native

    C = _native.load()
    dev = torch.device("cuda", torch.cuda.current_device())
    stage = int(os.environ.get("IMITATION_AMD_ONESHOT_MAX_BYTES", str(1024 * 1024)))
    stage = max(16, (stage + 15) // 16 * 16)
    timeout = float(os.environ.get("IMITATION_AMD_ONESHOT_TIMEOUT_S", "600"))  # = the process-group timeout
    # every pair of distinct devices must be peer-accessible (xGMI); ranks on one card
    # (the rehearsal path) share the device and need no peer mapping
    devs = [None] * world
    tdist.all_gather_object(devs, dev.index)
    try:
        peer_ok = all(d == dev.index or torch.cuda.can_device_access_peer(dev.index, d) for d in devs)
    except Exception:  # a local query: never skip the agreement collective below
        peer_ok = False
    if not _agree(peer_ok, dev):
        if mode not in ("auto",):
            raise RuntimeError("one-shot all-reduce: devices are not peer-accessible")
        return None
    comm = None
    try:
        comm = OneShotComm(C, tdist.get_rank(), world, dev, stage, timeout)
    except Exception as e:  # IPC unavailable on this node: keep torch.distributed
        if mode not in ("auto",):
            raise
        _disable(f"set-up failed: {e!r}")
        return None
    _COMM = adopt(comm, mode)
    return _COMM


DISABLED_REASON: Optional[str] = None


def _disable(reason: str) -> None:
    global DISABLED_REASON
    DISABLED_REASON = reason
    import logging

    logging.getLogger(__name__).warning("one-shot all-reduce disabled, using torch.distributed: %s", reason)


def adopt(comm, mode: str = "auto"):
    """Run ``comm``'s start-up self-test (:meth:`OneShotComm.self_test_report`); the communicator
    if it passed, else close it and return None with the reason logged and kept in
    :data:`DISABLED_REASON` (``mode`` other than ``auto``: raise instead)."""
    ok, reason = comm.self_test_report()
    if ok:
        return comm
    comm.close()
    if mode not in ("auto",):
        raise RuntimeError(f"one-shot all-reduce self-test failed: {reason}")
    _disable(f"self-test failed: {reason}")
    return None


def reset() -> None:
    """Drop the communicator (process-group teardown)."""
    global _COMM, _TRIED
    if _COMM is not None:
        try:
            _COMM.close()
        except Exception:
            pass
    _COMM = None
    _TRIED = False

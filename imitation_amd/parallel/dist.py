"""Data-parallel runtime: one process per GPU, RCCL over xGMI.

The reference has no distributed code at all. This module
adds the collectives the MI355X build needs, at the hook points listed there:

* :func:`init` -- ``torch.distributed`` process group from the torchrun env
  (``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_*``); backend ``"nccl"`` is RCCL
  on ROCm, ``"gloo"`` for CPU tests.
* :class:`GradBucket` -- every gradient of a module flattened into ONE contiguous
  fp32 bucket and all-reduced with a single collective per optimizer step. The
  models here are KB-sized, so the collective is latency bound; one message per
  step is the whole game on a point-to-point xGMI mesh.
* :func:`allreduce_moments` -- normaliser statistics (count, sum, sum of squares)
  reduced in one message so RunningNorm/EMANorm replicas stay identical.
* :func:`all_gather_rows` -- variable-length row all-gather (trajectories,
  preference fragments): counts first, then one padded ``all_gather_into_tensor``.
* :func:`broadcast_module` -- initial parameters/buffers from rank 0.
* :func:`allreduce_scalars` -- eval statistics.
* small fp32 buckets (gradients, moment sums; <= 1 MiB) go through the one-shot
  IPC all-reduce kernel of :mod:`imitation_amd.parallel.oneshot` when it is available
  (one xGMI hop instead of RCCL's 2(W-1)-hop ring), everything else through RCCL.
"""

from __future__ import annotations

import contextlib
import datetime
import os
from typing import Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as tdist

_NORM_SYNC = True


def _traced(name):
    from imitation_amd.utils import profiling

    return profiling.traced(name)


def is_initialized() -> bool:
    return tdist.is_available() and tdist.is_initialized()


def world_size() -> int:
    return tdist.get_world_size() if is_initialized() else 1


def rank() -> int:
    return tdist.get_rank() if is_initialized() else 0


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def is_main() -> bool:
    return rank() == 0


def init(backend: Optional[str] = None, timeout_s: float = 600.0) -> Tuple[int, int]:
    """Initialise the default process group from torchrun env vars (idempotent).

    Returns ``(rank, world_size)``. With ``WORLD_SIZE`` unset or 1 nothing is
    initialised and ``(0, 1)`` is returned.
    """
    if is_initialized():
        return rank(), world_size()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return 0, 1
    if backend is None:
        # IMITATION_AMD_DIST_BACKEND=gloo lets several ranks share one GPU (rehearsal of the
        # multi-GPU path on a single card; RCCL refuses two ranks on one device)
        backend = os.environ.get("IMITATION_AMD_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local_rank())
    kwargs = {}
    if backend == "nccl":
        kwargs["device_id"] = torch.device("cuda", local_rank())
    tdist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kwargs)
    from imitation_amd.parallel import oneshot

    oneshot.get()  # collective set-up of the small-bucket path at a point every rank reaches
    return rank(), world_size()


def shutdown() -> None:
    if is_initialized():
        from imitation_amd.parallel import oneshot

        oneshot.reset()
        tdist.destroy_process_group()


def _oneshot_for(t: torch.Tensor):
    """The one-shot communicator if it can reduce ``t`` (fp32 or fp64, contiguous, on this GPU, small)."""
    from imitation_amd.parallel import oneshot

    c = oneshot._COMM
    return c if c is not None and c.fits(t) else None


def barrier() -> None:
    if is_initialized():
        if tdist.get_backend() == "nccl":
            tdist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            tdist.barrier()


def norm_sync_active() -> bool:
    return _NORM_SYNC and world_size() > 1


@contextlib.contextmanager
def no_norm_sync():
    """Disable normaliser all-reduce (e.g. for rank-local evaluation)."""
    global _NORM_SYNC
    old = _NORM_SYNC
    _NORM_SYNC = False
    try:
        yield
    finally:
        _NORM_SYNC = old


def _comm_device(t: torch.Tensor) -> torch.Tensor:
    if is_initialized() and tdist.get_backend() == "nccl" and not t.is_cuda:
        return t.cuda()
    if is_initialized() and tdist.get_backend() == "gloo" and t.is_cuda:
        return t.cpu()
    return t


@_traced("comm/allreduce_moments")
def allreduce_moments(batch: torch.Tensor):
    """Global (mean, biased var, count) of ``batch`` rows across all ranks, one message."""
    b = batch.reshape(batch.shape[0], -1).double()
    n = torch.tensor([float(b.shape[0])], dtype=torch.float64, device=b.device)
    msg = torch.cat([n, b.sum(0), (b * b).sum(0)])
    m = _comm_device(msg)
    tdist.all_reduce(m)
    msg = m.to(b.device)
    f = b.shape[1]
    count = msg[0]
    mean = msg[1 : 1 + f] / count
    var = (msg[1 + f :] / count - mean * mean).clamp_min(0.0)
    shape = batch.shape[1:]
    return mean.to(batch.dtype).reshape(shape), var.to(batch.dtype).reshape(shape), int(count.item())


def allreduce_moments_device(batch: torch.Tensor):
    """Capture-safe variant of :func:`allreduce_moments` on the one-shot path: every rank
    puts its (count, mean, centred M2) in its own row of a zero ``[world, 2F + 1]`` fp32
    message, one sum all-reduce hands every rank all rows exactly (adding zeros is exact),
    and the rows are Chan-merged on the device in rank order -- no host sync, the count
    comes back as an int32 device tensor. None when the one-shot path cannot take it."""
    if world_size() <= 1 or not batch.is_cuda:
        return None
    from imitation_amd.parallel import oneshot

    c = oneshot._COMM
    b = batch.reshape(batch.shape[0], -1).float()
    f = b.shape[1]
    if c is None or world_size() * (2 * f + 1) * 4 > c.stage_bytes or b.device != c.device:
        return None
    mean_r = b.mean(0)
    m2_r = (b - mean_r).square().sum(0)
    msg = torch.zeros(world_size(), 2 * f + 1, dtype=torch.float32, device=b.device)
    # device-side fills / copies only (a Python-scalar setitem is a host->device copy,
    # which a capturing stream refuses)
    msg[rank()].copy_(torch.cat([b.new_full((1,), float(b.shape[0])), mean_r, m2_r]))
    c.allreduce_(msg)
    n_r = msg[:, :1]
    n = n_r.sum()
    mean = (n_r * msg[:, 1 : 1 + f]).sum(0) / n
    m2 = msg[:, 1 + f :].sum(0) + (n_r * (msg[:, 1 : 1 + f] - mean).square()).sum(0)
    shape = batch.shape[1:]
    return (mean.to(batch.dtype).reshape(shape), (m2 / n).to(batch.dtype).reshape(shape),
            n.round().to(torch.int32))


def oneshot_active() -> bool:
    """True when small fp32 collectives run on the (graph-capturable) one-shot kernel."""
    from imitation_amd.parallel import oneshot

    return world_size() > 1 and oneshot._COMM is not None


def check_comm(where: str = "", blocking: bool = False) -> None:
    """Raise if a one-shot reduction timed out on a lost / stalled peer (its output was
    poisoned with NaN). Once per round / epoch / iteration: non-blocking (a stream-ordered
    4-byte copy, read one check later -- see ``OneShotComm.check``); ``blocking`` at the end
    of a training call."""
    if world_size() <= 1:
        return
    from imitation_amd.parallel import oneshot

    c = oneshot._COMM
    if c is not None:
        c.check(where, blocking=blocking)


def allreduce_scalars(values: Sequence[float], op: str = "sum", device=None) -> List[float]:
    if not is_initialized():
        return list(values)
    dev = device or (torch.device("cuda") if tdist.get_backend() == "nccl" else torch.device("cpu"))
    t = torch.tensor(list(values), dtype=torch.float64, device=dev)
    tdist.all_reduce(t, op={"sum": tdist.ReduceOp.SUM, "max": tdist.ReduceOp.MAX, "min": tdist.ReduceOp.MIN}[op])
    return t.tolist()


class GradBucket:
    """Flat, persistent gradient bucket for a fixed parameter list.

    ``param.grad`` of every parameter is re-pointed at a view into one contiguous
    buffer, so backward writes straight into the bucket and :meth:`allreduce`
    is exactly one collective (no pack/unpack copies). The mean over ranks is
    formed by pre-scaling with 1/world (``ReduceOp.AVG`` is not available on
    every backend).
    """

    def __init__(self, params: Iterable[torch.nn.Parameter]):
        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            self.flat = None
            return
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self._views = []
        off = 0
        for p in self.params:
            v = self.flat[off : off + p.numel()].view_as(p)
            self._views.append(v)
            off += p.numel()
        self.bind()

    def bind(self) -> None:
        """(Re-)attach the bucket views as ``.grad`` (after ``zero_grad(set_to_none)``)."""
        if self.flat is None:
            return
        for p, v in zip(self.params, self._views):
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                if p.grad is not None:
                    v.copy_(p.grad)
                p.grad = v

    def zero(self) -> None:
        if self.flat is not None:
            self.flat.zero_()
            self.bind()

    def allreduce(self) -> None:
        if self.flat is None or world_size() <= 1:
            return
        self.bind()
        c = _oneshot_for(self.flat)
        if c is not None:
            c.allreduce_(self.flat, 1.0 / world_size())
            return
        self.flat.mul_(1.0 / world_size())
        buf = _comm_device(self.flat)
        tdist.all_reduce(buf)
        if buf is not self.flat:
            self.flat.copy_(buf)


class FlatGradBucket:
    """DP bucket over an optimizer that already keeps its gradients in flat buffers
    (:class:`imitation_amd.ops.optim.FusedAdam`): one mean all-reduce per buffer, no
    re-pointing of ``.grad``."""

    def __init__(self, optimizer):
        self.optimizer = optimizer

    def bind(self) -> None:
        for f in getattr(self.optimizer, "_flat", []):
            if f["n"]:
                self.optimizer._bind_grads(f)

    def zero(self) -> None:
        self.optimizer.zero_grad()

    def allreduce(self) -> None:
        if world_size() <= 1:
            return
        self.bind()
        for flat in self.optimizer.flat_grads:
            allreduce_grads_flat(flat)


def allreduce_grads(params: Iterable[torch.nn.Parameter]) -> None:
    """One-shot mean all-reduce of ``.grad`` over ranks (pack -> 1 collective -> unpack)."""
    if world_size() <= 1:
        return
    ps = [p for p in params if p.grad is not None]
    if not ps:
        return
    flat = torch.cat([p.grad.reshape(-1) for p in ps]).mul_(1.0 / world_size())
    buf = _comm_device(flat)
    tdist.all_reduce(buf)
    if buf is not flat:
        flat = buf.to(flat.device)
    off = 0
    for p in ps:
        n = p.grad.numel()
        p.grad.copy_(flat[off : off + n].view_as(p.grad))
        off += n


@_traced("comm/allreduce_sum")
def allreduce_sum_(t: torch.Tensor) -> None:
    """Sum all-reduce of ``t`` in place (one collective; no-op on one rank)."""
    if world_size() <= 1:
        return
    c = _oneshot_for(t)
    if c is not None:
        c.allreduce_(t)
        return
    buf = _comm_device(t)
    tdist.all_reduce(buf)
    if buf is not t:
        t.copy_(buf)


@_traced("comm/allreduce_grads")
def allreduce_grads_flat(flat: torch.Tensor) -> None:
    """Mean all-reduce of one flat gradient vector in place (one collective)."""
    if world_size() <= 1:
        return
    c = _oneshot_for(flat)
    if c is not None:
        c.allreduce_(flat, 1.0 / world_size())
        return
    flat.mul_(1.0 / world_size())
    buf = _comm_device(flat)
    tdist.all_reduce(buf)
    if buf is not flat:
        flat.copy_(buf)


def broadcast_module(module: torch.nn.Module, src: int = 0) -> None:
    """Broadcast all parameters and buffers from ``src`` (one flat message per dtype)."""
    if world_size() <= 1:
        return
    tensors = [t for t in list(module.parameters()) + list(module.buffers())]
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault(t.dtype, []).append(t)
    for dtype, ts in by_dtype.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        buf = _comm_device(flat)
        tdist.broadcast(buf, src=src)
        flat = buf.to(ts[0].device)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off : off + n].view_as(t))
                off += n


def all_gather_rows(x: torch.Tensor) -> torch.Tensor:
    """Concatenate ``x`` (``[n_r, ...]``, n_r may differ per rank) over ranks in rank order."""
    if world_size() <= 1:
        return x
    dev_x = _comm_device(x.contiguous())
    n = torch.tensor([dev_x.shape[0]], dtype=torch.int64, device=dev_x.device)
    counts = [torch.zeros_like(n) for _ in range(world_size())]
    tdist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    cap = max(counts)
    pad = torch.zeros((cap,) + tuple(dev_x.shape[1:]), dtype=dev_x.dtype, device=dev_x.device)
    pad[: dev_x.shape[0]] = dev_x
    out = torch.empty((world_size() * cap,) + tuple(dev_x.shape[1:]), dtype=dev_x.dtype, device=dev_x.device)
    if tdist.get_backend() == "nccl":
        tdist.all_gather_into_tensor(out, pad)
    else:
        chunks = list(out.chunk(world_size()))
        tdist.all_gather(chunks, pad)
    parts = [out[r * cap : r * cap + counts[r]] for r in range(world_size())]
    return torch.cat(parts).to(x.device)


@_traced("comm/all_gather")
def all_gather_flat(out: torch.Tensor, x: torch.Tensor) -> None:
    """Equal-size all-gather of ``x`` into ``out`` (``[world * n, ...]``, rank order), one collective."""
    if world_size() <= 1:
        out.copy_(x.reshape(out.shape))
        return
    if tdist.get_backend() == "nccl":
        tdist.all_gather_into_tensor(out, x.contiguous())
        return
    xc = _comm_device(x.contiguous())
    parts = [torch.empty_like(xc) for _ in range(world_size())]
    tdist.all_gather(parts, xc)
    out.copy_(torch.cat(parts).to(out.device).reshape(out.shape))


def all_gather_object(obj) -> list:
    if world_size() <= 1:
        return [obj]
    out = [None] * world_size()
    tdist.all_gather_object(out, obj)
    return out


def broadcast_object(obj, src: int = 0):
    if world_size() <= 1:
        return obj
    lst = [obj]
    tdist.broadcast_object_list(lst, src=src)
    return lst[0]

"""HIP-graph capture of launch-bound training steps.

A minibatch step of the small networks this framework trains (BC on NatureCNN / MLP
policies, reward models) is ~100 tiny kernels whose launch cost on the host exceeds their
GPU time. :class:`GraphedTrainStep` captures ``fn(*inputs)`` -- forward, ``backward()``
and ``optimizer.step()`` -- ONCE per input signature as a HIP graph over static input
buffers; later steps copy the new inputs into those buffers and replay the graph.

Semantics are those of the eager step ``zero_grad(set_to_none=True); fn(...)``:

* the first step of every signature runs eagerly on a side stream (PyTorch's required
  warm-up), and that run IS the step -- nothing is executed twice;
* the optimiser is switched to ``capturable`` mode (its step counters move to the device);
* gradients are written into the graph's private pool by every replay (the captured
  backward starts from ``grad=None``), so no ``zero_grad`` is needed between replays.

Only valid when ``fn`` has no host synchronisation and fixed shapes per signature (the
callers check this: one fixed minibatch size, no DP gradient bucket).
"""

from __future__ import annotations

import contextlib
import gc
import os
import threading
from typing import Any, Callable, Dict, Optional, Tuple

import torch as th


# Held for the whole of every capture: worker threads that make HIP calls (event queries /
# synchronisations, their own launches) take it around those calls, so that none lands inside
# a capture -- in the default (global) capture mode such a call from ANY thread invalidates it.
CAPTURE_LOCK = threading.RLock()


@contextlib.contextmanager
def capture(graph: "th.cuda.CUDAGraph", **kwargs):
    """``th.cuda.graph(graph, **kwargs)`` with Python's garbage collector held off for the
    capture: a collection inside it can run finalisers that free pinned host memory or
    destroy events (a synchronising call -- illegal while a stream is capturing), which
    aborts the process depending on when the collector happens to run. (No collection
    here: a full gc.collect() per capture costs ~100 ms on a large heap.) Holds
    :data:`CAPTURE_LOCK`."""
    enabled = gc.isenabled()
    gc.disable()
    try:
        with CAPTURE_LOCK, th.cuda.graph(graph, **kwargs):
            yield
    finally:
        if enabled:
            gc.enable()


def graphs_enabled(device: th.device, knob: str) -> bool:
    """Graph capture applies on GPU unless disabled with ``<knob>=0``."""
    return th.device(device).type == "cuda" and os.environ.get(knob, "1") != "0"


def make_capturable(optimizer: th.optim.Optimizer) -> None:
    """Switch an Adam-family optimiser to ``capturable`` mode (device step counters)."""
    for grp in optimizer.param_groups:
        if "capturable" in grp:
            grp["capturable"] = True
    for st in optimizer.state.values():
        step = st.get("step")
        if isinstance(step, th.Tensor) and not step.is_cuda:
            dev = next(t.device for t in st.values() if isinstance(t, th.Tensor) and t.is_cuda)
            st["step"] = step.to(dev, th.float32)


def supports_capture(optimizer: th.optim.Optimizer) -> bool:
    return all("capturable" in g for g in optimizer.param_groups)


class GraphedTrainStep:
    """``step(*inputs) -> outputs`` with ``fn`` captured as a HIP graph per input signature."""

    def __init__(self, fn: Callable[..., Any], optimizer: th.optim.Optimizer,
                 release: Optional[Callable[[], None]] = None):
        self.fn = fn
        self.optimizer = optimizer
        # drops references the caller's objects hold to an earlier autograd graph (e.g. the
        # policy's distribution object): such a graph keeps the parameters' AccumulateGrad
        # nodes alive with the stream they were created on, and a backward that meets them
        # inside the capture synchronises with that stream -- illegal during capture
        self.release = release
        self._graphs: Dict[Tuple, Tuple[Tuple[th.Tensor, ...], Any, Any]] = {}
        self.n_captures = 0
        self.n_replays = 0

    def __call__(self, *inputs: th.Tensor) -> Any:
        key = tuple((tuple(t.shape), t.dtype, t.device) for t in inputs)
        entry = self._graphs.get(key)
        if entry is not None:
            static, graph, out = entry
            for s, t in zip(static, inputs):
                if s.data_ptr() != t.data_ptr():  # persistent (``_ia_static``) inputs are read in place
                    s.copy_(t, non_blocking=True)
            graph.replay()
            self.n_replays += 1
            return out
        make_capturable(self.optimizer)
        if self.release is not None:
            self.release()
        # inputs flagged ``_ia_static`` (persistent producer buffers, e.g. the DAgger loader's
        # batch buffers) are captured in place: their replays need no input copy
        static = tuple(t if getattr(t, "_ia_static", False) else t.detach().clone() for t in inputs)
        side = th.cuda.Stream()
        side.wait_stream(th.cuda.current_stream())
        with th.cuda.stream(side):  # warm-up == this step
            self.optimizer.zero_grad(set_to_none=True)
            result = self.fn(*static)
            # on the warm-up stream: a fused optimiser's zero_grad launches ``grad.zero_()``
            # over the bucket, which must stay ordered behind the warm-up's backward + step
            self.optimizer.zero_grad(set_to_none=True)
        if self.release is not None:
            self.release()
        graph = th.cuda.CUDAGraph()
        # capture on the warm-up stream: the autograd nodes the warm-up created (e.g. the
        # parameters' AccumulateGrad) belong to that stream, and a capture on another stream
        # would make the engine synchronise with it inside the capture
        with capture(graph, stream=side):
            out = self.fn(*static)
        th.cuda.current_stream().wait_stream(side)
        self._graphs[key] = (static, graph, out)
        self.n_captures += 1
        return result

"""Run a function on ``world_size`` local ranks (gloo on CPU, or RCCL when asked) for tests.

Each rank gets ``RANK``/``WORLD_SIZE``/``MASTER_ADDR=127.0.0.1``/``MASTER_PORT`` and
an initialised process group; return values are collected in rank order.
"""

from __future__ import annotations

import os
import socket
import traceback
from typing import Any, Callable, List

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank: int, world_size: int, port: int, backend: str, fn: Callable, args: tuple, queue) -> None:
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world_size), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch

    torch.set_num_threads(1)
    from imitation_amd.parallel import dist as pdist

    try:
        pdist.init(backend=backend, timeout_s=120)
        out = fn(rank, world_size, *args)
        queue.put((rank, "ok", out))
    except Exception:  # pragma: no cover - surfaced in the parent
        queue.put((rank, "err", traceback.format_exc()))
    finally:
        pdist.shutdown()


def run_ranks(fn: Callable, world_size: int = 2, *args, backend: str = "gloo", timeout: float = 300.0) -> List[Any]:
    ctx = mp.get_context("spawn")
    queue = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world_size, port, backend, fn, args, queue)) for r in range(world_size)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world_size):
            rank, status, payload = queue.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{payload}")
            results[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [results[r] for r in range(world_size)]


def fake_gpu_trial(run_kwargs, observer_dir, run_name):
    """A stand-in trial for ``scripts.parallel.run_trials`` tests (``ex_name`` =
    ``"imitation_amd.testing.distributed:fake_gpu_trial"``): records the GPU slot its process was
    started with and its run interval, sleeps ``config_updates["sleep"]`` seconds."""
    import os
    import time

    t0 = time.time()
    time.sleep(float(run_kwargs.get("config_updates", {}).get("sleep", 0.2)))
    if run_kwargs.get("config_updates", {}).get("fail"):
        raise RuntimeError("trial failed on purpose")
    return {"result": {"imit_stats": {"monitor_return_mean": 1.0}, "hip": os.environ.get("HIP_VISIBLE_DEVICES"),
                       "pid": os.getpid(), "t0": t0, "t1": time.time()},
            "config_updates": run_kwargs.get("config_updates", {}), "named_configs": [], "status": "COMPLETED"}


def fake_objective_trial(run_kwargs, observer_dir, run_name):
    """A stand-in trial whose metric is a smooth function of ``config_updates`` (x in [0, 1],
    log-scale lr, a categorical ``arch``) plus seed noise: the TPE tests' objective."""
    import math

    cu = run_kwargs.get("config_updates", {})
    x, lr = float(cu.get("x", 0.5)), float(cu.get("lr", 1e-3))
    arch = {"small": -0.5, "medium": 0.0, "large": -0.2}[cu.get("arch", "medium")]
    seed = int(cu.get("seed", 0))
    noise = 0.01 * math.sin(seed * 12.9898)
    metric = -(x - 0.3) ** 2 - 0.1 * (math.log10(lr) + 3.0) ** 2 + arch + noise
    return {"result": {"imit_stats": {"monitor_return_mean": metric}}, "config_updates": cu, "named_configs": [],
            "status": "COMPLETED"}

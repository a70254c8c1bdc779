"""GPU-free multi-rank self-launch for the benchmark entry points (``bench.py``,
``benchmarking/bench_configs.py``).

``--gpus N`` without ``torchrun``: the launcher process counts the visible GPUs WITHOUT
initialising HIP (KFD sysfs topology filtered by ``*_VISIBLE_DEVICES``; a throwaway child
process if sysfs is unreadable), then starts N fresh rank processes (one per GPU, RCCL)
with the ``torch.distributed`` env contract (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
on 127.0.0.1) and waits for them. The launcher itself never touches the GPU, so nothing
is exec'd from a process that initialised HIP (the reference launches one job per seed and
GPU: ``benchmarking/run_benchmark_on_slurm.sh:2-24``).
"""

from __future__ import annotations

import glob
import os
import socket
import subprocess
import sys
import time
from typing import List, Optional, Sequence


def _visible_filter(n_phys: int) -> int:
    """Apply ROCR / HIP / CUDA ``*_VISIBLE_DEVICES`` to a physical GPU count."""
    n = n_phys
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        v = v.strip()
        if v == "":
            return 0
        ids = [x for x in v.split(",") if x.strip() != ""]
        n = min(n, len(ids))
    return n


def _count_sysfs() -> Optional[int]:
    """GPU agents in the KFD topology (nodes with SIMDs), or None if unreadable."""
    nodes = glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")
    if not nodes:
        return None
    n = 0
    try:
        for path in nodes:
            with open(path) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
                        break
    except (OSError, ValueError):
        return None
    return n


def _count_child() -> int:
    """torch.cuda.device_count() in a throwaway child (HIP initialised there, not here)."""
    try:
        out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                             capture_output=True, text=True, timeout=600)
        return int(out.stdout.strip().splitlines()[-1])
    except Exception:
        return 0


def count_gpus() -> int:
    """Visible GPUs, counted without initialising HIP in this process."""
    n = _count_sysfs()
    if n is None:
        return _count_child()
    return _visible_filter(n)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def hip_initialized() -> bool:
    """Whether this process already initialised the GPU runtime (then it must not spawn)."""
    th = sys.modules.get("torch")
    if th is None:
        return False
    try:
        return bool(th.cuda.is_initialized())
    except Exception:
        return False


def spawn_ranks(n: int, script: str, argv: Sequence[str], label: str = "launcher") -> int:
    """Start ``n`` rank processes of ``script argv`` and return the worst exit code (a rank
    that dies takes the others down: they would block in a collective).
    ``IMITATION_AMD_DIST_BACKEND=gloo`` rehearses the multi-rank path with every rank on one
    device (or on the CPU), so no GPU count is required then."""
    assert not hip_initialized(), f"{label}: the GPU runtime is initialised in the launcher; spawn before touching it"
    backend = os.environ.get("IMITATION_AMD_DIST_BACKEND", "nccl")
    if backend != "gloo":
        have = count_gpus()
        if have < n:
            print(f"{label}: --gpus {n} needs {n} visible GPUs, found {have} "
                  f"(set IMITATION_AMD_DIST_BACKEND=gloo to rehearse on fewer devices)", file=sys.stderr)
            return 2
    port = _free_port()
    procs: List[subprocess.Popen] = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script)] + list(argv), env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0:
                rc = rc or code
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc if rc >= 0 else 1

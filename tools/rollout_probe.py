"""Rollout step-chain timing of a bench recipe (RECIPE, default gail_halfcheetah): ms per T-step
chain launch of csrc/kernels/rollout.hip. (The per-phase cycle split in
profiles/r4_rollout_breakdown.md was taken once with clock64 stamps compiled into the chain; the
stamps cost ~10 % of the chain's time, so they are not kept in the kernel.)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch as th  # noqa: E402


def main():
    from imitation_amd import models

    b = models.build(os.environ.get("RECIPE", "gail_halfcheetah"), device=th.device("cuda"), seed=0)
    tr = b.trainer
    for _ in range(3):
        tr._launch_chain()
    th.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        tr._launch_chain()
    th.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"chain: T={tr.T} N={tr.N}: {1e3 * dt:.3f} ms per launch, {1e6 * dt / tr.T:.2f} us per step", flush=True)


if __name__ == "__main__":
    main()

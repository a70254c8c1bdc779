"""Per-phase cycle counters of the register-chained PPO kernel on the GAIL-HalfCheetah
bench config (8 envs x 512 steps, minibatch 64, 5 epochs), 1 GPU.

Prints cycles per minibatch for: chunk (forward + loss + backward chain + dW items),
exchange + |g|^2, clip + Adam, and per-wave forward / loss / backward-chain splits for
the actor (wave 0) and critic (wave 4). Also times the update with the counters off.
"""
import os
import sys
import time

import numpy as np
import torch as th

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from imitation_amd import models

    b = models.build("gail_halfcheetah", device="cuda", n_envs=8, engine="device", n_demo_timesteps=8192)
    tr = b.trainer
    print("path", tr._C.engine_ppo_path(tr._ppo_static), flush=True)
    tr._rollout()
    for _ in range(2):
        tr._ppo_update()
    th.cuda.synchronize()
    n = 5
    t0 = time.perf_counter()
    for _ in range(n):
        tr._ppo_update()
    th.cuda.synchronize()
    print(f"ppo update {1e3 * (time.perf_counter() - t0) / n:.3f} ms (no counters)", flush=True)
    t0 = time.perf_counter()
    for _ in range(n):
        tr._rollout()
    th.cuda.synchronize()
    print(f"rollout {1e3 * (time.perf_counter() - t0) / n:.3f} ms (unchanged kernel: box-speed reference)", flush=True)
    prof = th.zeros(20, dtype=th.int64, device="cuda")
    tr._ppo_static["prof"] = prof
    tr._ppo_update()
    th.cuda.synchronize()
    p = prof.cpu().numpy().astype(np.float64)
    K = tr._last_ppo_info[1]
    names = ["chunk(fwd+loss+bwd+dW)", "exchange+|g|^2", "clip+adam"]
    for i, nm in enumerate(names):
        print(f"{nm:>26s}: {p[i] / K:9.0f} cycles/minibatch", flush=True)
    print(f"wave 0: B1 wait {p[11] / K:.0f} dW items {p[12] / K:.0f}", flush=True)
    for w, base in (("actor", 3), ("critic", 7)):
        parts = ["rows/x", "forward", "loss", "bwd chain"]
        print(w, " ".join(f"{parts[i]}={p[base + i] / K:.0f}" for i in range(4)), flush=True)
    tr._ppo_static.pop("prof")


if __name__ == "__main__":
    main()

"""Why is bench.py's timed GAIL round slower when the expert was trained in the same process?

Round 6 call A: cold cache (expert trained in process) 3.475 ms / round, warm cache 2.771 ms.
This probe times the bench trainer (W=3 warm-up, K=20 rounds, one ``train()`` call, as bench.py)
in one process: fresh, after a 5M-step expert run, after ``gc.collect`` + ``empty_cache``, and
with the Python threads listed at each point.

    python tools/expert_inproc_probe.py [expert_steps]
"""

import gc
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch as th  # noqa: E402

from imitation_amd import models  # noqa: E402


def timed(tag, demos=None):
    b = models.build("gail_halfcheetah", device="cuda", env_id="HalfCheetah-v4", demonstrations=demos)
    tr = b.trainer
    spr = tr.gen_train_timesteps
    tr.train(3 * spr)
    th.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train(20 * spr)
    th.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / 20
    print(f"{tag}: {ms:.3f} ms/round; threads={[t.name for t in threading.enumerate()]}; "
          f"gc counts={gc.get_count()} tracked={len(gc.get_objects())}; "
          f"alloc={th.cuda.memory_allocated() / 2**20:.0f} MiB reserved={th.cuda.memory_reserved() / 2**20:.0f} MiB",
          flush=True)
    return tr


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
    t = timed("fresh")
    del t
    t = timed("fresh again")
    del t
    t0 = time.perf_counter()
    ex = models.build("gail_halfcheetah", device="cuda", seed=100, env_id="HalfCheetah-v4", debug_use_ground_truth=True)
    ex.trainer.train(steps)
    th.cuda.synchronize()
    print(f"expert {steps} steps: {time.perf_counter() - t0:.2f} s", flush=True)
    demos = ex.trainer.device_demonstrations(50_000, deterministic=False, seed=20_000)
    del ex
    t = timed("after expert (expert deleted)", demos)
    del t
    t = timed("after expert, second trainer", demos)
    del t
    gc.collect()
    th.cuda.empty_cache()
    t = timed("after gc.collect + empty_cache", demos)
    del t
    t = timed("random demos again")


if __name__ == "__main__":
    main()

"""Phase timing of one DRLHP (preference_walker2d recipe) iteration on the device agent:
agent training, trajectory sampling, fragmenting, preference gathering, reward training."""
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch as th  # noqa: E402


def main():
    from imitation_amd import models

    b = models.build("preference_walker2d", device=th.device("cuda"), seed=0)
    tr = b.trainer
    acc = defaultdict(float)
    calls = defaultdict(int)

    def timed(obj, name, label):
        fn = getattr(obj, name)

        def w(*a, **k):
            th.cuda.synchronize()
            t0 = time.perf_counter()
            prof = None
            if os.environ.get("PROBE_CPROFILE") == label and not calls[label]:
                import cProfile

                prof = cProfile.Profile()
                prof.enable()
            r = fn(*a, **k)
            th.cuda.synchronize()
            if prof is not None:
                import pstats

                prof.disable()
                pstats.Stats(prof).sort_stats("cumulative").print_stats(30)
            acc[label] += time.perf_counter() - t0
            calls[label] += 1
            return r

        setattr(obj, name, w)

    timed(tr.trajectory_generator, "train", "agent.train")
    timed(tr.trajectory_generator, "sample", "agent.sample")
    timed(tr.fragmenter, "__call__", "fragmenter") if False else None
    timed(tr.preference_gatherer, "__call__", "gatherer") if False else None
    timed(tr.reward_trainer, "train", "reward.train")
    it = tr.train_iter(b.extras["total_timesteps"], total_comparisons=5000)
    t0 = time.perf_counter()
    next(it)
    th.cuda.synchronize()
    print(f"warm-up iteration: {time.perf_counter() - t0:.2f} s " + " ".join(f"{k}={v:.3f}s/{calls[k]}" for k, v in acc.items()), flush=True)
    for i in range(2):
        acc.clear()
        calls.clear()
        t0 = time.perf_counter()
        next(it)
        th.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"iteration {i}: {dt:.3f} s ({b.env_steps_per_round / dt:.0f} env-steps/s) "
              + " ".join(f"{k}={v:.3f}s/{calls[k]}" for k, v in acc.items()), flush=True)
    ag = tr.trajectory_generator
    th.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        ag._rollout()
    th.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(5):
        ag._ppo_update()
    th.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"rollout {1e3 * (t1 - t0) / 5:.2f} ms, ppo update {1e3 * (t2 - t1) / 5:.2f} ms per {ag.T}x{ag.N} round", flush=True)


if __name__ == "__main__":
    main()

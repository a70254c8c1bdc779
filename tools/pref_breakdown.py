"""Where a DRLHP (preference comparisons) iteration's wall time goes: the bench_configs
``preference_walker2d`` iteration with per-phase wall clocks from patched methods (trajectory
sampling, fragmenting, preference gathering, dataset push, reward-model training, agent
training), after one warm-up iteration. Prints one JSON line.

Usage: python tools/pref_breakdown.py [--iters 3] [--comparisons 5000]"""
import argparse
import collections
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--comparisons", type=int, default=5000)
    args = p.parse_args()
    import torch as th

    from imitation_amd import models

    dev = th.device("cuda", 0)
    b = models.build("preference_walker2d", device=dev, seed=0)
    tr = b.trainer
    acc = collections.defaultdict(float)

    def timed(obj, name, key):
        orig = getattr(obj, name)

        def wrap(*a, **k):
            th.cuda.synchronize()
            t0 = time.perf_counter()
            out = orig(*a, **k)
            th.cuda.synchronize()
            acc[key] += time.perf_counter() - t0
            return out

        setattr(obj, name, wrap)

    timed(tr.trajectory_generator, "sample", "sample")
    timed(tr.trajectory_generator, "train", "agent_train")
    timed(tr.reward_trainer, "train", "reward_train")
    timed(tr.dataset, "push", "dataset_push")
    tr.fragmenter = _Timed(tr.fragmenter, acc, "fragment")
    tr.preference_gatherer = _Timed(tr.preference_gatherer, acc, "gather_prefs")
    import gc

    gc_t = {"start": 0.0}

    def gc_cb(phase, info):  # Python's cyclic collector pauses (generation 2 grows with the dataset)
        if phase == "start":
            gc_t["start"] = time.perf_counter()
        else:
            acc[f"gc_gen{info['generation']}"] += time.perf_counter() - gc_t["start"]
            acc[f"gc_gen{info['generation']}_n"] += 1e-3  # (reported x 1e3 / iters: collections per iter)

    gc.callbacks.append(gc_cb)
    it = tr.train_iter(b.extras["total_timesteps"], total_comparisons=args.comparisons)
    next(it)  # warm-up: the initial iteration
    th.cuda.synchronize()
    acc.clear()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        next(it)
    th.cuda.synchronize()
    wall = time.perf_counter() - t0
    out = dict(iters=args.iters, ms_per_iter=1e3 * wall / args.iters,
               env_steps_per_s=args.iters * b.env_steps_per_round / wall,
               phases_ms_per_iter={k: round(1e3 * v / args.iters, 2) for k, v in acc.items()})
    main = [v for k, v in out["phases_ms_per_iter"].items() if not (k.startswith("gc_") or k.endswith("_thread_cpu"))]
    out["phases_ms_per_iter"]["other"] = round(out["ms_per_iter"] - sum(main), 2)
    print(json.dumps(out), flush=True)


class _Timed:
    def __init__(self, fn, acc, key):
        self.fn, self.acc, self.key = fn, acc, key

    def __call__(self, *a, **k):
        import torch as th

        th.cuda.synchronize()
        t0, c0 = time.perf_counter(), time.thread_time()
        out = self.fn(*a, **k)
        th.cuda.synchronize()
        self.acc[self.key] += time.perf_counter() - t0
        self.acc[self.key + "_thread_cpu"] += time.thread_time() - c0  # (wall >> cpu: waiting, e.g. for the GIL)
        return out

    def __getattr__(self, name):
        return getattr(self.fn, name)


if __name__ == "__main__":
    main()

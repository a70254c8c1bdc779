"""Where a DAgger-Pong round's wall time goes: the bench_configs round
(``SimpleDAggerTrainer.train`` with >= 2048 env steps per round + one BC epoch over the
aggregate) with per-phase wall clocks (collect / demo save / BC) from patched methods, the
GPU-busy share from CUDA events, and a cProfile of the timed rounds (top cumulative entries).

``--reference-schedule``: the reference's ``SimpleDAggerTrainer.train`` defaults instead (>= 3 episodes
and >= 500 env steps per round, 4 BC epochs; ``bench_configs.py dagger_pong``).

Usage: python tools/dagger_breakdown.py [--rounds 4] [--warmup 1] [--profile] [--reference-schedule]"""
import argparse
import collections
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=4)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--round-steps", type=int, default=2048)
    p.add_argument("--profile", action="store_true")
    p.add_argument("--reference-schedule", action="store_true")
    args = p.parse_args()
    import torch as th

    from imitation_amd import models

    dev = th.device("cuda", 0)
    b = models.build("dagger_pong", device=dev, seed=0)
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

    # phases: the BC epoch, the round's collection (incl. the D2H of the frames), the demo save
    timed(tr.bc_trainer, "train", "bc_train")
    timed(tr, "_collect_round", "collect_round")  # device collection + frames to host + aggregate append
    timed(tr, "extend_and_update", "extend_and_update")  # aggregate + BC epoch
    if getattr(tr, "_device_collector", None) is not None:
        timed(tr._device_collector, "collect", "device_collect")

    def round_():
        if args.reference_schedule:
            tr.train(1, rollout_round_min_episodes=3, rollout_round_min_timesteps=500,
                     bc_train_kwargs=dict(n_epochs=tr.DEFAULT_N_EPOCHS, log_interval=10**9, progress_bar=False))
            return
        tr.train(args.round_steps, rollout_round_min_episodes=1, rollout_round_min_timesteps=args.round_steps,
                 bc_train_kwargs=dict(n_epochs=1, log_interval=10**9, progress_bar=False))

    for _ in range(args.warmup):
        round_()
    th.cuda.synchronize()
    acc.clear()
    if getattr(tr, "_device_collector", None) is not None:
        tr._device_collector.timing.clear()
    pr = cProfile.Profile() if args.profile else None
    t0 = time.perf_counter()
    n_steps = 0
    per_round = []
    for _ in range(args.rounds):
        t1 = time.perf_counter()
        if pr:
            pr.enable()
        round_()
        if pr:
            pr.disable()
        th.cuda.synchronize()
        per_round.append(dict(ms=1e3 * (time.perf_counter() - t1), steps=int(tr.last_train_timesteps_local),
                              aggregate=int(len(tr._device_agg)) if getattr(tr, "_device_collector", None) else None))
        n_steps += tr.last_train_timesteps_local
    wall = time.perf_counter() - t0
    t2 = time.perf_counter()
    tr.flush_demos()  # background demo-file writes still pending after the timed rounds
    acc["demo_flush_after"] = (time.perf_counter() - t2) * args.rounds
    out = dict(rounds=args.rounds, ms_per_round=1e3 * wall / args.rounds, env_steps_per_s=n_steps / wall,
               phases_ms_per_round={k: 1e3 * v / args.rounds for k, v in acc.items()}, per_round=per_round)
    col = getattr(tr, "_device_collector", None)
    if col is not None:
        out["collect_sections_ms_per_round"] = {k: round(1e3 * v / args.rounds, 2) for k, v in col.timing.items()}
    print(json.dumps(out), flush=True)
    if pr:
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
        print(s.getvalue())


if __name__ == "__main__":
    main()

#!/usr/bin/env python
"""Throughput + final-return harness for every BASELINE.json config (one JSON line each).

``bench.py`` is the driver's headline (GAIL HalfCheetah, 1/2/4/8 GPUs); this script
measures the other four configurations of BASELINE.json on the recipes of
``imitation_amd/models/recipes.py`` (same architectures / tuned hyper-parameters as the
reference configs; synthetic MuJoCo/Atari-shaped envs and demonstrations, random-init
weights -- there is no network and no MuJoCo):

=====================  ==================================================  =================
config                 one timed step                                      throughput unit
=====================  ==================================================  =================
bc_cartpole            ``BC.train(n_batches=50)`` (batch 32)               samples/s
gail_halfcheetah       one GAIL round (4096 env steps + PPO + 8 disc)      env-steps/s
airl_hopper            one AIRL round (8192 env steps + PPO + 16 disc)     env-steps/s
dagger_pong            one DAgger round (>= 2048 env steps + BC epochs)    env-steps/s
preference_walker2d    one DRLHP iteration (agent steps + pref. training)  env-steps/s
=====================  ==================================================  =================

Every config also reports ``final_eval_return`` (mean over ``--eval-episodes`` episodes
of the trained policy, outside the timed region). Usage::

    python benchmarking/bench_configs.py --configs all --steps 3 --warmup 1
    python benchmarking/bench_configs.py --configs airl_hopper --gpus 8   # DP, weak scaling (self-spawned ranks)
    torchrun --nproc-per-node 8 benchmarking/bench_configs.py --configs airl_hopper --gpus 8   # same, external launcher
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = ["bc_cartpole", "gail_halfcheetah", "airl_hopper", "dagger_pong", "preference_walker2d"]


def _sync(device):
    import torch as th

    if device.type == "cuda":
        th.cuda.synchronize()


def _eval(policy, venv, n):
    from imitation_amd.rl.evaluation import evaluate_policy

    if n <= 0:
        return None
    mean_r, _ = evaluate_policy(policy, venv, n_eval_episodes=n)
    return float(mean_r)


def make_step(name, device, rank, args):
    """(built recipe, step fn -> units done, unit name, policy for eval, eval venv)."""
    from imitation_amd import models

    if name == "bc_cartpole":
        b = models.build(name, device=device, seed=args.seed)
        tr = b.trainer

        def step():
            tr.train(n_batches=50, log_interval=10**9, progress_bar=False)
            return 50 * tr.minibatch_size if hasattr(tr, "minibatch_size") else 50 * 32

        return b, step, "samples/s", tr.policy, b.venv
    if name == "gail_halfcheetah":
        b = models.build(name, device=device, seed=args.seed, rank=rank)
        tr = b.trainer

        def step(k: int = 1):  # k rounds in one train() call (round r + 1 enqueued behind r)
            tr.train(k * tr.gen_train_timesteps)
            return k * tr.gen_train_timesteps

        step.multi = True
        return b, step, "env-steps/s", tr.gen_algo.policy, b.venv
    if name == "airl_hopper":
        b = models.build(name, device=device, seed=args.seed, rank=rank)
        tr = b.trainer

        def step(k: int = 1):  # k rounds in one train() call (round r + 1 enqueued behind r)
            tr.train(k * tr.gen_train_timesteps)
            return k * tr.gen_train_timesteps

        step.multi = True
        return b, step, "env-steps/s", tr.gen_algo.policy, b.venv
    if name == "dagger_pong":
        b = models.build(name, device=device, seed=args.seed, rank=rank)
        tr = b.trainer

        def step():
            tr.train(args.dagger_round_steps, rollout_round_min_episodes=1,
                     rollout_round_min_timesteps=args.dagger_round_steps,
                     bc_train_kwargs=dict(n_epochs=1, log_interval=10**9, progress_bar=False))
            return tr.last_train_timesteps_local  # this rank's steps (x world below)

        return b, step, "env-steps/s", tr.policy, b.venv
    if name == "preference_walker2d":
        # the reference schedule (5 iterations over 1e6 steps, 5000 comparisons); warm-up
        # steps run the initial iteration (initial comparisons x epoch multiplier 200), each
        # timed step is one later iteration: agent training (200K env steps) + sampling,
        # fragmenting, preference gathering and 3 reward epochs over the growing dataset
        b = models.build(name, device=device, seed=args.seed, rank=rank)
        tr = b.trainer
        it = tr.train_iter(b.extras["total_timesteps"], total_comparisons=args.pref_comparisons)

        def step():
            next(it)
            return b.env_steps_per_round

        return b, step, "env-steps/s", b.extras["agent"].policy, b.venv
    raise KeyError(name)


def run_config(name, args, device, rank, world):
    from imitation_amd.parallel import dist as pdist

    b, step, unit, policy, venv = make_step(name, device, rank, args)
    multi = getattr(step, "multi", False)  # the step runs k rounds in one call (as training does)
    if multi:
        if args.warmup:
            step(args.warmup)
    else:
        for _ in range(args.warmup):
            step()
    pdist.barrier()
    _sync(device)
    t0 = time.perf_counter()
    units = 0
    if multi:
        units = step(args.steps)
    else:
        for _ in range(args.steps):
            units += step()
    _sync(device)
    pdist.barrier()
    dt = pdist.allreduce_scalars([time.perf_counter() - t0], op="max")[0]
    total = units * world
    if hasattr(b.trainer, "sync_env_to_host"):
        b.trainer.sync_env_to_host()
    ret = _eval(policy, venv, args.eval_episodes)
    if ret is not None:
        ret = pdist.allreduce_scalars([ret], op="sum")[0] / world
    return {
        "config": name, "env": b.env_id, "value": round(total / dt, 2), "unit": unit, "n_gpus": world if device.type == "cuda" else 0,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / args.steps, 3),
        "final_eval_return": None if ret is None else round(float(ret), 3), "engine": b.extras.get("engine", "host"),
        "device": str(device), "data": "synthetic env + synthetic demos, random-init weights",
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="all")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--eval-episodes", type=int, default=5)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", default=None)
    p.add_argument("--dagger-round-steps", type=int, default=2048)
    p.add_argument("--pref-comparisons", type=int, default=5000)
    p.add_argument("--out", default=None, help="append JSON lines to this file (rank 0)")
    p.add_argument("--gpus", type=int, default=1,
                   help="data-parallel ranks, one per GPU (self-spawned without a launcher; weak scaling)")
    args = p.parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        from imitation_amd.parallel.launch import spawn_ranks

        sys.exit(spawn_ranks(args.gpus, __file__, sys.argv[1:], label="bench_configs.py"))
    import torch as th

    from imitation_amd.parallel import dist as pdist

    rank, world = pdist.init()
    if world != args.gpus and "WORLD_SIZE" in os.environ and args.gpus > 1:
        print(f"bench_configs.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        sys.exit(2)
    if args.device:
        device = th.device(args.device)
    elif th.cuda.is_available():
        th.cuda.set_device(pdist.local_rank() % th.cuda.device_count())
        device = th.device("cuda", th.cuda.current_device())
    else:
        device = th.device("cpu")
    names = CONFIGS if args.configs == "all" else args.configs.split(",")
    for name in names:
        th.manual_seed(args.seed + rank)
        np.random.seed(args.seed + rank)
        dev = th.device("cpu") if name == "bc_cartpole" and args.device is None else device
        res = run_config(name, args, dev, rank, world)
        if rank == 0:
            line = json.dumps(res)
            print(line, flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(line + "\n")
    pdist.shutdown()


if __name__ == "__main__":
    main()

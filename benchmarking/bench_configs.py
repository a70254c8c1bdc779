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
dagger_pong            one DAgger round at the reference's schedule        env-steps/s
                       (>= 3 episodes and >= 500 env steps per round,
                       then 4 BC epochs over the aggregate)
dagger_pong_1epoch     labelled extra: >= 2048 env steps + ONE BC epoch    env-steps/s
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
# timed steps when --steps is not given: the ms-scale GAIL / AIRL rounds are noisy over 3 rounds
# (AIRL 6.7-7.8 ms over 3 vs 6.36-6.44 ms over 10, round 5), the 100-500 ms rounds are not
DEFAULT_STEPS = {"gail_halfcheetah": 20, "airl_hopper": 10}


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
    demos = getattr(args, "_demos", {}).get(name)
    if name == "gail_halfcheetah":
        b = models.build(name, device=device, seed=args.seed, rank=rank, demonstrations=demos)
        tr = b.trainer

        def step(k: int = 1):  # k rounds in one train() call (round r + 1 enqueued behind r)
            tr.train(k * tr.gen_train_timesteps)
            return k * tr.gen_train_timesteps

        step.multi = True
        return b, step, "env-steps/s", tr.gen_algo.policy, b.venv
    if name == "airl_hopper":
        b = models.build(name, device=device, seed=args.seed, rank=rank, demonstrations=demos)
        tr = b.trainer

        def step(k: int = 1):  # k rounds in one train() call (round r + 1 enqueued behind r)
            tr.train(k * tr.gen_train_timesteps)
            return k * tr.gen_train_timesteps

        step.multi = True
        return b, step, "env-steps/s", tr.gen_algo.policy, b.venv
    if name == "dagger_pong":
        # the reference's SimpleDAggerTrainer.train defaults (src/imitation/algorithms/dagger.py:618-697):
        # rollout_round_min_episodes=3, rollout_round_min_timesteps=500, BC for DEFAULT_N_EPOCHS = 4
        # epochs per round (dagger.py:326,491-492); one timed step = one round
        b = models.build(name, device=device, seed=args.seed, rank=rank)
        tr = b.trainer

        def step():
            tr.train(1, rollout_round_min_episodes=3, rollout_round_min_timesteps=500,
                     bc_train_kwargs=dict(n_epochs=tr.DEFAULT_N_EPOCHS, log_interval=10**9, progress_bar=False))
            return tr.last_train_timesteps_local  # this rank's steps (x world below)

        return b, step, "env-steps/s", tr.policy, b.venv
    if name == "dagger_pong_1epoch":
        # labelled extra (rounds 2-5's config): >= --dagger-round-steps env steps per round, ONE BC epoch
        b = models.build("dagger_pong", device=device, seed=args.seed, rank=rank)
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


EXPERT_CONFIGS = ("gail_halfcheetah", "airl_hopper")


def make_expert(name, args, device):
    """Expert mode (``--expert-steps``): a PPO expert trained on the env reward by the device
    engine with the config's own generator (``debug_use_ground_truth``), its stochastic rollouts
    as the demonstrations (``DeviceGeneratorCore.device_demonstrations``); returns (demos,
    R_expert of its deterministic evaluation, expert training seconds)."""
    import torch as th

    from imitation_amd import models

    t0 = time.perf_counter()
    ex = models.build(name, device=device, seed=args.seed + 100, debug_use_ground_truth=True)
    ex.trainer.train(max(ex.trainer.gen_train_timesteps, args.expert_steps))
    _sync(device)
    t_ex = time.perf_counter() - t0
    r, _ = ex.trainer.device_evaluate(args.eval_episodes_expert, deterministic=True, seed=10_000 + args.seed)
    demos = ex.trainer.device_demonstrations(args.expert_demo_steps, deterministic=False, seed=20_000 + args.seed)
    del ex
    th.cuda.empty_cache()
    return demos, float(np.mean(r)), t_ex


def run_config(name, args, device, rank, world):
    from imitation_amd.parallel import dist as pdist

    steps = args.steps if args.steps is not None else DEFAULT_STEPS.get(name, 3)

    expert = None
    if args.expert_steps > 0 and name in EXPERT_CONFIGS:
        if world > 1:
            raise SystemExit("--expert-steps is a single-rank mode")
        demos, r_expert, t_ex = make_expert(name, args, device)
        args._demos = {name: demos}
        expert = dict(expert_return=round(r_expert, 3), expert_steps=args.expert_steps, expert_train_s=round(t_ex, 3),
                      n_demo_transitions=len(demos.acts))
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
        units = step(steps)
    else:
        for _ in range(steps):
            units += step()
    _sync(device)
    pdist.barrier()
    dt = pdist.allreduce_scalars([time.perf_counter() - t0], op="max")[0]
    total = units * world
    if expert is not None:  # imitation budget (untimed), then the normalised score
        from imitation_amd.testing import imitation_quality as iq

        done = (args.warmup + steps) * b.trainer.gen_train_timesteps
        if args.imit_steps > done:
            b.trainer.train((args.imit_steps - done) // b.trainer.gen_train_timesteps * b.trainer.gen_train_timesteps)
        r, _ = b.trainer.device_evaluate(args.eval_episodes_expert, deterministic=True, seed=10_000 + args.seed)
        rand = iq.random_return(b.env_id, args.eval_episodes_expert, args.seed)
        expert.update(learner_return=round(float(np.mean(r)), 3), random_return=round(rand, 3),
                      imit_steps=max(args.imit_steps, done),
                      normalized_score=round(iq.normalized_score(float(np.mean(r)), rand, expert["expert_return"]), 4))
    if hasattr(b.trainer, "sync_env_to_host"):
        b.trainer.sync_env_to_host()
    ret = _eval(policy, venv, args.eval_episodes)
    if ret is not None:
        ret = pdist.allreduce_scalars([ret], op="sum")[0] / world
    out = {
        "config": name, "env": b.env_id, "value": round(total / dt, 2), "unit": unit, "n_gpus": world if device.type == "cuda" else 0,
        "steps": steps, "warmup": args.warmup, "ms_per_step": round(1e3 * dt / steps, 3),
        "final_eval_return": None if ret is None else round(float(ret), 3), "engine": b.extras.get("engine", "host"),
        "device": str(device), "data": "synthetic env + synthetic demos, random-init weights",
    }
    if expert is not None:
        out.update(expert, data="synthetic env; demonstrations = rollouts of a device-PPO expert trained on the env "
                                "reward; random-init learner")
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", default="all")
    p.add_argument("--steps", type=int, default=None, help="timed steps (default: 20 GAIL, 10 AIRL, 3 others)")
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--eval-episodes", type=int, default=5)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", default=None)
    p.add_argument("--dagger-round-steps", type=int, default=2048)
    p.add_argument("--pref-comparisons", type=int, default=5000)
    p.add_argument("--out", default=None, help="append JSON lines to this file (rank 0)")
    p.add_argument("--expert-steps", type=int, default=0,
                   help="expert mode (gail_halfcheetah / airl_hopper): train a PPO expert on the env reward for this "
                        "many steps, imitate its rollouts, report the normalised score")
    p.add_argument("--expert-demo-steps", type=int, default=50_000)
    p.add_argument("--imit-steps", type=int, default=5_000_000, help="expert mode: learner env steps before scoring")
    p.add_argument("--eval-episodes-expert", type=int, default=50)
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

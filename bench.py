#!/usr/bin/env python
"""Headline benchmark: GAIL on the HalfCheetah-shaped env, PPO generator, 8 envs per GPU.

Metric (BASELINE.json): whole-node env-steps/s of GAIL training on
seals/HalfCheetah at 1/2/4/8 MI355X. Config = the reference's tuned
``gail_seals_half_cheetah_best_hp_eval.json``:

* 8 envs per rank, PPO generator ``FeedForward32Policy`` + ``NormalizeFeaturesExtractor``
  (RunningNorm), rl batch 4096 (n_steps 512), minibatch 64, 5 epochs, clip 0.1,
  γ=λ=0.95, lr 2.625e-4, ent 3.99e-6, vf 0.1148, max_grad_norm 0.8;
* reward: ``BasicRewardNet`` (RunningNorm input) wrapped in ``NormalizedRewardNet``;
* demo_batch_size 8192, gen_replay_buffer_capacity 512, 8 discriminator updates / round.

One bench *step* = one full GAIL round (4096 env steps of generator rollout with the
learned reward, the PPO update, 8 discriminator updates). Weak scaling: every rank
runs the full per-GPU config; DP averages PPO and discriminator gradients with one
RCCL all-reduce per optimizer step. ``value`` = total env steps of all ranks per
second.

Data: MuJoCo is not available, so the env is the synthetic HalfCheetah-shaped
locomotion model (obs 17, act 6, horizon 1000) and the "expert" demonstrations are
synthetic trajectories of that env (random-init policy); weights are random-init.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--engine", choices=["device", "host"], default=os.environ.get("IA_BENCH_ENGINE", "device"))
    p.add_argument("--env", default="seals/HalfCheetah-v1")
    p.add_argument("--n-envs", type=int, default=8)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--profile-dir", default=None)
    return p.parse_args()


BASELINE_VALUE = None  # the reference publishes no throughput number


def main():
    args = parse()
    import torch as th

    from imitation_amd.parallel import dist as pdist

    rank, world = pdist.init()
    if th.cuda.is_available():
        th.cuda.set_device(pdist.local_rank())
        device = th.device("cuda", pdist.local_rank())
    else:
        device = th.device("cpu")
    th.manual_seed(args.seed + rank)
    np.random.seed(args.seed + rank)

    from imitation_amd.data import rollout
    from imitation_amd.policies.base import FeedForward32Policy, NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicRewardNet, NormalizedRewardNet
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import logger as imit_logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    rng = np.random.default_rng(args.seed + 1000 * rank)
    venv = make_vec_env(args.env, rng=rng, n_envs=args.n_envs)
    # synthetic demonstrations: random-policy trajectories of the same env (>= demo batch)
    demo_env = make_vec_env(args.env, rng=np.random.default_rng(12345), n_envs=16)
    demos = rollout.generate_trajectories(None, demo_env, rollout.make_min_timesteps(16384), rng=np.random.default_rng(0))
    transitions = rollout.flatten_trajectories(demos)

    rl_kwargs = dict(batch_size=64, clip_range=0.1, ent_coef=3.992371122209408e-6, gae_lambda=0.95, gamma=0.95,
                     learning_rate=0.00026250519057717037, max_grad_norm=0.8, n_epochs=5, vf_coef=0.11483689492120866)
    policy_kwargs = dict(features_extractor_class=NormalizeFeaturesExtractor,
                         features_extractor_kwargs=dict(normalize_class=RunningNorm))
    n_steps = 4096 // args.n_envs
    gen = PPO(FeedForward32Policy, venv, n_steps=n_steps, policy_kwargs=policy_kwargs, device=device, seed=args.seed, **rl_kwargs)
    reward_net = NormalizedRewardNet(
        BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm), RunningNorm
    )
    log = imit_logger.configure(os.path.join("/tmp", f"ia_bench_{os.getpid()}"), format_strs=[])
    algo_kwargs = dict(demo_batch_size=8192, gen_replay_buffer_capacity=512, n_disc_updates_per_round=8)
    if args.engine == "device":
        from imitation_amd.engine.gail import DeviceGAIL

        trainer = DeviceGAIL(demonstrations=transitions, venv=venv, gen_algo=gen, reward_net=reward_net,
                             custom_logger=log, **algo_kwargs)
    else:
        from imitation_amd.algorithms.adversarial.gail import GAIL

        trainer = GAIL(demonstrations=transitions, venv=venv, gen_algo=gen, reward_net=reward_net, custom_logger=log,
                       **algo_kwargs)
    steps_per_round = trainer.gen_train_timesteps

    def one_round():
        trainer.train(steps_per_round)

    for _ in range(args.warmup):
        one_round()
    pdist.barrier()
    if device.type == "cuda":
        th.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_round()
    if device.type == "cuda":
        th.cuda.synchronize()
    pdist.barrier()
    dt = time.perf_counter() - t0
    dt = pdist.allreduce_scalars([dt], op="max")[0]
    total_steps = steps_per_round * args.steps * world
    value = total_steps / dt
    if rank == 0:
        out = {
            "metric": "env-steps/sec (whole node), GAIL seals/HalfCheetah-v1-shaped, PPO generator, 8 envs/GPU",
            "value": round(value, 2),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else value / BASELINE_VALUE,
            "dtype": "bf16",
            "data": "synthetic (HalfCheetah-shaped native env, random-policy demos, random-init nets)",
            "config": {
                "model": "GAIL: FeedForward32Policy[32,32]+RunningNorm / BasicRewardNet(32,32)+RunningNorm",
                "global_batch": 4096 * world,
                "seq_len": n_steps,
                "parallelism": f"dp{world}",
                "engine": args.engine,
                "env": args.env,
            },
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()

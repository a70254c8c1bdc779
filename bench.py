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
locomotion model (obs 17, act 6, horizon 1000); weights are random-init.

Imitation quality (the reference benchmark's ``imit_stats.monitor_return_mean``, normalised
``(R - R_random) / (R_expert - R_random)``: ``benchmarking/README.md:94-98``,
``benchmarking/sacred_output_to_markdown_summary.py:79-140``), all OUTSIDE the timed region:

1. before the trainer is built, a PPO expert of the same generator config is trained on the
   env reward by the device engine (``--expert-steps``), scored over 50 deterministic
   episodes, and 50K transitions of its stochastic rollouts become the demonstrations
   (cached under ``--expert-cache``, keyed by config + seed + rank, so a repeated run skips it);
2. the timed GAIL trainer imitates those demonstrations (the timed region is unchanged:
   ``tests/test_bench_contract.py`` pins its text);
3. after the K timed rounds, training continues untimed to ``--quality-steps`` env steps
   per rank, then ``final_eval_return`` = mean of 50 deterministic ``device_evaluate``
   episodes; ``expert_return``, ``random_return`` and ``normalized_score`` are reported
   alongside. ``--quality-steps 0`` (or the host engine) falls back to random-policy demos.
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
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--engine", choices=["auto", "device", "host"], default=os.environ.get("IA_BENCH_ENGINE", "auto"))
    p.add_argument("--env", default="HalfCheetah-v4")
    p.add_argument("--eval-episodes", type=int, default=50, help="final eval episodes (after timing); 0 = skip")
    p.add_argument("--quality-steps", type=int, default=1_000_000,
                   help="imitation budget per rank (env steps, timed rounds included) before the final evaluation; "
                        "0 = imitate random-policy demos and skip the expert (device engine only)")
    p.add_argument("--expert-steps", type=int, default=5_000_000, help="PPO expert budget (env reward), untimed")
    p.add_argument("--expert-cache", default=os.environ.get("IA_BENCH_EXPERT_CACHE", "/tmp/ia_bench_expert"),
                   help="directory caching the expert demonstrations ('' = no cache)")
    p.add_argument("--n-envs", type=int, default=8)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--profile-dir", default=None)
    return p.parse_args()


BASELINE_VALUE = None  # the reference publishes no throughput number


def spawn_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: N rank processes (one per GPU, RCCL), started before
    anything touches the GPU (devices counted from sysfs, :mod:`imitation_amd.parallel.launch`);
    returns the worst exit code. ``IMITATION_AMD_DIST_BACKEND=gloo`` rehearses the
    multi-rank path with every rank on one device (or on the CPU)."""
    from imitation_amd.parallel.launch import spawn_ranks as _spawn

    return _spawn(n, __file__, sys.argv[1:], label="bench.py")


def fill_expert_cache(args):
    """Train the expert (or find it cached) in a CHILD process on this rank's GPU, before this
    process touches the GPU: the measuring process then only loads the cached demonstrations, as
    a warm-cache run does (hosting the 5M-step expert run in the same process left the timed
    rounds ~25% slower, ``profiles/r6_bench_quality.md``). The child runs without a process group
    (one GPU, the same seed on every rank; the demonstrations' seed differs by rank). Returns
    whether the child found the cache filled already (None: no child ran, or it failed)."""
    import subprocess

    from imitation_amd.parallel.launch import count_gpus

    n = count_gpus()
    if n < 1:
        return None
    rank = int(os.environ.get("RANK", "0"))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                                                               "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK")}
    cmd = [sys.executable, "-m", "imitation_amd.testing.imitation_quality", "expert", "--env", args.env,
           "--seed", str(args.seed), "--expert-steps", str(args.expert_steps), "--n-eval", str(args.eval_episodes),
           "--rank", str(rank), "--n-envs", str(args.n_envs), "--device", f"cuda:{int(os.environ.get('LOCAL_RANK', '0')) % n}",
           "--cache-dir", args.expert_cache]
    try:  # (bounded: a stuck child must not hang the bench; ~5 s normally)
        p = subprocess.run(cmd, env=env, cwd=os.path.dirname(os.path.abspath(__file__)), stdout=subprocess.PIPE,
                           text=True, timeout=900)
    except subprocess.TimeoutExpired:
        print("bench.py: expert child timed out; the expert trains in this process instead", file=sys.stderr)
        return None
    sys.stderr.write(p.stdout)
    if p.returncode:
        print(f"bench.py: expert child exited {p.returncode}; the expert trains in this process instead", file=sys.stderr)
        return None
    return "cached=True" in p.stdout


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    child_cached = None
    if args.quality_steps > 0 and args.eval_episodes > 0 and args.engine != "host" and args.expert_cache:
        child_cached = fill_expert_cache(args)
    import torch as th

    from imitation_amd.parallel import dist as pdist

    rank, world = pdist.init()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        sys.exit(2)
    if th.cuda.is_available():
        dev_idx = pdist.local_rank() % th.cuda.device_count()  # == local rank on a full node
        th.cuda.set_device(dev_idx)
        device = th.device("cuda", dev_idx)
    else:
        device = th.device("cpu")
    th.manual_seed(args.seed + rank)
    np.random.seed(args.seed + rank)

    from imitation_amd import models

    # imitation quality (reference benchmarking/README.md:94-98): untimed, before the trainer is
    # built -- a device-PPO expert trained on the env reward, its stochastic rollouts are the
    # demonstrations the timed GAIL trainer imitates (cached under --expert-cache)
    quality = args.quality_steps > 0 and args.eval_episodes > 0 and device.type == "cuda" and args.engine != "host"
    expert = None
    if quality:
        from imitation_amd.testing import imitation_quality as iq

        expert = iq.expert_demonstrations("gail_halfcheetah", args.env, seed=args.seed,
                                          expert_timesteps=args.expert_steps, n_demo_timesteps=50_000,
                                          n_eval=args.eval_episodes, device=device, rank=rank, world=world,
                                          n_envs=args.n_envs, cache_dir=args.expert_cache or None)

    # the reference's tuned gail_seals_half_cheetah config (imitation_amd/models/recipes.py)
    built = models.build("gail_halfcheetah", device=device, n_envs=args.n_envs, engine=args.engine, seed=args.seed,
                         rank=rank, env_id=args.env, log_dir=os.path.join("/tmp", f"ia_bench_{os.getpid()}"),
                         demonstrations=None if expert is None else expert["demos"])
    trainer, venv = built.trainer, built.venv
    engine = built.extras["engine"]
    n_steps = trainer.gen_algo.n_steps
    steps_per_round = trainer.gen_train_timesteps

    # --- timed region (tests/test_bench_contract.py pins its text) ---
    # W warm-up rounds, then K timed rounds as ONE train() call, as a training run issues them:
    # the trainer enqueues round r + 1's rollout behind round r's PPO update before it logs
    # round r, so the device never waits for the host between rounds (one call per round
    # would end every round with a host round trip)
    if args.warmup:
        trainer.train(steps_per_round * args.warmup)
    pdist.barrier()
    if device.type == "cuda":
        th.cuda.synchronize()
    t0 = time.perf_counter()
    trainer.train(steps_per_round * args.steps)
    if device.type == "cuda":
        th.cuda.synchronize()
    pdist.barrier()
    dt_local = time.perf_counter() - t0
    per_rank = [round(1000.0 * x / args.steps, 3) for x in pdist.all_gather_object(dt_local)]
    dt = pdist.allreduce_scalars([dt_local], op="max")[0]
    total_steps = steps_per_round * args.steps * world
    value = total_steps / dt
    # --- end of timed region ---
    eval_return = None
    qual = dict(expert_return=None, random_return=None, normalized_score=None)
    if quality and engine == "device":  # untimed: imitate to the budget, then 50 deterministic episodes on the GPU
        from imitation_amd.testing.imitation_quality import normalized_score

        done = steps_per_round * (args.warmup + args.steps)
        rest = -(-max(0, args.quality_steps - done) // steps_per_round) * steps_per_round
        if rest:
            trainer.train(rest)
        rets, _ = trainer.device_evaluate(args.eval_episodes, deterministic=True, seed=10_000 + args.seed)
        eval_return = float(pdist.allreduce_scalars([float(np.mean(rets))], op="sum")[0]) / world
        ex_r = float(pdist.allreduce_scalars([expert["expert_return"]], op="sum")[0]) / world
        rnd_r = float(expert["random_return"])
        qual = dict(expert_return=round(ex_r, 3), random_return=round(rnd_r, 3),
                    normalized_score=round(normalized_score(eval_return, rnd_r, ex_r), 4),
                    imitation_env_steps_per_rank=done + rest, expert_env_steps=args.expert_steps,
                    expert_cached=bool(expert["cached"] if child_cached is None else child_cached),
                    expert_in_child_process=child_cached is not None, expert_train_s=round(float(expert["expert_train_s"]), 3),
                    eval_episodes=args.eval_episodes)
        eval_return = round(eval_return, 3)
    elif args.eval_episodes > 0:  # outside the timed region: mean return of the trained generator
        from imitation_amd.rl.evaluation import evaluate_policy

        if hasattr(trainer, "sync_env_to_host"):
            trainer.sync_env_to_host()
        mean_r, _ = evaluate_policy(trainer.gen_algo.policy, venv, n_eval_episodes=args.eval_episodes)
        eval_return = round(float(pdist.allreduce_scalars([float(mean_r)], op="sum")[0]) / world, 3)
    if rank == 0:
        out = {
            "metric": "env-steps/sec (whole node) + final eval return, GAIL HalfCheetah-v4 at 1/2/4/8 MI355X",
            "value": round(value, 2),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else value / BASELINE_VALUE,
            # fp32 master weights / accumulation; PPO MFMA products split-bf16 x3, discriminator bf16 operands
            "dtype": "mixed (fp32 master weights and accumulation; PPO products as split-bf16 x3 ~fp32, discriminator bf16)",
            "final_eval_return": eval_return,
            **qual,
            "per_rank_ms_per_step": per_rank,
            "data": ("synthetic (native HalfCheetah-v4-shaped env; demos = stochastic rollouts of a device-PPO expert "
                     "trained on the env reward, untimed and cached; random-init learner)" if qual["normalized_score"]
                     is not None else "synthetic (native HalfCheetah-v4-shaped env, random-policy demos, random-init nets)"),
            "config": {
                "model": "GAIL: FeedForward32Policy[32,32]+RunningNorm / BasicRewardNet(32,32)+RunningNorm",
                "global_batch": 4096 * world,
                "seq_len": n_steps,
                "parallelism": f"dp{world}",
                "engine": engine,
                "env": args.env,
            },
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()

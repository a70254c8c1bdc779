"""Imitation quality of the device engines: does the learner approach the expert?

The reference's benchmark reports ``imit_stats/monitor_return_mean`` normalised as
``(score - random) / (expert - random)`` (``benchmarking/README.md:94-98``,
``benchmarking/sacred_output_to_markdown_summary.py:79-140``). This module reproduces that
measurement for :class:`~imitation_amd.engine.gail.DeviceGAIL` and
:class:`~imitation_amd.engine.airl.DeviceAIRL`:

* **CartPole** (``seals/CartPole-v0``): the checked-in reference expert
  (``tests/testdata/expert_models/cartpole_0/policies/final/model.zip``) is rolled out for the
  demonstrations, learner / trainer hyper-parameters are the reference tutorials'
  (``docs/tutorials/3_train_gail.ipynb``, ``4_train_airl.ipynb``).
* **Pendulum** (``Pendulum-v1``): the checked-in demonstrations
  ``tests/testdata/expert_models/pendulum_0/rollouts/final.npz`` (their mean return is the
  expert score).
* **Synthetic locomotion** (``expert`` mode of ``benchmarking/bench_configs.py``): a PPO expert
  is trained on the device engine with the env reward first (``debug_use_ground_truth``), its
  deterministic rollouts are the demonstrations.

Every score is measured by :meth:`DeviceGeneratorCore.device_evaluate` (SB3 ``evaluate_policy``
semantics, deterministic actions, on the GPU). The random-policy score uses the native
``RandomPolicy`` on the host env.
"""

from __future__ import annotations

import os
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch as th

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
TESTDATA = os.path.join(ROOT, "tests", "testdata", "expert_models")
CARTPOLE_EXPERT_ZIP = os.path.join(TESTDATA, "cartpole_0", "policies", "final", "model.zip")
PENDULUM_DEMOS = os.path.join(TESTDATA, "pendulum_0", "rollouts", "final.npz")


def normalized_score(score: float, random_score: float, expert_score: float) -> float:
    """``(score - random) / (expert - random)`` (reference benchmark summary)."""
    return float((score - random_score) / (expert_score - random_score))


def random_return(env_id: str, n_episodes: int = 50, seed: int = 0) -> float:
    """Mean return of the uniform-random policy (reference: ``random`` policy type)."""
    from imitation_amd.data import rollout
    from imitation_amd.util.util import make_vec_env

    venv = make_vec_env(env_id, rng=np.random.default_rng(seed), n_envs=8)
    venv.action_space.seed(seed)
    trajs = rollout.generate_trajectories(None, venv, rollout.make_min_episodes(n_episodes), rng=np.random.default_rng(seed))
    return float(np.mean([t.rews.sum() for t in trajs[:n_episodes]]))


def cartpole_expert_demos(n_episodes: int = 60, seed: int = 0):
    """Rollouts of the checked-in reference CartPole expert on ``seals/CartPole-v0``."""
    from imitation_amd.data import rollout
    from imitation_amd.data.wrappers import RolloutInfoWrapper
    from imitation_amd.policies import serialize
    from imitation_amd.util.util import make_vec_env

    venv = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(seed), n_envs=8,
                        post_wrappers=[lambda e, _: RolloutInfoWrapper(e)])
    expert = serialize.load_policy("ppo", venv, path=CARTPOLE_EXPERT_ZIP)
    trajs = rollout.rollout(expert, venv, rollout.make_sample_until(min_timesteps=None, min_episodes=n_episodes),
                            rng=np.random.default_rng(seed))
    return trajs


def pendulum_expert_demos():
    from imitation_amd.data import serialize

    return serialize.load_with_rewards(PENDULUM_DEMOS)


def _cartpole_trainer(algo: str, demos, seed: int, device, logger, cap: int = 512):
    """The reference tutorials' GAIL / AIRL CartPole setups on the device engines."""
    from imitation_amd.engine.airl import DeviceAIRL
    from imitation_amd.engine.gail import DeviceGAIL
    from imitation_amd.rewards.reward_nets import BasicRewardNet, BasicShapedRewardNet
    from imitation_amd.rl.policies import ActorCriticPolicy
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    venv = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(seed), n_envs=8)
    if algo == "gail":
        learner = PPO(ActorCriticPolicy, venv, batch_size=64, ent_coef=0.0, learning_rate=4e-4, gamma=0.95, n_epochs=5,
                      seed=seed, device=device)
        rn = BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm)
        tr = DeviceGAIL(demonstrations=demos, demo_batch_size=1024, gen_replay_buffer_capacity=cap,
                        n_disc_updates_per_round=8, venv=venv, gen_algo=learner, reward_net=rn, custom_logger=logger)
    else:
        learner = PPO(ActorCriticPolicy, venv, batch_size=64, ent_coef=0.0, learning_rate=5e-4, gamma=0.95,
                      clip_range=0.1, vf_coef=0.1, n_epochs=5, seed=seed, device=device)
        rn = BasicShapedRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm)
        tr = DeviceAIRL(demonstrations=demos, demo_batch_size=2048, gen_replay_buffer_capacity=cap,
                        n_disc_updates_per_round=16, venv=venv, gen_algo=learner, reward_net=rn, custom_logger=logger)
    return tr


def _pendulum_trainer(algo: str, demos, seed: int, device, logger, cap: int = 512, n_disc: Optional[int] = None,
                      demo_batch: Optional[int] = None, normalize_output: bool = False):
    """Pendulum-v1 (continuous): SB3 MlpPolicy PPO with the rl-zoo Pendulum settings
    (gamma 0.9, gae_lambda 0.95, lr 1e-3, n_steps 1024 x 4 envs, 10 epochs, use_sde off).
    ``n_disc`` / ``demo_batch`` override the tutorial's discriminator schedule;
    ``normalize_output`` wraps the reward net in ``NormalizedRewardNet`` (the reference scripts'
    default ``normalize_output_layer=RunningNorm``)."""
    from imitation_amd.engine.airl import DeviceAIRL
    from imitation_amd.engine.gail import DeviceGAIL
    from imitation_amd.rewards.reward_nets import BasicRewardNet, BasicShapedRewardNet
    from imitation_amd.rl.policies import ActorCriticPolicy
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    venv = make_vec_env("Pendulum-v1", rng=np.random.default_rng(seed), n_envs=8)
    learner = PPO(ActorCriticPolicy, venv, n_steps=1024, batch_size=64, gamma=0.9, gae_lambda=0.95, learning_rate=1e-3,
                  n_epochs=10, ent_coef=0.0, clip_range=0.2, seed=seed, device=device)
    from imitation_amd.rewards.reward_nets import NormalizedRewardNet

    if algo == "gail":
        rn = BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm)
        if normalize_output:
            rn = NormalizedRewardNet(rn, RunningNorm)
        tr = DeviceGAIL(demonstrations=demos, demo_batch_size=demo_batch or 1024, gen_replay_buffer_capacity=cap,
                        n_disc_updates_per_round=n_disc or 8, venv=venv, gen_algo=learner, reward_net=rn,
                        custom_logger=logger)
    else:
        rn = BasicShapedRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm)
        if normalize_output:
            rn = NormalizedRewardNet(rn, RunningNorm)
        tr = DeviceAIRL(demonstrations=demos, demo_batch_size=demo_batch or 2048, gen_replay_buffer_capacity=cap,
                        n_disc_updates_per_round=n_disc or 16, venv=venv, gen_algo=learner, reward_net=rn,
                        custom_logger=logger)
    return tr


def run(algo: str = "gail", env: str = "cartpole", total_timesteps: int = 200_000, seed: int = 0, n_eval: int = 50,
        eval_every: Optional[int] = None, device: Any = "cuda", verbose: bool = False, cap: int = 512,
        trainer_kwargs: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """Train ``algo`` (``gail`` / ``airl``) on ``env`` (``cartpole`` / ``pendulum``) with expert
    demonstrations and report returns + normalised scores (before, during, after)."""
    from imitation_amd.util import logger as imit_logger

    th.manual_seed(seed)
    np.random.seed(seed)
    if env == "cartpole":
        env_id = "seals/CartPole-v0"
        demos = cartpole_expert_demos(seed=seed)
        make = _cartpole_trainer
    elif env == "pendulum":
        env_id = "Pendulum-v1"
        demos = pendulum_expert_demos()
        make = _pendulum_trainer
    else:
        raise ValueError(f"unknown env {env!r}")
    expert = float(np.mean([t.rews.sum() for t in demos]))
    rand = random_return(env_id, n_eval, seed)
    log = imit_logger.configure(f"/tmp/ia_quality_{os.getpid()}", format_strs=[])
    tr = make(algo, demos, seed, device, log, cap=cap, **(trainer_kwargs or {}))

    last: Dict[str, List[float]] = {}

    def score() -> float:
        r, _ = tr.device_evaluate(n_eval, deterministic=True, seed=10_000 + seed)
        last["returns"] = list(r)
        return float(np.mean(r))

    r0 = score()
    returns_before = last["returns"]
    curve: List[Dict[str, float]] = [dict(timesteps=0, ret=r0, norm=normalized_score(r0, rand, expert))]
    step = int(eval_every or total_timesteps)
    step = max(tr.gen_train_timesteps, step // tr.gen_train_timesteps * tr.gen_train_timesteps)
    done = 0
    t_train = 0.0
    while done < total_timesteps:
        k = min(step, total_timesteps - done)
        k = max(tr.gen_train_timesteps, k // tr.gen_train_timesteps * tr.gen_train_timesteps)
        t0 = time.perf_counter()
        tr.train(k)
        th.cuda.synchronize()
        t_train += time.perf_counter() - t0
        done += k
        r = score()
        curve.append(dict(timesteps=done, ret=r, norm=normalized_score(r, rand, expert)))
        if verbose:
            print(f"{algo}/{env} seed {seed}: {done} steps: return {r:.1f} (normalised {curve[-1]['norm']:.3f})", flush=True)
    final = curve[-1]["ret"]
    return dict(algo=algo, env=env_id, seed=seed, expert_return=expert, random_return=rand, learner_return_before=r0,
                learner_return=final, normalized_score=normalized_score(final, rand, expert), curve=curve,
                total_timesteps=done, train_s=round(t_train, 3), n_eval_episodes=n_eval, n_demo_episodes=len(demos),
                returns_before=returns_before, returns_after=last["returns"])


LOCOMOTION = {"halfcheetah": ("seals/HalfCheetah-v1", "gail_halfcheetah"),
              "hopper": ("seals/Hopper-v1", "airl_hopper")}

_EXPERT_CACHE_VERSION = 1


def expert_demonstrations(recipe: str, env_id: str, seed: int = 0, expert_timesteps: int = 5_000_000,
                          n_demo_timesteps: int = 50_000, n_eval: int = 50, device: Any = "cuda", rank: int = 0,
                          world: int = 1, n_envs: int = 8, cache_dir: Optional[str] = None) -> Dict[str, Any]:
    """Expert mode of :func:`run_locomotion` as a reusable (and cached) step: train the recipe's
    generator on the env reward (``debug_use_ground_truth``) for ``expert_timesteps`` per rank,
    score it (``n_eval`` deterministic ``device_evaluate`` episodes), roll out
    ``n_demo_timesteps`` stochastic demonstration transitions and score the uniform-random
    policy on the same env. Returns ``dict(demos, expert_return, random_return, expert_train_s,
    cached)``.

    ``cache_dir``: the result is stored there as ``expert_<key>.npz`` (atomic rename), keyed by
    every argument that changes it (recipe, env, seed, budgets, rank -- the demonstrations' seed
    --, envs per rank), and reused on the next call. ``bench.py`` fills the cache from a child
    process (:func:`main`, one GPU, no process group) so the measuring process never hosts the
    expert run. Under data parallelism every rank must call this together: whether the cache is
    used is agreed over the process group (a cache miss trains the expert data-parallel in
    process, so a lone rank training would wait for the others forever)."""
    import hashlib
    import json

    from imitation_amd import models
    from imitation_amd.data import types
    from imitation_amd.parallel import dist as pdist

    key = dict(v=_EXPERT_CACHE_VERSION, recipe=recipe, env=env_id, seed=seed, expert_timesteps=expert_timesteps,
               n_demo=n_demo_timesteps, n_eval=n_eval, rank=rank, n_envs=n_envs)
    path = None
    loaded = None
    if cache_dir:
        digest = hashlib.sha256(json.dumps(key, sort_keys=True).encode()).hexdigest()[:16]
        path = os.path.join(cache_dir, f"expert_{digest}.npz")
        if os.path.exists(path):
            try:
                with np.load(path, allow_pickle=False) as z:
                    loaded = {k: z[k] for k in z.files}
            except (OSError, ValueError):  # torn / foreign file: retrain
                loaded = None
    have = 1.0 if loaded is not None else 0.0
    if world > 1:
        have = pdist.allreduce_scalars([have], op="min")[0]
    if have > 0.5:
        demos = types.Transitions(obs=loaded["obs"], acts=loaded["acts"], next_obs=loaded["next_obs"],
                                  dones=loaded["dones"], infos=np.array([{}] * len(loaded["acts"])))
        return dict(demos=demos, expert_return=float(loaded["expert_return"]),
                    random_return=float(loaded["random_return"]), expert_train_s=float(loaded["expert_train_s"]),
                    cached=True)
    t0 = time.perf_counter()
    ex = models.build(recipe, device=device, seed=seed + 100, n_envs=n_envs, env_id=env_id,
                      debug_use_ground_truth=True)
    ex.trainer.train(max(ex.trainer.gen_train_timesteps, expert_timesteps))
    if th.cuda.is_available():
        th.cuda.synchronize()
    t_expert = time.perf_counter() - t0
    r_exp, _ = ex.trainer.device_evaluate(n_eval, deterministic=True, seed=10_000 + seed)
    expert = float(np.mean(r_exp))
    demos = ex.trainer.device_demonstrations(n_demo_timesteps, deterministic=False, seed=20_000 + seed + 97 * rank)
    del ex
    rand = random_return(env_id, n_eval, seed)
    if path is not None:
        os.makedirs(cache_dir, exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp.npz"
        np.savez(tmp, obs=demos.obs, acts=demos.acts, next_obs=demos.next_obs, dones=demos.dones,
                 expert_return=np.float64(expert), random_return=np.float64(rand), expert_train_s=np.float64(t_expert))
        os.replace(tmp, path)
    return dict(demos=demos, expert_return=expert, random_return=rand, expert_train_s=t_expert, cached=False)


def run_locomotion(algo: str = "gail", env: str = "halfcheetah", expert_timesteps: int = 5_000_000,
                   total_timesteps: int = 5_000_000, n_demo_timesteps: int = 50_000, seed: int = 0, n_eval: int = 50,
                   eval_every: Optional[int] = None, device: Any = "cuda", verbose: bool = False) -> Dict[str, Any]:
    """Expert mode of the benchmark configs on the synthetic MuJoCo-shaped envs (no MuJoCo /
    HF experts here): (1) a PPO expert is trained on the env reward by the device engine with the
    recipe's own generator config (``debug_use_ground_truth``), (2) its stochastic rollouts are
    the demonstrations (as the reference rolls out its experts), (3) the recipe's GAIL
    (``gail_halfcheetah``) or AIRL (``airl_hopper``) learner imitates them; normalised score as
    in :func:`run`, R_expert = the expert's deterministic evaluation."""
    from imitation_amd import models

    env_id, _ = LOCOMOTION[env]
    recipe = "gail_halfcheetah" if algo == "gail" else "airl_hopper"
    th.manual_seed(seed)
    np.random.seed(seed)
    t0 = time.perf_counter()
    ex = models.build(recipe, device=device, seed=seed + 100, env_id=env_id, debug_use_ground_truth=True)
    ex.trainer.train(max(ex.trainer.gen_train_timesteps, expert_timesteps))
    th.cuda.synchronize()
    t_expert = time.perf_counter() - t0
    r_exp, _ = ex.trainer.device_evaluate(n_eval, deterministic=True, seed=10_000 + seed)
    expert = float(np.mean(r_exp))
    demos = ex.trainer.device_demonstrations(n_demo_timesteps, deterministic=False, seed=20_000 + seed)
    demo_return = None
    del ex
    rand = random_return(env_id, n_eval, seed)
    b = models.build(recipe, device=device, seed=seed, env_id=env_id, demonstrations=demos)
    tr = b.trainer
    last: Dict[str, List[float]] = {}

    def score() -> float:
        r, _ = tr.device_evaluate(n_eval, deterministic=True, seed=10_000 + seed)
        last["returns"] = list(r)
        return float(np.mean(r))

    r0 = score()
    returns_before = last["returns"]
    curve: List[Dict[str, float]] = [dict(timesteps=0, ret=r0, norm=normalized_score(r0, rand, expert))]
    step = max(tr.gen_train_timesteps, int(eval_every or total_timesteps) // tr.gen_train_timesteps * tr.gen_train_timesteps)
    done, t_train = 0, 0.0
    while done < total_timesteps:
        k = max(tr.gen_train_timesteps, min(step, total_timesteps - done) // tr.gen_train_timesteps * tr.gen_train_timesteps)
        t1 = time.perf_counter()
        tr.train(k)
        th.cuda.synchronize()
        t_train += time.perf_counter() - t1
        done += k
        r = score()
        curve.append(dict(timesteps=done, ret=r, norm=normalized_score(r, rand, expert)))
        if verbose:
            print(f"{algo}/{env} seed {seed}: {done} steps: return {r:.1f} (normalised {curve[-1]['norm']:.3f})", flush=True)
    return dict(algo=algo, env=env_id, mode="expert", seed=seed, expert_return=expert, expert_timesteps=expert_timesteps,
                expert_train_s=round(t_expert, 3), random_return=rand, learner_return_before=r0,
                learner_return=curve[-1]["ret"], normalized_score=curve[-1]["norm"], curve=curve, total_timesteps=done,
                train_s=round(t_train, 3), n_eval_episodes=n_eval, n_demo_transitions=len(demos.acts),
                demo_return=demo_return, returns_before=returns_before, returns_after=last["returns"])


def main(argv: Optional[List[str]] = None) -> int:
    """``python -m imitation_amd.testing.imitation_quality expert ...``: fill the expert cache of
    :func:`expert_demonstrations` in a process of its own (``bench.py`` runs this before it touches
    the GPU, so its timed process starts as clean as a cached run). Single GPU, no process group."""
    import argparse

    p = argparse.ArgumentParser(prog="imitation_quality")
    p.add_argument("cmd", choices=["expert"])
    p.add_argument("--recipe", default="gail_halfcheetah")
    p.add_argument("--env", default="HalfCheetah-v4")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--expert-steps", type=int, default=5_000_000)
    p.add_argument("--n-demo", type=int, default=50_000)
    p.add_argument("--n-eval", type=int, default=50)
    p.add_argument("--rank", type=int, default=0)
    p.add_argument("--n-envs", type=int, default=8)
    p.add_argument("--device", default="cuda")
    p.add_argument("--cache-dir", required=True)
    a = p.parse_args(argv)
    dev = th.device(a.device)
    if dev.type == "cuda":
        th.cuda.set_device(dev)
    th.manual_seed(a.seed)
    np.random.seed(a.seed)
    r = expert_demonstrations(a.recipe, a.env, seed=a.seed, expert_timesteps=a.expert_steps, n_demo_timesteps=a.n_demo,
                              n_eval=a.n_eval, device=dev, rank=a.rank, world=1, n_envs=a.n_envs, cache_dir=a.cache_dir)
    print(f"expert {a.recipe}/{a.env} rank {a.rank}: return {r['expert_return']:.1f} (random {r['random_return']:.1f}), "
          f"{len(r['demos'].acts)} demo transitions, cached={r['cached']}, train {r['expert_train_s']:.2f} s", flush=True)
    return 0


if __name__ == "__main__":
    import sys

    sys.exit(main())

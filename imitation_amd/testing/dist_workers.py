"""Rank bodies for the multi-process data-parallel tests (importable for spawn)."""

from __future__ import annotations

import numpy as np
import torch as th


def moments_worker(rank, world, data):
    from imitation_amd.parallel import dist as pdist

    x = th.as_tensor(data[rank])
    mean, var, count = pdist.allreduce_moments(x)
    return mean.numpy(), var.numpy(), count


def running_norm_worker(rank, world, data):
    from imitation_amd.util import networks

    norm = networks.RunningNorm(data[0][0].shape[1])
    for chunk in data[rank]:
        norm.update_stats(th.as_tensor(chunk))
    return norm.running_mean.numpy(), norm.running_var.numpy(), int(norm.count.item())


def grad_bucket_worker(rank, world):
    from imitation_amd.parallel import dist as pdist

    lin = th.nn.Linear(3, 2)
    pdist.broadcast_module(lin)
    bucket = pdist.GradBucket(lin.parameters())
    x = th.full((4, 3), float(rank + 1))
    lin(x).sum().backward()
    bucket.allreduce()
    return [p.grad.clone().numpy() for p in lin.parameters()], [p.detach().clone().numpy() for p in lin.parameters()]


def gather_rows_worker(rank, world):
    from imitation_amd.parallel import dist as pdist

    x = th.arange((rank + 1) * 2, dtype=th.float32).reshape(rank + 1, 2) + 100 * rank
    return pdist.all_gather_rows(x).numpy()


def bc_dp_worker(rank, world, obs, acts, batch, n_steps, seed):
    """Each rank sees its contiguous shard of every global batch (global batch = world * batch)."""
    from imitation_amd.algorithms import bc
    from imitation_amd.envs import spaces

    th.manual_seed(seed + rank)  # different init per rank: broadcast_module must fix it
    obs_space = spaces.Box(-np.inf, np.inf, (obs.shape[1],))
    act_space = spaces.Discrete(int(acts.max()) + 1)
    data = []
    gb = world * batch
    for s in range(n_steps):
        lo = s * gb + rank * batch
        data.append({"obs": th.as_tensor(obs[lo:lo + batch]), "acts": th.as_tensor(acts[lo:lo + batch])})
    trainer = bc.BC(observation_space=obs_space, action_space=act_space, rng=np.random.default_rng(0), demonstrations=data,
                    batch_size=batch, optimizer_kwargs=dict(lr=1e-2))
    trainer.train(n_batches=n_steps, log_interval=10**9)
    return [p.detach().numpy().copy() for p in trainer.policy.parameters()]


def ppo_dp_worker(rank, world, seed):
    """Two PPO ranks on differently-seeded envs stay bit-identical in parameters."""
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import util

    venv = util.make_vec_env("CartPole-v1", rng=np.random.default_rng(seed + rank), n_envs=2)
    model = PPO("MlpPolicy", venv, n_steps=32, batch_size=32, n_epochs=2, seed=seed + rank, device="cpu",
                policy_kwargs=dict(net_arch=[16]))
    model.learn(128)
    return [p.detach().numpy().copy() for p in model.policy.parameters()]

"""Rank bodies for the multi-process data-parallel tests (importable for spawn)."""

from __future__ import annotations

import numpy as np
import torch as th

from imitation_amd.utils import graphs


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


def device_gail_dp_worker(rank, world, seed, batch):
    """Replicated data-parallel device PPO update on ``cuda:0`` (ranks share the card over gloo).

    Returns this rank's updated policy parameters and, on rank 0, the max deviation from
    the fp32 PyTorch reference run on the all-gathered rows with the global minibatch."""
    import os

    from imitation_amd.data import rollout
    from imitation_amd.engine.gail import DeviceGAIL
    from imitation_amd.policies.base import FeedForward32Policy, NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicRewardNet, NormalizedRewardNet
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.testing.ppo_reference import torch_ppo_reference
    from imitation_amd.util import logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    th.manual_seed(seed + rank)
    np.random.seed(seed + rank)
    rng = np.random.default_rng(seed + rank)
    venv = make_vec_env("seals/HalfCheetah-v1", rng=rng, n_envs=4)
    demo_env = make_vec_env("seals/HalfCheetah-v1", rng=np.random.default_rng(7), n_envs=4)
    demos = rollout.flatten_trajectories(rollout.generate_trajectories(None, demo_env, rollout.make_min_timesteps(512), rng=rng))
    gen = PPO(FeedForward32Policy, venv, n_steps=32, batch_size=batch, n_epochs=2, device="cuda", seed=seed,
              ent_coef=0.01, policy_kwargs=dict(features_extractor_class=NormalizeFeaturesExtractor))
    rn = NormalizedRewardNet(BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm), RunningNorm)
    tr = DeviceGAIL(demonstrations=demos, demo_batch_size=128, venv=venv, gen_algo=gen, reward_net=rn,
                    n_disc_updates_per_round=1, custom_logger=logger.configure(f"/tmp/ia_dp_dev_{rank}", format_strs=[]))
    assert tr._dp_replicated, "replicated DP path not selected"
    tr._rollout()
    pol = gen.policy
    norm = pol.features_extractor.normalize
    p0 = [p.detach().clone() for p in pol.parameters()]
    n0 = (norm.running_mean.clone(), norm.running_var.clone(), norm.count.clone())
    perm_round = tr._perm_round
    tr._ppo_update()
    th.cuda.synchronize()
    out = {"params": [p.detach().cpu().numpy().copy() for p in pol.parameters()],
           "norm": (norm.running_mean.cpu().numpy().copy(), norm.running_var.cpu().numpy().copy())}
    if rank == 0:
        gl = tr._dp_global
        D, Aw = tr._dp_cols
        rows_g = gl.shape[0]
        tr._perm_round = perm_round  # replay the update's minibatch orders
        perm = tr._epoch_perms(rows_g, tr._dp_perm_seed).long()
        p_dev = [p.detach().clone() for p in pol.parameters()]
        with th.no_grad():
            for p, q in zip(pol.parameters(), p0):
                p.copy_(q)
            norm.running_mean.copy_(n0[0]); norm.running_var.copy_(n0[1]); norm.count.copy_(n0[2])
        from imitation_amd.parallel import dist as pdist

        os.environ["IMITATION_AMD_FUSED"] = "0"
        try:
            with pdist.no_norm_sync():  # rank-local reference: no collectives
                torch_ppo_reference(gen, gl[:, :D], gl[:, D:D + Aw], gl[:, D + Aw], gl[:, D + Aw + 1], gl[:, D + Aw + 2],
                                    perm, clip=float(gen.clip_range(1.0)), lr=float(gen.lr_schedule(1.0)),
                                    batch=batch * world)
        finally:
            os.environ.pop("IMITATION_AMD_FUSED", None)
        out["max_dev"] = max(float((q.detach() - r).abs().max()) for q, r in zip(pol.parameters(), p_dev))
        out["max_ref"] = max(float(q.detach().abs().max()) for q in pol.parameters())
    return out


def _pref_dataset(P: int, L: int, seed: int):
    from imitation_amd.algorithms import preference_comparisons as pc
    from imitation_amd.data import types

    rng = np.random.default_rng(seed)

    def frag():
        return types.TrajectoryWithRew(obs=rng.standard_normal((L + 1, 5)).astype(np.float32),
                                       acts=rng.standard_normal((L, 2)).astype(np.float32), infos=None, terminal=False,
                                       rews=rng.standard_normal(L).astype(np.float32))

    ds = pc.PreferenceDataset()
    pairs = [(frag(), frag()) for _ in range(P)]
    ds.push(pairs, rng.uniform(0, 1, P).astype(np.float32))
    return ds


def pref_reward_dp_worker(rank, world, P, L, mb, epochs, seed, device="cpu", report=False):
    """BasicRewardTrainer on a replicated preference dataset; returns the trained parameters
    (and with ``report`` whether the minibatch ran as a HIP-graph replay)."""
    import torch as th

    from imitation_amd.algorithms import preference_comparisons as pc
    from imitation_amd.envs import spaces
    from imitation_amd.rewards.reward_nets import BasicRewardNet
    from imitation_amd.util import logger
    from imitation_amd.util.networks import RunningNorm

    th.manual_seed(seed)
    net = BasicRewardNet(spaces.Box(-1, 1, (5,)), spaces.Box(-1, 1, (2,)), normalize_input_layer=RunningNorm).to(device)
    tr = pc.BasicRewardTrainer(pc.PreferenceModel(net), pc.CrossEntropyRewardLoss(), rng=np.random.default_rng(seed),
                               batch_size=mb, epochs=epochs, lr=1e-2,
                               custom_logger=logger.configure(f"/tmp/ia_pref_dp_{rank}", format_strs=[]))
    ds = _pref_dataset(P, L, seed)
    assert tr._fast_path_ok(ds)
    tr.train(ds)
    norm = net.mlp.normalize_input if hasattr(net.mlp, "normalize_input") else None
    out = [p.detach().cpu().numpy().copy() for p in net.parameters()]
    out += [b.detach().cpu().numpy().copy() for b in net.buffers()]
    if report:
        g = getattr(tr, "_mb_graph", None)
        return out, (0 if g is None else len(g.graphs))
    return out


def pref_gather_worker(rank, world, seed):
    """PreferenceComparisons under DP: every replica pushes the same all-gathered pairs."""
    from imitation_amd.algorithms import preference_comparisons as pc

    rng = np.random.default_rng(seed + rank)
    ds = _pref_dataset(3 + rank, 4, seed + rank)
    frags, prefs = pc._all_gather_pairs(list(zip(ds.fragments1, ds.fragments2)), ds.preferences)
    return [f[0].obs.sum() for f in frags], prefs.tolist()


def dagger_dp_worker(rank, world, scratch, seed):
    """SimpleDAggerTrainer under DP (host collector, gloo): per-rank scratch trees, the
    all-gathered demo union, identical BC replicas."""
    import os

    import torch as th

    from imitation_amd.algorithms import bc, dagger
    from imitation_amd.policies.base import ZeroPolicy
    from imitation_amd.util import logger
    from imitation_amd.util.util import make_vec_env

    th.manual_seed(seed)
    venv = make_vec_env("seals/CartPole-v0", rng=np.random.default_rng(seed + rank), n_envs=2)
    log = logger.configure(os.path.join(scratch, f"log{rank}"), format_strs=[])
    bct = bc.BC(observation_space=venv.observation_space, action_space=venv.action_space,
                rng=np.random.default_rng(seed + rank), batch_size=16, custom_logger=log)
    expert = ZeroPolicy(venv.observation_space, venv.action_space)
    tr = dagger.SimpleDAggerTrainer(venv=venv, scratch_dir=scratch, expert_policy=expert, rng=np.random.default_rng(seed + rank),
                                    bc_trainer=bct, custom_logger=log)
    tr.train(1000 * world, rollout_round_min_episodes=1, rollout_round_min_timesteps=500,
             bc_train_kwargs=dict(n_batches=8, progress_bar=False))
    local_files = sum(len(tr._store.files(r)) for r in range(tr.round_num))
    return dict(params=[p.detach().numpy().copy() for p in tr.policy.parameters()], round_num=tr.round_num,
                n_demos=len(tr._all_demos), local_files=local_files, scratch=str(tr.scratch_dir),
                last=tr.last_train_timesteps, local=tr.last_train_timesteps_local)


def oneshot_worker(rank, world, sizes, scale, seed):
    """One-shot all-reduce (``parallel/oneshot.py``) on ``cuda:0`` shared by the ranks:
    rank-seeded buckets reduced eagerly and from a captured HIP graph, plus the latency
    of a small bucket. Returns this rank's results for the parent to check."""
    import time

    from imitation_amd.parallel import oneshot

    c = oneshot.get()
    assert c is not None, "one-shot path not set up"
    dev = c.device
    out = {"eager": [], "graph": []}
    for n in sizes:
        x = th.as_tensor(np.random.default_rng(seed * 100 + rank * 7 + n).normal(size=n).astype(np.float32), device=dev)
        c.allreduce_(x, scale)
        out["eager"].append(x.cpu().numpy())
    # fp64 buckets (normaliser column sums) interleaved with fp32 ones: same slices, same
    # generation counters
    out["f64"] = []
    for n in sizes[:4]:
        x = th.as_tensor(np.random.default_rng(seed * 100 + rank * 7 + n + 5).normal(size=n), device=dev)
        c.allreduce_(x, scale)
        y = th.ones(n + 3, device=dev)
        c.allreduce_(y)
        out["f64"].append(x.cpu().numpy())
    # graph-captured launch: the generation counter lives on the device, so replays stay in step
    buf = th.zeros(sizes[-1], device=dev)
    side = th.cuda.Stream(device=dev)
    side.wait_stream(th.cuda.current_stream(dev))
    g = th.cuda.CUDAGraph()
    with th.cuda.stream(side):
        with graphs.capture(g, stream=side):
            c.allreduce_(buf, scale)
    th.cuda.current_stream(dev).wait_stream(side)
    for rep in range(3):
        buf.copy_(th.as_tensor(np.random.default_rng(seed * 100 + rank * 7 + 1000 + rep).normal(size=buf.numel()).astype(np.float32)))
        g.replay()
        out["graph"].append(buf.cpu().numpy())
    small = th.ones(1024, device=dev)
    for _ in range(20):
        c.allreduce_(small)
    th.cuda.synchronize(dev)
    from imitation_amd.parallel import dist as pdist

    pdist.barrier()
    iters = 200
    t0 = time.perf_counter()
    for _ in range(iters):
        c.allreduce_(small, 1.0 / world)
    th.cuda.synchronize(dev)
    out["us_per_call_4KB"] = (time.perf_counter() - t0) / iters * 1e6
    out["error"] = c.error()
    return out


def oneshot_timeout_worker(rank, world, timeout_s):
    """Rank 0 reduces while rank 1 never joins: the bounded wait must give up, write NaN and
    raise the error word instead of hanging the GPU."""
    from imitation_amd.parallel import oneshot

    c = oneshot.get()
    assert c is not None
    res = {}
    if rank == 0:
        c.timeout_s = timeout_s
        x = th.ones(4096 + 3, device=c.device)
        c.allreduce_(x)
        th.cuda.synchronize(c.device)
        res = {"all_nan": bool(th.isnan(x).all().item()), "error": c.error()}
        try:  # the training loops' once-per-round check raises and clears the word
            c.check("test", blocking=True)
            res["raised"] = False
        except RuntimeError:
            res["raised"] = True
        res["error_after"] = c.error()
    from imitation_amd.parallel import dist as pdist

    pdist.barrier()
    return res


def gail_round_worker(rank, world, seed):
    """One fused-discriminator DeviceGAIL round on ``cuda:0`` shared by the ranks (gloo group);
    returns the reward-net and policy parameters and how many one-shot all-reduces ran."""
    from imitation_amd.data import rollout
    from imitation_amd.engine.gail import DeviceGAIL
    from imitation_amd.parallel import oneshot
    from imitation_amd.policies.base import FeedForward32Policy, NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicRewardNet, NormalizedRewardNet
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    th.manual_seed(seed + rank)
    np.random.seed(seed + rank)
    rng = np.random.default_rng(seed + rank)
    venv = make_vec_env("seals/HalfCheetah-v1", rng=rng, n_envs=4)
    demo_env = make_vec_env("seals/HalfCheetah-v1", rng=np.random.default_rng(7), n_envs=4)
    demo_env.action_space.seed(11 + rank)  # random-policy demos: reproducible across runs
    demos = rollout.flatten_trajectories(rollout.generate_trajectories(None, demo_env, rollout.make_min_timesteps(512), rng=rng))
    gen = PPO(FeedForward32Policy, venv, n_steps=32, batch_size=64, n_epochs=2, device="cuda", seed=seed,
              ent_coef=0.01, policy_kwargs=dict(features_extractor_class=NormalizeFeaturesExtractor))
    rn = NormalizedRewardNet(BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm), RunningNorm)
    tr = DeviceGAIL(demonstrations=demos, demo_batch_size=128, venv=venv, gen_algo=gen, reward_net=rn,
                    n_disc_updates_per_round=2, custom_logger=logger.configure(f"/tmp/ia_dp_round_{rank}", format_strs=[]))
    tr.train(tr.gen_train_timesteps)
    th.cuda.synchronize()
    c = oneshot._COMM
    return {"reward": [p.detach().cpu().numpy().copy() for p in rn.parameters()],
            "policy": [p.detach().cpu().numpy().copy() for p in gen.policy.parameters()],
            "oneshot_calls": 0 if c is None else c.calls}


def airl_round_worker(rank, world, seed, rounds=1):
    """One DeviceAIRL round (shaped reward net) on ``cuda:0`` shared by the ranks; reports
    whether the discriminator update ran fused (airl_disc.hip) or as a HIP-graph replay of
    the generic autograd update (``IMITATION_AMD_AIRL_FUSED=0``)."""
    from imitation_amd.data import rollout
    from imitation_amd.engine.airl import DeviceAIRL
    from imitation_amd.parallel import oneshot
    from imitation_amd.policies.base import NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicShapedRewardNet, NormalizedRewardNet
    from imitation_amd.rl.policies import ActorCriticPolicy
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    th.manual_seed(seed + rank)
    np.random.seed(seed + rank)
    rng = np.random.default_rng(seed + rank)
    venv = make_vec_env("seals/Hopper-v1", rng=rng, n_envs=4)
    demo_env = make_vec_env("seals/Hopper-v1", rng=np.random.default_rng(7), n_envs=4)
    demo_env.action_space.seed(7 + rank)
    demos = rollout.flatten_trajectories(rollout.generate_trajectories(None, demo_env, rollout.make_min_timesteps(1024), rng=rng))
    gen = PPO(ActorCriticPolicy, venv, n_steps=64, batch_size=64, n_epochs=2, device="cuda", seed=seed,
              policy_kwargs=dict(net_arch=dict(pi=[64, 64], vf=[64, 64]), activation_fn=th.nn.ReLU,
                                 features_extractor_class=NormalizeFeaturesExtractor))
    rn = NormalizedRewardNet(BasicShapedRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm),
                             RunningNorm)
    tr = DeviceAIRL(demonstrations=demos, demo_batch_size=256, venv=venv, gen_algo=gen, reward_net=rn,
                    n_disc_updates_per_round=3, custom_logger=logger.configure(f"/tmp/ia_dp_airl_{rank}", format_strs=[]))
    graphed = tr._graphed_disc_ok()
    tr.train(rounds * tr.gen_train_timesteps)
    th.cuda.synchronize()
    c = oneshot._COMM
    g = getattr(tr, "_disc_graph", None)
    return {"reward": [p.detach().cpu().numpy().copy() for p in rn.parameters()],
            "policy": [p.detach().cpu().numpy().copy() for p in gen.policy.parameters()],
            "split": bool(getattr(tr, "_disc_split", False)),
            "norm": [b.detach().cpu().numpy().copy() for b in rn.buffers()],
            "graphed": graphed, "replays": 0 if g is None else g.n_replays,
            "fused": bool(getattr(tr, "_fused_disc", False)),
            "oneshot_calls": 0 if c is None else c.calls}


def oneshot_cpu_worker(rank, world):
    """On a CPU gloo group the one-shot path stays off (no device to map) and every
    collective keeps torch.distributed semantics."""
    from imitation_amd.parallel import dist as pdist
    from imitation_amd.parallel import oneshot

    t = th.full((5,), float(rank + 1))
    pdist.allreduce_sum_(t)
    return {"comm": oneshot.get() is not None, "active": pdist.oneshot_active(),
            "moments_device": pdist.allreduce_moments_device(th.ones(3, 2)) is not None, "sum": t.tolist()}


def oneshot_stress_worker(rank, world, iters, seed):
    """Uneven arrival: every rank runs a random amount of GPU work (and host sleep) before each
    one-shot reduction of a fresh rank-dependent bucket of random size; returns the max error
    of every reduction against the closed-form sum (checked over every word)."""
    import time

    from imitation_amd.parallel import oneshot

    c = oneshot.get()
    assert c is not None
    dev = c.device
    rng = np.random.default_rng(seed)  # same size sequence on every rank
    local = np.random.default_rng(seed * 31 + rank)  # rank-local load pattern
    a = th.randn(512, 512, device=dev)
    errs = []
    for it in range(iters):
        n = int(rng.integers(1, 70000))
        for _ in range(int(local.integers(0, 6))):
            a = th.tanh(a @ a * 1e-3)
        if local.random() < 0.2:
            time.sleep(float(local.random()) * 2e-3)
        base = th.arange(n, device=dev, dtype=th.float32) % 97
        x = base * float(rank + 1) + float(it)
        c.allreduce_(x)
        exp = base * float(world * (world + 1) / 2) + float(it * world)
        errs.append((x - exp).abs().max())
    th.cuda.synchronize(dev)
    return {"max_err": float(th.stack(errs).max()), "error": c.error()}


def oneshot_block_change_worker(rank, world, reps, seed):
    """Back-to-back one-shot reductions whose block counts change call to call (1, 2, 4, 1
    blocks), captured in ONE HIP graph and replayed with rank-skewed GPU load in front of each
    replay; every word of every bucket is checked against the rank-order sum (the
    staging slice of a block must not depend on the call's size)."""
    from imitation_amd.parallel import oneshot

    c = oneshot.get()
    assert c is not None
    dev = c.device
    per = c.block_floats()
    sizes = [per // 2 + 3, per + per // 2, 3 * per + 5, 7]
    blocks = [c.blocks(n) for n in sizes]
    bufs = [th.zeros(n, device=dev) for n in sizes]
    side = th.cuda.Stream(device=dev)
    side.wait_stream(th.cuda.current_stream(dev))
    g = th.cuda.CUDAGraph()
    with th.cuda.stream(side):
        with graphs.capture(g, stream=side):
            for b in bufs:
                c.allreduce_(b)
    th.cuda.current_stream(dev).wait_stream(side)
    local = np.random.default_rng(seed * 13 + rank)
    a = th.randn(256, 256, device=dev)
    bad = 0
    for rep in range(reps):
        for i, b in enumerate(bufs):
            b.copy_(th.arange(b.numel(), device=dev, dtype=th.float32) % 89 * float(rank + 1) + float(rep + i))
        for _ in range(int(local.integers(0, 4))):
            a = th.tanh(a @ a * 1e-3)
        g.replay()
        for i, b in enumerate(bufs):
            exp = th.arange(b.numel(), device=dev, dtype=th.float32) % 89 * float(world * (world + 1) / 2) + float((rep + i) * world)
            bad += int((b != exp).sum().item())
    th.cuda.synchronize(dev)
    return {"bad_words": bad, "blocks": blocks, "error": c.error()}


def pref_device_iter_worker(rank, world, seed):
    """Full preference-comparisons iterations (DeviceAgentTrainer agent on ``cuda:0`` shared by
    the ranks, replicated-DP PPO, all-gathered pairs, DP reward trainer) from the
    ``preference_walker2d`` recipe at a reduced size; returns what the parent compares:
    replica parameters (must be bit-identical) and each rank's env state (must differ)."""
    import torch as th

    from imitation_amd import models

    dev = th.device("cuda", 0)
    th.manual_seed(seed + rank)
    np.random.seed(seed + rank)
    b = models.build("preference_walker2d", device=dev, seed=seed, rank=rank, n_envs=4, n_steps=64,
                     fragment_length=16, total_timesteps=2 * 4 * 64 * 2, num_iterations=2, engine="device")
    tr = b.trainer
    gen = tr.trajectory_generator
    assert type(gen).__name__ == "DeviceAgentTrainer", type(gen)
    tr.train(2 * 4 * 64 * 2, total_comparisons=24)
    th.cuda.synchronize()
    return {"reward": [p.detach().cpu().numpy().copy() for p in tr.model.parameters()],
            "policy": [p.detach().cpu().numpy().copy() for p in b.extras["agent"].policy.parameters()],
            "n_pairs": len(tr.dataset), "env_state": gen.state.detach().cpu().numpy().copy(),
            "cur_obs": gen.cur_obs.detach().cpu().numpy().copy()}


def dagger_device_round_worker(rank, world, seed, scratch):
    """DAgger rounds with the device collector (Pong-shaped frames rendered on ``cuda:0``,
    shared by the ranks) from the ``dagger_pong`` recipe: BC replicas must stay bit-identical,
    each rank's env must follow its own seed."""
    import os

    import torch as th

    from imitation_amd import models

    dev = th.device("cuda", 0)
    th.manual_seed(seed + rank)
    np.random.seed(seed + rank)
    b = models.build("dagger_pong", device=dev, seed=seed, rank=rank, n_envs=2, batch_size=32,
                     scratch_dir=os.path.join(scratch, "dagger"))
    tr = b.trainer
    assert tr.collector_kind == "device", tr.collector_kind
    tr.train(256 * world, rollout_round_min_episodes=1, rollout_round_min_timesteps=256,
             bc_train_kwargs=dict(n_batches=4, progress_bar=False, log_interval=10**9))
    th.cuda.synchronize()
    col = tr._device_collector
    dp_step = getattr(tr.bc_trainer, "_dp_step", None)
    run = getattr(tr.bc_trainer, "_epoch_run", None)
    return {"policy": [p.detach().cpu().numpy().copy() for p in tr.policy.parameters()],
            "env_state": col.state.detach().cpu().numpy().copy(), "round_num": tr.round_num,
            "local": tr.last_train_timesteps_local, "dp_fused_replays": dp_step.n_replays if dp_step else 0,
            "dp_epoch_runner": run is not None and run._comm is not None}


def oneshot_selftest_worker(rank, world, corrupt, mode="auto"):
    """``oneshot.adopt`` on a stand-in communicator (gloo on CPU) whose reduction is correct, or
    corrupted on rank 1 only (``corrupt``): returns (adopted?, reason, closed?) on every rank."""
    import torch
    import torch.distributed as tdist

    from imitation_amd.parallel import oneshot

    class FakeComm(oneshot.OneShotComm):
        def __init__(self):  # no IPC: the reduction is the process group's
            self.rank, self.world, self.device = rank, world, torch.device("cpu")
            self.stage_bytes, self.timeout_s = 1 << 16, 5.0
            self.local, self._opened, self.closed = None, [], False

        def allreduce_(self, t, scale=1.0):
            tdist.all_reduce(t)
            if corrupt == "value" and self.rank == 1:
                t.view(-1)[-1] += 1.0
            if corrupt == "ulp" and self.rank == 1:
                t.view(-1)[0] = torch.nextafter(t.view(-1)[0], torch.tensor(float("inf")))

        def error(self):
            return 0

        def close(self):
            self.closed = True

    comm = FakeComm()
    oneshot.DISABLED_REASON = None
    try:
        got = oneshot.adopt(comm, mode)
    except RuntimeError as e:
        return ("raised", str(e), comm.closed)
    return (got is comm, oneshot.DISABLED_REASON, comm.closed)


def oneshot_selftest_gpu_worker(rank, world):
    """The real communicator after ``dist.init`` (IMITATION_AMD_ONESHOT=1): adopted, and its
    start-up self-test (closed form + bitwise cross-check vs the process group) passes again."""
    from imitation_amd.parallel import oneshot

    c = oneshot._COMM
    rep = c.self_test_report() if c is not None else (False, "no communicator")
    return (c is not None, oneshot.DISABLED_REASON, rep)


def bc_dp_epoch_worker(rank, world, mode, n_epochs=2, n_rows=32 * 9 + 5, profile_dir=None):
    """Data-parallel BC on the fused NatureCNN step over a device aggregate (the DAgger-Pong learner),
    ``IMITATION_AMD_BC_EPOCH_GRAPH=mode``: "1" the graph-resident epoch runner (16-step graphs with
    the one-shot gradient all-reduce captured inside), "0" the per-minibatch ``_DPFusedStep``
    (graph, eager all-reduce, graph). Same frames on every rank, per-rank minibatch orders."""
    import os

    import torch as th

    os.environ["IMITATION_AMD_BC_EPOCH_GRAPH"] = mode
    from imitation_amd.algorithms import bc
    from imitation_amd.engine.dagger import DeviceDemoAggregate, DeviceTransitionsLoader
    from imitation_amd.envs.vec_env import native_spaces
    from imitation_amd.rl.policies import ActorCriticCnnPolicy
    from imitation_amd.util import logger as ilog

    dev = th.device("cuda", 0)
    obs_space, act_space = native_spaces("PongNoFrameskip-v4")
    g = th.Generator(device=dev).manual_seed(5)
    obs = th.randint(0, 256, (n_rows, 84, 84, 4), generator=g, device=dev, dtype=th.int64).to(th.uint8)
    acts = th.randint(0, int(act_space.n), (n_rows,), generator=g, device=dev)
    th.manual_seed(11)
    pol = ActorCriticCnnPolicy(obs_space, act_space, lambda _: th.finfo(th.float32).max).to(dev)
    agg = DeviceDemoAggregate(dev)
    agg.append(obs, acts, gather=False)
    log = ilog.configure(format_strs=[])
    recorded = []
    orig_dump = log.dump

    def dump(step=0):
        recorded.append((step, {k: v for k, v in log.name_to_value.items() if k.startswith("bc/")}))
        orig_dump(step)

    log.dump = dump
    trainer = bc.BC(observation_space=obs_space, action_space=act_space, rng=np.random.default_rng(rank), policy=pol,
                    batch_size=32, device=dev, custom_logger=log)
    trainer.set_demonstrations(DeviceTransitionsLoader(agg, 32, seed=3 + rank))
    trainer.train(n_epochs=n_epochs, log_interval=4, progress_bar=False)
    th.cuda.synchronize()
    run = getattr(trainer, "_epoch_run", None)
    f = trainer.optimizer._flat[0]
    return {"params": [p.detach().cpu().numpy().copy() for p in pol.parameters()], "m": f["m"].cpu().numpy().copy(),
            "v": f["v"].cpu().numpy().copy(), "recorded": recorded,
            "epoch_runner": run is not None and run._comm is not None,
            "dp_fused_replays": getattr(getattr(trainer, "_dp_step", None), "n_replays", 0)}

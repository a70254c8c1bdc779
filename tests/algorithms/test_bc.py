"""Behavioral cloning (reference: tests/algorithms/test_bc.py)."""

import numpy as np
import pytest
import torch as th

from imitation_amd.algorithms import bc
from imitation_amd.data import rollout, types
from imitation_amd.policies import base as policy_base
from imitation_amd.testing import reward_improvement
from imitation_amd.util import util


@pytest.fixture
def expert_transitions(cartpole_expert_trajectories):
    return rollout.flatten_trajectories(cartpole_expert_trajectories[:10])


@pytest.mark.parametrize("data_kind", ["transitions", "trajectories", "data_loader", "dict_iter"])
def test_bc_accepts_demonstration_kinds(data_kind, cartpole_venv, cartpole_expert_trajectories, expert_transitions, rng,
                                        custom_logger):
    if data_kind == "transitions":
        demos = expert_transitions
    elif data_kind == "trajectories":
        demos = cartpole_expert_trajectories[:3]
    elif data_kind == "data_loader":
        demos = th.utils.data.DataLoader(expert_transitions, batch_size=32, shuffle=True, drop_last=True,
                                         collate_fn=types.transitions_collate_fn)
    else:
        demos = [types.transitions_collate_fn([expert_transitions[i] for i in range(j, j + 32)]) for j in range(0, 320, 32)]
    trainer = bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space,
                    rng=rng, demonstrations=demos, batch_size=32, custom_logger=custom_logger)
    trainer.train(n_batches=5)


def test_bc_train_requires_exactly_one_duration(cartpole_venv, expert_transitions, rng):
    trainer = bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space,
                    rng=rng, demonstrations=expert_transitions, batch_size=32)
    with pytest.raises(ValueError):
        trainer.train(n_epochs=1, n_batches=1)
    with pytest.raises(ValueError):
        trainer.train()


def test_bc_improves_policy(cartpole_venv, cartpole_expert_trajectories, rng):
    """BC on CartPole expert data improves returns significantly (reference test_bc.py:200-232)."""
    trainer = bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space,
                    rng=rng, demonstrations=rollout.flatten_trajectories(cartpole_expert_trajectories), batch_size=64)
    before = rollout.rollout(trainer.policy, cartpole_venv, rollout.make_min_episodes(15), rng=rng, deterministic_policy=True)
    trainer.train(n_epochs=3)
    after = rollout.rollout(trainer.policy, cartpole_venv, rollout.make_min_episodes(15), rng=rng, deterministic_policy=True)
    old = [t.rews.sum() for t in before]
    new = [t.rews.sum() for t in after]
    assert reward_improvement.mean_reward_improved_by(old, new, 50)
    assert reward_improvement.is_significant_reward_improvement(old, new, p_value=0.05)


def test_gradient_accumulation_matches_large_batch(cartpole_venv, expert_transitions):
    """minibatch_size accumulation == one big batch (reference test_bc.py:235-283)."""
    batch_size, mini = 64, 16
    trainers = []
    for mb in (batch_size, mini):
        th.manual_seed(0)
        pol = policy_base.FeedForward32Policy(observation_space=cartpole_venv.observation_space,
                                              action_space=cartpole_venv.action_space,
                                              lr_schedule=lambda _: th.finfo(th.float32).max)
        trainers.append(bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space,
                              rng=np.random.default_rng(0), policy=pol, demonstrations=None, batch_size=batch_size,
                              minibatch_size=mb, optimizer_kwargs=dict(lr=1e-3)))
    # identical data stream for both
    data = [types.transitions_collate_fn([expert_transitions[i] for i in range(j, j + batch_size)])
            for j in range(0, 4 * batch_size, batch_size)]
    trainers[0].set_demonstrations(data)
    small = []
    for d in data:
        for k in range(0, batch_size, mini):
            small.append({key: (v[k:k + mini] if not isinstance(v, list) else v[k:k + mini]) for key, v in d.items()})
    trainers[1].set_demonstrations(small)
    trainers[0].train(n_batches=4)
    trainers[1].train(n_batches=4)
    for p1, p2 in zip(trainers[0].policy.parameters(), trainers[1].policy.parameters()):
        np.testing.assert_allclose(p1.detach().numpy(), p2.detach().numpy(), atol=1e-5, rtol=1e-4)


def test_bc_policy_save_load(tmp_path, cartpole_venv, expert_transitions, rng):
    trainer = bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space,
                    rng=rng, demonstrations=expert_transitions, batch_size=32)
    trainer.train(n_batches=3)
    path = tmp_path / "policy.pt"
    util.save_policy(trainer.policy, path) if hasattr(util, "save_policy") else trainer.save_policy(path)
    pol = bc.reconstruct_policy(str(path), device="cpu")
    obs = np.asarray(expert_transitions.obs[:20])
    a1, _ = trainer.policy.predict(obs, deterministic=True)
    a2, _ = pol.predict(obs, deterministic=True)
    np.testing.assert_array_equal(a1, a2)


def test_bc_loss_calculator_values():
    calc = bc.BehaviorCloningLossCalculator(ent_weight=1e-3, l2_weight=0.0)
    assert calc.ent_weight == 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("env_id", ["CartPole-v1", "PongNoFrameskip-v4"])
@pytest.mark.filterwarnings("error:The AccumulateGrad node's stream")
def test_bc_graph_replay_matches_eager(monkeypatch, env_id):
    """The HIP-graph BC step (utils/graphs.GraphedTrainStep) == the eager step: same
    parameters after several batches and the same logged metrics (both with the
    capturable Adam arithmetic)."""
    import torch as th

    from imitation_amd.algorithms import bc as bc_mod
    from imitation_amd.data import rollout
    from imitation_amd.util import logger as imit_logger
    from imitation_amd.util.util import make_vec_env

    venv = make_vec_env(env_id, rng=np.random.default_rng(0), n_envs=2)
    trajs = rollout.generate_trajectories(None, venv, rollout.make_min_timesteps(300), rng=np.random.default_rng(1))
    demos = rollout.flatten_trajectories(trajs)
    out = []
    for mode in ("0", "1"):
        monkeypatch.setenv("IMITATION_AMD_BC_GRAPH", mode)
        th.manual_seed(0)
        np.random.seed(0)  # the demo loader's shuffling seed comes from the global numpy RNG
        log = imit_logger.configure(format_strs=[])
        tr = bc_mod.BC(observation_space=venv.observation_space, action_space=venv.action_space,
                       rng=np.random.default_rng(2), demonstrations=demos, batch_size=32, device="cuda",
                       custom_logger=log)
        for g in tr.optimizer.param_groups:
            g["capturable"] = True
        tr.train(n_batches=6, log_interval=2, progress_bar=False)
        g = getattr(tr, "_graph_step", None)
        assert (g is not None and g.n_replays == 5) == (mode == "1")
        out.append([p.detach().clone() for p in tr.policy.parameters()])
    for a, b in zip(*out):
        th.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_multibc_trains_on_agent_concatenated_batches():
    """MultiBC (fork addition, reference bc.py:512-776): every minibatch is the agents' slices
    concatenated along the batch axis (bc.py:758-759) -- its loss equals BC's loss on that
    concatenation -- and training learns a per-agent rule shared by both agents."""
    import torch as th

    from imitation_amd.algorithms import bc
    from imitation_amd.data import types
    from imitation_amd.envs import spaces
    from imitation_amd.util import logger

    rng = np.random.default_rng(0)
    d, n_agents, N = 3, 2, 512
    obs = rng.standard_normal((N, d * n_agents)).astype(np.float32)
    acts = np.stack([(obs[:, d * i] > 0).astype(np.int64) for i in range(n_agents)], axis=1)  # action = sign of feature 0
    obs_over = lambda i, o: o[:, d * i: d * i + d]  # noqa: E731
    act_over = lambda i, a: a[:, i]  # noqa: E731
    demos = types.TransitionsMinimal(obs=obs, acts=acts, infos=np.array([{}] * N))
    th.manual_seed(0)
    trainer = bc.MultiBC(single_agent_observation_space=spaces.Box(-10, 10, (d,)), single_agent_action_space=spaces.Discrete(2),
                         observation_overide=obs_over, action_overide=act_over, num_agents=n_agents,
                         rng=np.random.default_rng(0), demonstrations=demos, batch_size=64,
                         optimizer_kwargs=dict(lr=3e-3), custom_logger=logger.configure(format_strs=[]))
    batch = {"obs": obs[:8], "acts": th.as_tensor(acts[:8])}
    o_cat, a_cat = trainer._prepare_batch(batch)
    assert o_cat.shape == (16, d) and a_cat.shape == (16,)
    np.testing.assert_array_equal(o_cat.numpy(), np.concatenate([obs[:8, :d], obs[:8, d:]]))
    np.testing.assert_array_equal(a_cat.numpy(), np.concatenate([acts[:8, 0], acts[:8, 1]]))
    m1 = trainer.loss_calculator(trainer.policy, o_cat, a_cat)
    m2 = trainer.loss_calculator(trainer.policy, th.as_tensor(np.concatenate([obs[:8, :d], obs[:8, d:]])),
                                 th.as_tensor(np.concatenate([acts[:8, 0], acts[:8, 1]])))
    th.testing.assert_close(m1.loss, m2.loss)
    trainer.train(n_epochs=15, progress_bar=False, log_interval=10**9)
    pred, _ = trainer.policy.predict(obs, deterministic=True)
    assert pred.shape == (N, n_agents)
    assert (pred == acts).mean() > 0.9


@pytest.mark.gpu
@pytest.mark.filterwarnings("error:The AccumulateGrad node's stream")
def test_multibc_homogeneous_policy_runs_on_wide_kernel():
    """The fork's MultiBC with its default HomogenousFeedForward32Policy ([256, 256, 128],
    reference policies/base.py:222-234): the agent-concatenated batch goes through the wide
    MFMA kernels (wlin.hip), the loss equals the fp32 torch loss on the same concatenation
    within bf16 tolerance, and a few training steps run on the kernel."""
    import torch as th

    from imitation_amd import ops
    from imitation_amd.algorithms import bc
    from imitation_amd.data import types
    from imitation_amd.envs import spaces
    from imitation_amd.ops import mlp as mlp_ops
    from imitation_amd.util import logger

    rng = np.random.default_rng(0)
    d, n_agents, N = 12, 4, 1024
    obs = rng.standard_normal((N, d * n_agents)).astype(np.float32)
    acts = np.stack([(obs[:, d * i] > 0).astype(np.int64) for i in range(n_agents)], axis=1)
    obs_over = lambda i, o: o[:, d * i: d * i + d]  # noqa: E731
    act_over = lambda i, a: a[:, i]  # noqa: E731
    demos = types.TransitionsMinimal(obs=obs, acts=acts, infos=np.array([{}] * N))
    th.manual_seed(0)
    trainer = bc.MultiBC(single_agent_observation_space=spaces.Box(-10, 10, (d,)), single_agent_action_space=spaces.Discrete(2),
                         observation_overide=obs_over, action_overide=act_over, num_agents=n_agents,
                         rng=np.random.default_rng(0), demonstrations=demos, batch_size=64, device="cuda",
                         optimizer_kwargs=dict(lr=1e-3), custom_logger=logger.configure(format_strs=[]))
    pol = mlp_ops.set_wide_bf16(trainer.policy)  # the bf16 wide path is opt-in
    plan = pol._fusion()
    assert plan, "homogeneous policy heads must be fused"
    dims = [pol.features_dim] + [l.out_features for l in plan["pi"]]
    assert dims[1:3] == [256, 256] and not mlp_ops.kernel_supports(dims) and mlp_ops.wide_supports(dims)
    batch = {"obs": obs[:64], "acts": th.as_tensor(acts[:64])}
    o_cat, a_cat = trainer._prepare_batch(batch)
    o_cat, a_cat = o_cat.cuda(), a_cat.cuda()
    loss_kernel = float(trainer.loss_calculator(pol, o_cat, a_cat).loss.detach())
    import os

    os.environ["IMITATION_AMD_FUSED"] = "0"
    try:
        loss_torch = float(trainer.loss_calculator(pol, o_cat, a_cat).loss.detach())
    finally:
        os.environ.pop("IMITATION_AMD_FUSED", None)
    assert abs(loss_kernel - loss_torch) < 2e-2 * max(1.0, abs(loss_torch))
    # the metrics (and the policy's distribution object, which training releases) are the
    # only holders of these eager graphs: nothing may keep one alive into the graph capture
    p0 = [p.detach().clone() for p in pol.parameters()]
    trainer.train(n_batches=20, progress_bar=False, log_interval=10**9)
    th.cuda.synchronize()
    assert all(th.isfinite(p).all() for p in pol.parameters())
    assert any(not th.equal(a, b) for a, b in zip(p0, pol.parameters()))


@pytest.mark.gpu
def test_fused_cnn_bc_step_matches_autograd():
    """ops/bc_cnn.FusedCnnBCStep (conv trunk + FC + fused head kernel, gradients straight into
    the FusedAdam bucket) == the autograd BC loss on the same kernels: metrics and every
    parameter's gradient."""
    import torch as th

    from imitation_amd.algorithms import bc as bc_mod
    from imitation_amd.envs.vec_env import native_spaces
    from imitation_amd.ops import bc_cnn
    from imitation_amd.ops import optim as optim_ops
    from imitation_amd.rl.policies import ActorCriticCnnPolicy

    obs_space, act_space = native_spaces("PongNoFrameskip-v4")
    th.manual_seed(0)
    pol = ActorCriticCnnPolicy(obs_space, act_space, lambda _: 1e-3).cuda()
    opt = optim_ops.FusedAdam(pol.parameters(), lr=1e-3)
    g = th.Generator().manual_seed(1)
    obs = th.randint(0, 256, (32, 84, 84, 4), generator=g, dtype=th.uint8).cuda()
    acts = th.randint(0, act_space.n, (32,), generator=g).cuda()
    step = bc_cnn.FusedCnnBCStep.maybe(pol, opt, obs, 1e-3, 0.0)
    assert step is not None
    opt.zero_grad()
    m = step(obs, acts).clone()
    fused = [p.grad.detach().clone() for p in pol.parameters()]
    opt.zero_grad()
    calc = bc_mod.BehaviorCloningLossCalculator(1e-3, 0.0)
    ref = calc(pol, obs, acts)
    ref.loss.backward()
    want = th.stack([ref.neglogp, ref.entropy, ref.ent_loss, ref.prob_true_act, ref.l2_norm, ref.l2_loss, ref.loss]).detach()
    th.testing.assert_close(m[:7], want, rtol=1e-4, atol=1e-5)
    for name_p, a in zip(pol.named_parameters(), fused):
        name, p = name_p
        b = p.grad if p.grad is not None else th.zeros_like(p)
        th.testing.assert_close(a, b, rtol=2e-3, atol=2e-5, msg=lambda s: f"{name}: {s}")
    assert float(fused[-2].abs().sum()) == 0.0  # value head: no gradient


def test_multibc_column_map_probe():
    """MultiBC overrides that select columns are recognised (and folded into the device gather);
    anything else (arithmetic, row-dependent selection) is not."""
    from imitation_amd.algorithms.bc import _column_map

    assert _column_map(lambda i, o: o[:, 3 * i: 3 * i + 3], 1, 12, th.float32) == ([3, 4, 5], False)
    assert _column_map(lambda i, a: a[:, i], 2, 4, th.int64) == ([2], True)
    assert _column_map(lambda i, o: o[:, [5, 1]], 0, 8, th.float32) == ([5, 1], False)
    assert _column_map(lambda i, o: o[:, :3] * 2.0, 0, 8, th.float32) is None
    assert _column_map(lambda i, o: o[:, :3] - o[:, 3:6], 0, 8, th.float32) is None
    assert _column_map(lambda i, o: o.flip(0)[:, :2], 0, 8, th.float32) is None
    assert _column_map(lambda i, o: (_ for _ in ()).throw(ValueError("no")), 0, 8, th.float32) is None
    # 1-D actions: only the identity folds (as a 1-D gather)
    assert _column_map(lambda i, a: a, 1, 1, th.int64, one_d=True) == ([0], True)
    assert _column_map(lambda i, a: a + i, 1, 1, th.int64, one_d=True) is None


def test_multibc_agent_gather_confirms_maps_on_real_rows():
    """a probe-accepted map must reproduce the override on real demo rows, shape
    included, else MultiBC falls back to the host loader; 1-D identity actions keep the
    reference's ``[n_agents * B]`` shape."""
    from imitation_amd.algorithms import bc
    from imitation_amd.data import types

    rng = np.random.default_rng(0)
    d, n_agents, N, B = 4, 3, 256, 32
    obs = rng.standard_normal((N, d * n_agents)).astype(np.float32)
    acts2 = rng.integers(0, 2, (N, n_agents))
    demos = types.TransitionsMinimal(obs=obs, acts=acts2, infos=np.array([{}] * N))
    sel = lambda i, o: o[:, d * i: d * i + d]  # noqa: E731
    ok = bc._AgentGatherLoader.maybe(demos, sel, lambda i, a: a[:, i], n_agents, B, "cpu", 0)
    assert isinstance(ok, bc._AgentGatherLoader)
    # agent-dependent in-range shift: the probe accepts it (columns shifted), real rows do not
    shift = lambda i, o: o[:, d * i: d * i + d] - i  # noqa: E731
    assert bc._column_map(shift, 1, d * n_agents, th.float32) is not None
    assert bc._AgentGatherLoader.maybe(demos, shift, lambda i, a: a[:, i], n_agents, B, "cpu", 0) is None
    # 1-D actions with an identity override: [n_agents * B] like th.cat of the overrides
    demos1 = types.TransitionsMinimal(obs=obs, acts=acts2[:, 0].copy(), infos=np.array([{}] * N))
    ld = bc._AgentGatherLoader.maybe(demos1, sel, lambda i, a: a, n_agents, B, "cpu", 0)
    assert ld is not None and ld.acts_ag.shape == (n_agents * N,) and ld.bufs[1].shape == (n_agents * B,)


@pytest.mark.gpu
def test_multibc_device_agent_gather_matches_cat_of_overrides():
    """The device agent-gather loader (one gather launch per batch) yields exactly the
    agent-concatenation the reference builds with observation_overide / action_overide + th.cat,
    for the rows of its permutation; training on it runs as graph replays."""
    from imitation_amd.algorithms import bc
    from imitation_amd.data import types
    from imitation_amd.envs import spaces
    from imitation_amd.ops import rl as rl_ops
    from imitation_amd.util import logger

    rng = np.random.default_rng(0)
    d, n_agents, N, B = 12, 4, 1024, 64
    obs = rng.standard_normal((N, d * n_agents)).astype(np.float32)
    acts = np.stack([(obs[:, d * i] > 0).astype(np.int64) for i in range(n_agents)], axis=1)
    obs_over = lambda i, o: o[:, d * i: d * i + d]  # noqa: E731
    act_over = lambda i, a: a[:, i]  # noqa: E731
    demos = types.TransitionsMinimal(obs=obs, acts=acts, infos=np.array([{}] * N))
    trainer = bc.MultiBC(single_agent_observation_space=spaces.Box(-10, 10, (d,)), single_agent_action_space=spaces.Discrete(2),
                         observation_overide=obs_over, action_overide=act_over, num_agents=n_agents,
                         rng=np.random.default_rng(0), demonstrations=demos, batch_size=B, device="cuda",
                         optimizer_kwargs=dict(lr=1e-3), custom_logger=logger.configure(format_strs=[]))
    p0 = [p.detach().clone() for p in trainer.policy.parameters()]
    trainer.train(n_batches=20, progress_bar=False, log_interval=10**9)
    th.cuda.synchronize()
    loader = trainer._demo_data_loader
    assert isinstance(loader, bc._AgentGatherLoader)
    assert trainer._graph_step.n_replays >= 18
    assert any(not th.equal(a, b) for a, b in zip(p0, trainer.policy.parameters()))
    # one more epoch by hand: batch b holds the overrides' concatenation of rows perm[b*B:(b+1)*B]
    ep = loader._epoch + 1
    perm = rl_ops.random_permutations(1, N, loader._seed * 1000003 + ep, "cuda")[0].long().cpu()
    it = iter(loader)
    for b in range(3):
        got = next(it)
        rows = perm[b * B:(b + 1) * B]
        o_all, a_all = th.as_tensor(obs)[rows], th.as_tensor(acts)[rows]
        want_o = th.cat([obs_over(i, o_all) for i in range(n_agents)])
        want_a = th.cat([act_over(i, a_all) for i in range(n_agents)])
        assert th.equal(got["obs"].cpu(), want_o) and th.equal(got["acts"].cpu(), want_a)


def test_weight_decay_in_optimizer_raises(cartpole_venv, rng):
    """weight_decay belongs in l2_weight (reference test_that_weight_decay_in_optimizer_raises_error)."""
    with pytest.raises(ValueError, match=".*weight_decay.*"):
        bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space,
              demonstrations=None, optimizer_kwargs=dict(weight_decay=1e-4), rng=rng, device="cpu")


@pytest.mark.parametrize("duration_args", [dict(n_epochs=1, n_batches=10), dict(), dict(n_epochs=None, n_batches=None)])
def test_wrong_training_duration_raises(cartpole_venv, expert_transitions, rng, duration_args):
    tr = bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space,
               demonstrations=expert_transitions, rng=rng, device="cpu")
    with pytest.raises(ValueError, match="exactly one.*n_epochs"):
        tr.train(**duration_args)


@pytest.mark.parametrize("no_yield_after_iter", [1, 2, 6])
def test_bc_raises_when_the_data_loader_runs_dry(cartpole_venv, expert_transitions, rng, no_yield_after_iter):
    """A loader that stops yielding makes train() fail instead of looping without updates
    (reference test_that_bc_raises_error_when_data_loader_is_empty)."""
    import dataclasses

    tr = bc.BC(observation_space=cartpole_venv.observation_space, action_space=cartpole_venv.action_space,
               demonstrations=expert_transitions, rng=rng, device="cpu")
    one_batch = dataclasses.asdict(expert_transitions[: tr.batch_size])

    class _Dries:
        def __init__(self):
            self.iters = 0

        def __iter__(self):
            if self.iters < no_yield_after_iter:
                yield one_batch
            self.iters += 1

    n_batches = 0

    def on_batch_end():
        nonlocal n_batches
        n_batches += 1

    tr.set_demonstrations(_Dries())
    with pytest.raises(AssertionError, match=".*no data.*"):
        tr.train(n_batches=20, on_batch_end=on_batch_end)
    assert n_batches == no_yield_after_iter


@pytest.mark.parametrize("fc_off,fc_n", [(77984, 1_605_632), (77985, 1_605_632), (77984, 1_605_630)])
def test_dp_bc_reduction_ranges_cover_the_bucket_once(fc_off, fc_n):
    """The graph-resident DP BC step reduces the FC weight gradient early (overlapping the conv
    backward) and the rest after it: the chunks cover the flat bucket exactly once, none exceeds
    the one-shot staging slot, and the early range is exactly the FC weight -- or, when it does not
    sit on 16-B boundaries, empty (a neighbour's gradient is not final at that point)."""
    import types

    flat = th.zeros(fc_off + fc_n + 1000)
    runner = bc._DeviceEpochRunner.__new__(bc._DeviceEpochRunner)
    runner.trainer = types.SimpleNamespace(optimizer=types.SimpleNamespace(flat_grads=[flat]))
    runner._comm = types.SimpleNamespace(stage_bytes=1 << 20)
    runner._f = types.SimpleNamespace(g_lin=[flat[fc_off : fc_off + fc_n]])
    fc, rest = runner._dp_ranges()
    base = flat.data_ptr()
    spans = sorted(((t.data_ptr() - base) // 4, t.numel()) for t in fc + rest)
    pos = 0
    for o, n in spans:
        assert o == pos and 0 < n <= (1 << 20) // 4
        pos += n
    assert pos == flat.numel()
    aligned = fc_off % 4 == 0 and (fc_off + fc_n) % 4 == 0
    if aligned:
        assert (fc[0].data_ptr() - base) // 4 == fc_off and sum(t.numel() for t in fc) == fc_n
        assert all((t.data_ptr() - base) % 16 == 0 for t in fc)
    else:
        assert fc == []

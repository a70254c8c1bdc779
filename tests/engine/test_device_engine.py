"""Device engine kernels vs host/PyTorch references (GPU only)."""

import os

import numpy as np
import pytest
import torch as th

gpu = pytest.mark.gpu


def _setup(env_id="seals/HalfCheetah-v1", n_envs=4, n_steps=32, batch=64, n_epochs=2, seed=0, discrete=False,
           net_arch=None, activation=None, init_seed=None):
    from imitation_amd.data import rollout
    from imitation_amd.engine.gail import DeviceGAIL
    from imitation_amd.policies.base import FeedForward32Policy, NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicRewardNet, NormalizedRewardNet
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    th.manual_seed(seed)
    np.random.seed(seed)
    rng = np.random.default_rng(seed)
    venv = make_vec_env(env_id, rng=rng, n_envs=n_envs)
    demo_env = make_vec_env(env_id, rng=np.random.default_rng(7), n_envs=4)
    demo_env.action_space.seed(7)  # random-policy demos: reproducible across setups
    demos = rollout.flatten_trajectories(rollout.generate_trajectories(None, demo_env, rollout.make_min_timesteps(1024), rng=rng))
    from imitation_amd.rl.policies import ActorCriticPolicy

    if init_seed is not None:  # same demonstrations, different initial weights / engine seeds
        th.manual_seed(init_seed)
        np.random.seed(init_seed)
        seed = init_seed
    pk = dict(features_extractor_class=NormalizeFeaturesExtractor)
    policy_cls = FeedForward32Policy
    if net_arch is not None:
        pk["net_arch"] = net_arch
        policy_cls = ActorCriticPolicy
    if activation is not None:
        pk["activation_fn"] = activation
    gen = PPO(policy_cls, venv, n_steps=n_steps, batch_size=batch, n_epochs=n_epochs, device="cuda", seed=seed,
              ent_coef=0.01, policy_kwargs=pk)
    rn = NormalizedRewardNet(BasicRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm), RunningNorm)
    tr = DeviceGAIL(demonstrations=demos, demo_batch_size=256, venv=venv, gen_algo=gen, reward_net=rn,
                    n_disc_updates_per_round=1, custom_logger=logger.configure("/tmp/ia_test_engine", format_strs=[]))
    return tr, venv, gen, rn


@gpu
def test_rollout_matches_host_env_policy_and_reward():
    from imitation_amd.envs.vec_env import NativeVecEnv

    tr, venv, gen, rn = _setup()
    nat = tr._native
    st0 = {k: v.copy() for k, v in nat.get_state().items()}
    obs0 = tr.cur_obs.cpu().numpy().copy()
    tr._rollout()
    th.cuda.synchronize()
    b = {k: v.cpu().numpy() for k, v in tr.buf.items()}
    T, N = b["dones"].shape
    # 1) env: replay the device's env actions on the host runtime
    nat.set_state(st0)
    obs = obs0
    for t in range(T):
        np.testing.assert_allclose(b["obs_buf"][t], obs, rtol=2e-3, atol=2e-3)
        o, r, d, infos = nat.step(b["act_env"][t])
        np.testing.assert_allclose(b["env_rew"][t], r, rtol=2e-3, atol=2e-3)
        assert (b["dones"][t] > 0.5).tolist() == d.tolist()
        nxt = np.stack([infos[i]["terminal_observation"] if d[i] else o[i] for i in range(N)])
        np.testing.assert_allclose(b["next_obs"][t], nxt, rtol=2e-3, atol=2e-3)
        obs = o
    # 2) policy log-prob / value of the stored samples (fp32 torch reference)
    os.environ["IMITATION_AMD_FUSED"] = "0"
    try:
        pol = gen.policy
        pol.set_training_mode(False)
        with th.no_grad():
            o_t = th.as_tensor(b["obs_buf"].reshape(T * N, -1), device="cuda")
            a_t = th.as_tensor(b["act_raw"].reshape(T * N, -1), device="cuda")
            v, lp, _ = pol.evaluate_actions(o_t, a_t)
        np.testing.assert_allclose(lp.cpu().numpy(), b["logp"].reshape(-1), rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(v.cpu().numpy().reshape(-1), b["values"].reshape(-1), rtol=1e-4, atol=1e-4)
        # 3) learned reward = GAIL reward_train on (s, a_env, s', done) (+ bootstrap only on truncation)
        rew = tr.reward_train.predict(b["obs_buf"].reshape(T * N, -1), b["act_env"].reshape(T * N, -1),
                                      b["next_obs"].reshape(T * N, -1), b["dones"].reshape(-1) > 0.5)
        np.testing.assert_allclose(rew, b["rewards"].reshape(-1), rtol=1e-4, atol=1e-4)
    finally:
        os.environ.pop("IMITATION_AMD_FUSED", None)


def _assert_adam_params_close(q_ref, q_dev, lr, n_steps, max_frac=0.01):
    """Device PPO parameters vs the fp32 torch replay. Every element must agree within
    rtol 2e-3 / atol 2e-4, except that up to ``max_frac`` of a tensor's elements may differ by
    up to Adam's largest possible displacement over the run (lr per step): an element whose
    gradient sits at the rounding-noise floor (a feature that normalises to ~0 on every row)
    takes a full-size Adam step of either sign, and the kernel's split-bf16 products (~2^-16
    relative error) and the reference's fp32 sums round that noise differently."""
    q_ref = q_ref.detach().float()
    err = (q_ref - q_dev.float()).abs()
    bad = err > 2e-4 + 2e-3 * q_ref.abs()
    assert float(err.max()) <= 2.0 * lr * n_steps + 1e-6, f"max |diff| {float(err.max()):.3g} beyond Adam's reach"
    assert int(bad.sum()) <= max(1, int(max_frac * err.numel())), (
        f"{int(bad.sum())} / {err.numel()} elements off (max {float(err.max()):.3g})")


def _torch_ppo_reference(gen, obs, acts, old_logp, adv, ret, perm, clip, lr, norm_count=None):
    from imitation_amd.testing.ppo_reference import torch_ppo_reference

    torch_ppo_reference(gen, obs, acts, old_logp, adv, ret, perm, clip, lr)


@gpu
@pytest.mark.parametrize("env_id,allow_rc,batch,gmax,net_arch,path", [
    # ":ns" = net split: one net per workgroup over 64-row chunks, 2 x G workgroups
    ("seals/HalfCheetah-v1", 1, 64, 0, None, "rc:g1x1x64:kt2:ns"),
    ("seals/HalfCheetah-v1", 0, 64, 0, None, "lds"),
    ("seals/CartPole-v0", 1, 64, 0, None, "rc:g1x1x64:kt2:ns"),
    ("seals/CartPole-v0", 0, 64, 0, None, "lds"),
    # cooperating workgroups (sc1 partial exchange) and multi-chunk workgroups
    ("seals/HalfCheetah-v1", 1, 128, 0, None, "rc:g2x1x64:kt2:ns"),
    ("seals/HalfCheetah-v1", 1, 128, 1, None, "rc:g1x2x64:kt2:ns"),
    ("seals/HalfCheetah-v1", 1, 256, 2, None, "rc:g2x2x64:kt2:ns"),
    ("seals/CartPole-v0", 1, 256, 0, None, "rc:g4x1x64:kt2:ns"),
    # 64-wide nets (AIRL-Hopper MlpPolicy [64, 64])
    ("seals/Hopper-v1", 1, 64, 0, dict(pi=[64, 64], vf=[64, 64]), "rc:g1x1x64:kt4:ns"),
    ("seals/Hopper-v1", 1, 256, 4, dict(pi=[64, 64], vf=[64, 64]), "rc:g4x1x64:kt4:ns"),
    # the shape-specialised 64-wide ReLU builds: AIRL-Hopper (minibatch 512, 8 row groups x
    # 2 nets, two-level exchange) and DRLHP-Walker
    ("seals/Hopper-v1", 1, 64, 0, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g1x1x64:kt4:ns"),
    ("seals/Hopper-v1", 1, 512, 0, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g8x1x64:kt4:ns"),
    ("seals/Walker2d-v1", 1, 128, 0, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g2x1x64:kt4:ns"),
    # G > 16 (AIRL's 4- / 8-rank DP minibatch): item-split first level from the LDS stash
    ("seals/Hopper-v1", 1, 2048, 0, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g32x1x64:kt4:ns"),
    ("seals/Hopper-v1", 1, 4096, 0, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g64x1x64:kt4:ns"),
    # both nets per workgroup (IMITATION_AMD_PPO_NETSPLIT=0): 64-row chunks for <= 32-wide
    # nets, 32-row chunks (2 row-tile waves per net) for 64-wide ones
    ("seals/HalfCheetah-v1", 1, 64, 0, "nons", "rc:g1x1x64:kt2"),
    ("seals/HalfCheetah-v1", 1, 256, 2, "nons", "rc:g2x2x64:kt2"),
    ("seals/CartPole-v0", 1, 256, 0, "nons", "rc:g4x1x64:kt2"),
    # [64, 64] Tanh, both nets per workgroup: the family build (obs dim <= 16)
    ("seals/Hopper-v1", 1, 64, 0, dict(pi=[64, 64], vf=[64, 64], nons=True), "rc:g2x1x32:kt4"),
    ("seals/HalfCheetah-v1", 1, 64, 0, dict(pi=[64, 64], vf=[64, 64], act="relu", nons=True), "rc:g2x1x32:kt4"),
    ("seals/Hopper-v1", 1, 512, 0, dict(pi=[64, 64], vf=[64, 64], act="relu", nons=True), "rc:g16x1x32:kt4"),
    ("seals/Walker2d-v1", 1, 128, 0, dict(pi=[64, 64], vf=[64, 64], act="relu", nons=True), "rc:g4x1x32:kt4"),
    # SB3's default MlpPolicy ([64, 64] Tanh; reference scripts/ingredients/rl.py:58-66) and
    # other [64, 64] nets on the spill-free family builds (obs dim <= 16 / <= 32, Tanh / ReLU,
    # Gaussian / categorical heads)
    ("seals/CartPole-v0", 1, 64, 0, dict(pi=[64, 64], vf=[64, 64]), "rc:g1x1x64:kt4:ns"),
    ("seals/CartPole-v0", 1, 128, 0, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g2x1x64:kt4:ns"),
    ("seals/HalfCheetah-v1", 1, 64, 0, dict(pi=[64, 64], vf=[64, 64]), "rc:g1x1x64:kt4:ns"),
    ("seals/HalfCheetah-v1", 1, 128, 0, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g2x1x64:kt4:ns"),
    ("Pendulum-v1", 1, 64, 0, dict(pi=[64, 64], vf=[64, 64]), "rc:g1x1x64:kt4:ns"),
    # minibatch of 32: the generic <= 32-wide both-nets build at one wave per SIMD
    ("Pendulum-v1", 1, 32, 0, None, "rc:g1x1x32:kt2"),
])
def test_ppo_kernel_matches_torch_reference(env_id, allow_rc, batch, gmax, net_arch, path, monkeypatch):
    act = None
    nons = net_arch == "nons" or (isinstance(net_arch, dict) and net_arch.get("nons"))
    if net_arch == "nons":
        net_arch = None
    if nons:
        monkeypatch.setenv("IMITATION_AMD_PPO_NETSPLIT", "0")
    if net_arch is not None:
        if net_arch.get("act") == "relu":
            act = th.nn.ReLU
        net_arch = {k: v for k, v in net_arch.items() if k not in ("act", "nons")}
    tr, venv, gen, rn = _setup(env_id=env_id, n_envs=max(8, batch // 64) if batch > 64 else 4, n_steps=64 if batch > 256 else 32,
                               batch=batch, n_epochs=2, net_arch=net_arch, activation=act)
    tr._ppo_static["allow_rc"] = allow_rc
    tr._ppo_static["rc_gmax"] = gmax
    assert tr._C.engine_ppo_path(tr._ppo_static) == path
    tr._rollout()
    pol = gen.policy
    norm = pol.features_extractor.normalize
    p0 = [p.detach().clone() for p in pol.parameters()]
    n0 = (norm.running_mean.clone(), norm.running_var.clone(), norm.count.clone())
    # device update with a known permutation
    rows = tr.T * tr.N
    perm_round = tr._perm_round
    tr._ppo_update()
    p_dev = [p.detach().clone() for p in pol.parameters()]
    mean_dev, var_dev = norm.running_mean.clone(), norm.running_var.clone()
    # reference: restore and replay with the same permutation
    tr._perm_round = perm_round
    perm = tr._epoch_perms(rows, tr._seed).long()
    with th.no_grad():
        for p, q in zip(pol.parameters(), p0):
            p.copy_(q)
        norm.running_mean.copy_(n0[0]); norm.running_var.copy_(n0[1]); norm.count.copy_(n0[2])
    from imitation_amd.ops import rl as rl_ops

    adv, ret = rl_ops.gae_reference(*(x.cpu() for x in (tr.buf["rewards"], tr.buf["values"], tr.buf["starts"], tr.buf["last_values"], tr.cur_start)), gen.gamma, gen.gae_lambda)
    os.environ["IMITATION_AMD_FUSED"] = "0"
    try:
        _torch_ppo_reference(gen, tr.buf["obs_buf"].reshape(rows, -1), tr.buf["act_raw"].reshape(rows, -1),
                             tr.buf["logp"].reshape(rows), adv.reshape(rows).cuda(), ret.reshape(rows).cuda(), perm,
                             clip=float(gen.clip_range(1.0)), lr=float(gen.lr_schedule(1.0)), norm_count=None)
    finally:
        os.environ.pop("IMITATION_AMD_FUSED", None)
    th.testing.assert_close(norm.running_mean, mean_dev, rtol=1e-5, atol=1e-5)
    th.testing.assert_close(norm.running_var, var_dev, rtol=1e-4, atol=1e-5)
    n_steps = gen.n_epochs * (rows // batch)
    for q_ref, q_dev in zip(pol.parameters(), p_dev):
        _assert_adam_params_close(q_ref, q_dev, float(gen.lr_schedule(1.0)), n_steps)


@gpu
@pytest.mark.parametrize("env_id,batch,n_envs,n_steps,net_arch,path", [
    # 32-wide GAIL plan at 8 cooperating row groups (the emulated W=8 minibatch)
    ("seals/HalfCheetah-v1", 512, 16, 64, None, "rc:g8x1x64:kt2:ns"),
    # 64-wide plans past 16 groups: the first exchange level goes through the LDS partial
    # stash, which borrows the activation images
    ("seals/Hopper-v1", 2048, 32, 64, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g32x1x64:kt4:ns"),
    ("seals/Hopper-v1", 4096, 64, 64, dict(pi=[64, 64], vf=[64, 64], act="relu"), "rc:g64x1x64:kt4:ns"),
])
def test_ppo_exchange_levels_are_bitwise_equal(env_id, batch, n_envs, n_steps, net_arch, path, monkeypatch):
    """The one-level (every workgroup sums all G partials) and two-level (reduce-then-share,
    with the LDS stash past 16 groups) partial exchanges add the same numbers in the same group
    order: the updates must be bitwise equal (a clobbered image or a mis-ordered sum breaks it)."""
    act = None
    if net_arch is not None:
        if net_arch.get("act") == "relu":
            act = th.nn.ReLU
        net_arch = {k: v for k, v in net_arch.items() if k != "act"}
    tr, venv, gen, rn = _setup(env_id=env_id, n_envs=n_envs, n_steps=n_steps, batch=batch, n_epochs=2,
                               net_arch=net_arch, activation=act)
    assert tr._C.engine_ppo_path(tr._ppo_static) == path
    tr._rollout()
    pol = gen.policy
    norm = tr.pol_norm
    dst = list(pol.parameters()) + [tr.exp_avg, tr.exp_avg_sq, tr.adam_step]
    if norm is not None:
        dst += [norm.running_mean, norm.running_var, norm.count, tr.norm_count]
    s0 = [t.detach().clone() for t in dst]
    pr = tr._perm_round
    res = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("IMITATION_AMD_PPO_XCHG2", mode)
        with th.no_grad():
            for d, v in zip(dst, s0):
                d.copy_(v)
        tr._perm_round = pr
        tr._ppo_update()
        th.cuda.synchronize()
        res[mode] = [t.detach().clone() for t in dst]
    for a, b in zip(res["0"], res["1"]):
        assert th.equal(a, b)
    tr.check_errors(blocking=True)


@gpu
def test_device_gail_rounds_run_and_learn_something():
    tr, venv, gen, rn = _setup(n_envs=8, n_steps=64, batch=64, n_epochs=2)
    before = [p.detach().clone() for p in gen.policy.parameters()]
    tr.train(3 * tr.gen_train_timesteps)
    th.cuda.synchronize()
    after = list(gen.policy.parameters())
    assert any(not th.equal(a, b) for a, b in zip(after, before))
    assert all(th.isfinite(p).all() for p in after)
    assert tr._gen_dev.size() > 0


@gpu
def test_disc_overlap_is_bitwise_the_serial_order(monkeypatch):
    """Discriminator updates on the side stream, concurrent with PPO, with the policy-norm
    merges deferred: parameters, Adam moments and both RunningNorms equal the serial run."""
    names = None
    runs = []
    modes = os.environ.get("IA_OVERLAP_MODES", "serial,deferred-same-stream,overlap").split(",")
    for mode in modes:
        monkeypatch.setenv("IMITATION_AMD_DISC_OVERLAP", "0" if mode == "serial" else "1")
        tr, venv, gen, rn = _setup(n_envs=8, n_steps=64, batch=64, n_epochs=2)
        if mode == "deferred-same-stream":
            tr._side_stream = th.cuda.current_stream()
        tr.n_disc_updates_per_round = 3
        tr.train(3 * tr.gen_train_timesteps)
        th.cuda.synchronize()
        pn = tr.pol_norm
        named = [(f"policy.{k}", v) for k, v in gen.policy.named_parameters()] + \
                [(f"reward.{k}", v) for k, v in rn.named_parameters()] + \
                [("pol_mean", pn.running_mean), ("pol_var", pn.running_var), ("pol_count", pn.count),
                 ("disc_m", tr._r_m), ("disc_v", tr._r_v), ("rew_mean", tr._rnorm.running_mean),
                 ("rew_count", tr._rnorm.count)]
        names = [k for k, _ in named]
        runs.append([v.detach().cpu().clone() for _, v in named])
        assert tr._disc_step == 9
    bad = []
    for i, k in enumerate(names):
        for j in range(1, len(modes)):
            if not th.equal(runs[0][i], runs[j][i]):
                bad.append((k, j, float((runs[0][i].double() - runs[j][i].double()).abs().max())))
    for b in bad:
        print("DIFF", *b)
    assert not bad


def _disc_reference(tr, e_idx, g_idx, mb_rows):
    """fp32 PyTorch reference of one fused discriminator minibatch: norm updates + BCE grads
    (MFMA operands emulated in bf16 so ReLU branches agree)."""
    import copy

    import torch.nn.functional as F

    from imitation_amd.engine.gail import _mlp_layers
    from imitation_amd.ops.mlp import tmlp_reference

    base = tr._reward_net.base
    norm, lins, hid, _ = _mlp_layers(base.mlp)
    rnorm = copy.deepcopy(norm)
    pnorm = copy.deepcopy(tr.pol_norm)
    ed, gd = tr._endless_expert_iterator.data, tr._gen_dev._arrays
    obs = th.cat([ed["obs"][e_idx], gd["obs"][g_idx]])
    acts = th.cat([ed["acts"][e_idx], gd["acts"][g_idx]])
    x = th.cat([obs, acts], 1)
    pnorm.update_stats(obs)
    rnorm.update_stats(x)
    Ws = [l.weight.detach().clone().requires_grad_() for l in lins]
    bs = [l.bias.detach().clone().requires_grad_() for l in lins]
    logits = tmlp_reference(x, Ws, bs, hid, 0, rnorm.running_mean, rnorm.running_var, rnorm.eps,
                            emulate_bf16_operands=True).reshape(-1)
    labels = th.cat([th.ones(mb_rows // 2), th.zeros(mb_rows // 2)]).cuda()
    loss = F.binary_cross_entropy_with_logits(logits, labels) * (tr.demo_minibatch_size / tr.demo_batch_size)
    loss.backward()
    grads = th.cat([t.grad.reshape(-1) for pair in zip(Ws, bs) for t in pair])
    return rnorm, pnorm, grads, logits.detach(), loss.detach()


@gpu
def test_fused_disc_grads_and_norms_match_reference():
    tr, venv, gen, rn = _setup(n_envs=8, n_steps=32, batch=64)
    assert tr._fused_disc, tr._fused_disc_why
    tr.train_gen()
    th.cuda.synchronize()
    B = tr.demo_batch_size
    e_idx = th.randperm(len(tr._endless_expert_iterator.data["obs"]), device="cuda")[:B].contiguous()
    g_idx = th.randint(0, tr._gen_dev.size(), (B,), device="cuda")
    rnorm, pnorm, grads_ref, logits, loss = _disc_reference(tr, e_idx, g_idx, 2 * B)
    plan = tr._disc_plan
    stats = th.zeros(8, device="cuda")
    plan.gather(0, e_idx, g_idx)
    plan.norm(0, 0, True, True)
    plan.fwd_bwd(0)
    plan.adam(1, 0, 0.0, 1.0, stats)
    th.cuda.synchronize()
    norm = tr._rnorm
    th.testing.assert_close(norm.running_mean, rnorm.running_mean, rtol=1e-5, atol=1e-5)
    th.testing.assert_close(norm.running_var, rnorm.running_var, rtol=1e-4, atol=1e-5)
    assert int(norm.count) == int(rnorm.count)
    th.testing.assert_close(tr.pol_norm.running_mean, pnorm.running_mean, rtol=1e-5, atol=1e-5)
    th.testing.assert_close(tr.pol_norm.running_var, pnorm.running_var, rtol=1e-4, atol=1e-5)
    assert int(tr.pol_norm.count) == int(pnorm.count)
    g = tr._disc_ws["grads"]
    # backward MFMA operands (dZ, H) are bf16 as well: elementwise error ~1e-3 of the largest grad
    th.testing.assert_close(g, grads_ref, rtol=2e-2, atol=2.5e-3 * float(grads_ref.abs().max()))
    assert float(th.nn.functional.cosine_similarity(g, grads_ref, dim=0)) > 0.9999
    s = tr._disc_stats_dict(stats.tolist())
    from imitation_amd.algorithms.adversarial.common import compute_train_stats

    labels = th.cat([th.ones(B), th.zeros(B)]).long().cuda()
    ref = compute_train_stats(logits, labels, loss)
    for k in ("disc_loss", "disc_entropy"):
        assert abs(s[k] - ref[k]) < 2e-3 * max(1.0, abs(ref[k])), (k, s[k], ref[k])
    for k in ("disc_acc", "disc_acc_expert", "disc_acc_gen", "disc_proportion_expert_pred"):
        assert abs(s[k] - ref[k]) < 0.02, (k, s[k], ref[k])  # a few near-zero logits may flip sign in bf16
    assert s["n_expert"] == ref["n_expert"] and s["n_generated"] == ref["n_generated"]


@gpu
def test_fused_disc_adam_matches_torch_adam():
    tr, venv, gen, rn = _setup(n_envs=8, n_steps=32, batch=64)
    assert tr._fused_disc
    params = tr._rflat.params
    clones = [p.detach().clone().requires_grad_() for p in params]
    opt = th.optim.Adam(clones, **{k: v for k, v in tr._disc_opt.defaults.items()
                                   if k in ("lr", "betas", "eps", "weight_decay")})
    g = tr._disc_ws["grads"]
    for step in range(1, 4):
        gr = th.randn(g.numel(), device="cuda") * 0.1
        g.copy_(gr)
        off = 0
        for c in clones:
            c.grad = gr[off : off + c.numel()].view_as(c).clone()
            off += c.numel()
        opt.step()
        b1, b2 = tr._disc_opt.defaults["betas"]
        lr = tr._disc_opt.defaults["lr"]
        tr._disc_plan.adam(0, 1, lr / (1 - b1**step), (1 - b2**step) ** 0.5, None)
    th.cuda.synchronize()
    for p, c in zip(params, clones):
        th.testing.assert_close(p.detach(), c.detach(), rtol=1e-6, atol=1e-7)


@gpu
def test_fused_disc_train_logs_and_matches_generic_path_shape():
    tr, venv, gen, rn = _setup(n_envs=8, n_steps=32, batch=64)
    assert tr._fused_disc
    before = [p.detach().clone() for p in rn.parameters()]
    tr.train(2 * tr.gen_train_timesteps)
    stats = tr.train_disc()
    assert set(stats) >= {"disc_loss", "disc_acc", "disc_entropy", "n_expert", "n_generated"}
    assert all(np.isfinite(v) for k, v in stats.items() if k != "disc_acc_expert")
    assert stats["n_expert"] == stats["n_generated"] == tr.demo_minibatch_size
    assert any(not th.equal(a, b) for a, b in zip(before, rn.parameters()))
    st = tr._disc_opt.state[tr._rflat.params[0]]
    assert float(st["step"]) == tr._disc_step == 3
    # the generic (autograd + torch Adam) path shares the same optimizer state
    tr.train_disc(expert_samples=next(tr._endless_expert_iterator), gen_samples=tr._gen_sample(tr.demo_batch_size))
    assert float(tr._disc_opt.state[tr._rflat.params[0]]["step"]) == 4
    assert tr._disc_opt.state[tr._rflat.params[0]]["exp_avg"].data_ptr() == tr._r_m.data_ptr()


def _setup_airl(n_envs=4, n_steps=64, batch=64, seed=0, normalize_output=True, init_seed=None, env_id="seals/Hopper-v1"):
    from imitation_amd.data import rollout
    from imitation_amd.engine.airl import DeviceAIRL
    from imitation_amd.policies.base import NormalizeFeaturesExtractor
    from imitation_amd.rewards.reward_nets import BasicShapedRewardNet, NormalizedRewardNet
    from imitation_amd.rl.policies import ActorCriticPolicy
    from imitation_amd.rl.ppo import PPO
    from imitation_amd.util import logger
    from imitation_amd.util.networks import RunningNorm
    from imitation_amd.util.util import make_vec_env

    th.manual_seed(seed)
    np.random.seed(seed)
    rng = np.random.default_rng(seed)
    venv = make_vec_env(env_id, rng=rng, n_envs=n_envs)
    demo_env = make_vec_env(env_id, rng=np.random.default_rng(7), n_envs=4)
    demo_env.action_space.seed(7)  # the random demo policy samples from the action space
    demos = rollout.flatten_trajectories(rollout.generate_trajectories(None, demo_env, rollout.make_min_timesteps(1024), rng=rng))
    if init_seed is not None:  # same demonstrations, different initial weights / engine seeds
        th.manual_seed(init_seed)
        np.random.seed(init_seed)
        seed = init_seed
    gen = PPO(ActorCriticPolicy, venv, n_steps=n_steps, batch_size=batch, n_epochs=2, device="cuda", seed=seed,
              policy_kwargs=dict(net_arch=dict(pi=[64, 64], vf=[64, 64]), activation_fn=th.nn.ReLU,
                                 features_extractor_class=NormalizeFeaturesExtractor))
    rn = BasicShapedRewardNet(venv.observation_space, venv.action_space, normalize_input_layer=RunningNorm)
    if normalize_output:
        rn = NormalizedRewardNet(rn, RunningNorm)
    tr = DeviceAIRL(demonstrations=demos, demo_batch_size=256, venv=venv, gen_algo=gen, reward_net=rn,
                    n_disc_updates_per_round=2, custom_logger=logger.configure("/tmp/ia_test_airl", format_strs=[]))
    return tr, venv, gen, rn


@gpu
@pytest.mark.parametrize("normalize_output", [True, False])
def test_device_airl_rollout_reward_matches_reward_train(normalize_output):
    """Shaped reward (+ output normalisation replayed step by step) == AIRL.reward_train.predict_processed."""
    import copy

    tr, venv, gen, rn = _setup_airl(normalize_output=normalize_output)
    # give the reward nets non-trivial normaliser state first
    tr.train(tr.gen_train_timesteps)
    host = copy.deepcopy(rn)
    tr._rollout()
    th.cuda.synchronize()
    b = {k: v.cpu().numpy() for k, v in tr.buf.items()}
    T, N = b["dones"].shape
    boot = tr._boot.cpu().numpy() if normalize_output else None
    exp = []
    os.environ["IMITATION_AMD_FUSED"] = "0"  # fp32 PyTorch reference (the fused MLP op is bf16)
    try:
        for t in range(T):
            r = host.predict_processed(b["obs_buf"][t], b["act_env"][t], b["next_obs"][t], b["dones"][t] > 0.5)
            exp.append(r)
    finally:
        os.environ.pop("IMITATION_AMD_FUSED", None)
    exp = np.stack(exp)
    got = b["rewards"] - (boot if normalize_output else 0.0)
    if not normalize_output:  # bootstrap only where truncated: compare on the other rows
        mask = ~((b["dones"] > 0.5))
        np.testing.assert_allclose(got[mask], exp[mask], rtol=2e-3, atol=2e-3)
    else:
        np.testing.assert_allclose(got, exp, rtol=2e-3, atol=2e-3)
        onorm = rn.normalize_output_layer
        th.testing.assert_close(onorm.running_mean.cpu(), host.normalize_output_layer.running_mean.cpu(), rtol=1e-4, atol=1e-5)
        th.testing.assert_close(onorm.running_var.cpu(), host.normalize_output_layer.running_var.cpu(), rtol=1e-4, atol=1e-5)
        assert int(onorm.count) == int(host.normalize_output_layer.count)


@gpu
def test_device_airl_rounds_train():
    tr, venv, gen, rn = _setup_airl(n_envs=8, n_steps=128, batch=256)
    assert tr._C.engine_ppo_path(tr._ppo_static).startswith("rc:")
    p0 = [p.detach().clone() for p in gen.policy.parameters()]
    r0 = [p.detach().clone() for p in rn.parameters()]
    tr.train(3 * tr.gen_train_timesteps)
    th.cuda.synchronize()
    assert all(th.isfinite(p).all() for p in list(gen.policy.parameters()) + list(rn.parameters()))
    assert any(not th.equal(a, b) for a, b in zip(p0, gen.policy.parameters()))
    assert any(not th.equal(a, b) for a, b in zip(r0, rn.parameters()))


@gpu
def test_device_airl_graphed_disc_matches_eager():
    """The generic discriminator update as a HIP-graph replay (AIRL's shaped reward net):
    same reward-net parameters and logged statistics as the eager autograd updates
    (IMITATION_AMD_DISC_GRAPH=0), over rounds where the graph is captured then replayed."""
    def run(graph: bool):
        os.environ["IMITATION_AMD_DISC_GRAPH"] = "1" if graph else "0"
        os.environ["IMITATION_AMD_AIRL_FUSED"] = "0"  # the generic update (fused: test_device_airl_fused_disc_*)
        try:
            tr, venv, gen, rn = _setup_airl(n_envs=4, n_steps=64, batch=64, seed=3)
            assert tr._graphed_disc_ok() == graph
            recs = []
            if graph:
                orig = tr._record_disc
                tr._record_disc = lambda stats, step: (recs.append((step, dict(stats))), orig(stats, step))
            else:  # the host loop logs inside train_disc, which returns the same statistics
                orig_td = tr.train_disc
                tr.train_disc = lambda **kw: (lambda st: (recs.append((tr._disc_step, dict(st))), st)[1])(orig_td(**kw))
            tr.train(3 * tr.gen_train_timesteps)
            th.cuda.synchronize()
            if graph:
                assert tr._disc_graph.n_captures == 1 and tr._disc_graph.n_replays == 3 * 2 - 1
            return [p.detach().cpu().clone() for p in rn.parameters()], recs
        finally:
            os.environ.pop("IMITATION_AMD_DISC_GRAPH", None)
            os.environ.pop("IMITATION_AMD_AIRL_FUSED", None)

    p_g, rec_g = run(True)
    p_e, rec_e = run(False)
    assert [s for s, _ in rec_g] == [s for s, _ in rec_e]
    for a, b in zip(p_g, p_e):
        th.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    for (_, a), (_, b) in zip(rec_g, rec_e):
        assert a.keys() == b.keys()
        for k in a:
            assert abs(a[k] - b[k]) <= 1e-3 * max(1.0, abs(b[k])), (k, a[k], b[k])


def _airl_state(tr, rn):
    from imitation_amd.engine.airl import _split
    from imitation_amd.engine.gail import _mlp_layers

    _, shaped = _split(rn)
    norms = [_mlp_layers(shaped.base.mlp)[0], _mlp_layers(shaped.potential._potential_net)[0], tr.pol_norm]
    assert all(n is not None for n in norms)
    return norms


@gpu
@pytest.mark.parametrize("normalize_output,env_id", [(True, "seals/Hopper-v1"), (False, "seals/Hopper-v1"),
                                                     (True, "Pendulum-v1"), (False, "Pendulum-v1")])
def test_device_airl_fused_disc_matches_autograd(normalize_output, env_id):
    """airl_disc.hip (gather, norm merges, policy log-prob + shaped reward fwd / BCE / bwd, Adam)
    vs AdversarialTrainer.train_disc's autograd path on the SAME rows: reward-net gradients
    within bf16 tolerance, every RunningNorm (policy, base, potential twice) equal, loss and
    accuracy statistics close; then one full fused step changes the parameters like Adam.
    Pendulum: continuous actions that the env clips to [-2, 2] -- the replay
    rows hold the clipped env actions, whose diag-Gaussian log-prob enters the logit
    ``r - log pi(a|s)`` (reference ``airl.py:114-119``, ``common.py:476-519``); the loss /
    accuracy statistics are functions of those logits, the gradients of their BCE."""
    from imitation_amd.util import networks

    tr, venv, gen, rn = _setup_airl(n_envs=4, n_steps=64, batch=64, seed=5, normalize_output=normalize_output,
                                    env_id=env_id)
    assert tr._fused_disc, tr._fused_disc_why
    tr.train(tr.gen_train_timesteps)  # replay ring + non-trivial normaliser / optimizer state
    th.cuda.synchronize()
    B = tr.demo_batch_size
    e_idx = tr._endless_expert_iterator.next_indices().clone()
    g_idx = th.randint(0, tr._gen_dev.size(), (B,), device="cuda")
    norms = _airl_state(tr, rn)
    snap = [(n.running_mean.clone(), n.running_var.clone(), n.count.clone()) for n in norms]
    p0 = [p.detach().clone() for p in rn.parameters()]
    m0, v0 = tr._r_m.clone(), tr._r_v.clone()
    step0 = float(tr._disc_opt.state[tr._rflat.params[0]]["step"])
    # fused: gradients only
    with networks.training(tr.reward_train):
        tr._fused_disc_update(0, e_idx=e_idx, g_idx=g_idx, apply=False)
    th.cuda.synchronize()
    g_fused = tr._disc_ws["grads"].clone()
    st_fused = tr._disc_stats[0].clone()
    n_fused = [(n.running_mean.clone(), n.running_var.clone(), n.count.clone()) for n in norms]
    # restore, then the autograd path on the same rows
    with th.no_grad():
        for n, (mu, var, c) in zip(norms, snap):
            n.running_mean.copy_(mu); n.running_var.copy_(var); n.count.copy_(c)
    ed = tr._endless_expert_iterator.data
    ex = {k: ed[k].index_select(0, e_idx) for k in ("obs", "acts", "next_obs", "dones")}
    ga = tr._gen_dev._arrays
    gs = {k: ga[k].index_select(0, g_idx) for k in ("obs", "acts", "next_obs", "dones")}
    lo, hi = (th.as_tensor(x, device="cuda", dtype=th.float32) for x in (venv.action_space.low, venv.action_space.high))
    assert bool(((gs["acts"] >= lo) & (gs["acts"] <= hi)).all())  # the replay holds the env's (clipped) actions
    os.environ["IMITATION_AMD_FUSED"] = "0"  # fp32 PyTorch reference
    try:
        with networks.training(tr.reward_train):
            stats = tr.train_disc(expert_samples=ex, gen_samples=gs)
    finally:
        os.environ.pop("IMITATION_AMD_FUSED", None)
    th.cuda.synchronize()
    g_ref = th.cat([p.grad.reshape(-1) for p in tr._rflat.params])
    scale = float(g_ref.abs().max())
    th.testing.assert_close(g_fused, g_ref, rtol=5e-2, atol=3e-2 * scale)
    cos = float(th.nn.functional.cosine_similarity(g_fused, g_ref, dim=0))
    assert cos > 0.995, cos
    for (mu, var, c), n in zip(n_fused, norms):
        th.testing.assert_close(mu, n.running_mean, rtol=1e-4, atol=1e-5)
        th.testing.assert_close(var, n.running_var, rtol=1e-4, atol=1e-5)
        assert int(c) == int(n.count)
    fs = tr._disc_stats_dict(st_fused.tolist())
    assert abs(fs["disc_loss"] - stats["disc_loss"]) < 2e-2 * max(1.0, abs(stats["disc_loss"]))
    assert abs(fs["disc_acc"] - stats["disc_acc"]) < 0.03
    # one full fused update from the snapshot: Adam moves every parameter with a gradient
    with th.no_grad():
        for p, q in zip(rn.parameters(), p0):
            p.copy_(q)
        tr._r_m.copy_(m0); tr._r_v.copy_(v0)
        for n, (mu, var, c) in zip(norms, snap):
            n.running_mean.copy_(mu); n.running_var.copy_(var); n.count.copy_(c)
    for p in tr._rflat.params:
        tr._disc_opt.state[p]["step"].fill_(step0)
    with networks.training(tr.reward_train):
        tr._fused_disc_update(1, e_idx=e_idx, g_idx=g_idx)
    th.cuda.synchronize()
    moved = th.cat([(p.detach() - q).reshape(-1) for p, q in zip(rn.parameters(), p0)])
    assert bool(th.isfinite(moved).all()) and float(moved.abs().max()) > 0
    assert float(tr._disc_opt.state[tr._rflat.params[0]]["step"]) == step0 + 1


@gpu
def test_device_airl_fused_rounds_train_and_log():
    tr, venv, gen, rn = _setup_airl(n_envs=8, n_steps=128, batch=256)
    # pipelined rounds with the discriminator updates behind PPO on the main stream
    assert tr._fused_disc and tr._overlap_disc and tr._disc_on_main
    r0 = [p.detach().clone() for p in rn.parameters()]
    tr.train(3 * tr.gen_train_timesteps)
    th.cuda.synchronize()
    assert all(th.isfinite(p).all() for p in list(gen.policy.parameters()) + list(rn.parameters()))
    assert any(not th.equal(a, b) for a, b in zip(r0, rn.parameters()))
    assert tr._disc_step == 3 * tr.n_disc_updates_per_round


def _plan_dict(batch: int, rows: int, rc_cus: int, width: int = 32, act: int = 2):
    pi = [17, width, width, 6]
    vf = [17, width, width, 1]
    return dict(D=17, A=6, discrete=0, pi_dims=pi, vf_dims=vf, batch=batch, rows=rows, log_std_off=0,
                rc_gmax=0, rc_cw=0, rc_cus=rc_cus, hidden_act=act)


def test_ppo_plan_caps_cooperating_groups_by_device_cus():
    """ppo_rc_plan (csrc/kernels/ppo_rc.hip) keeps every spinning workgroup co-resident: the
    working blocks (2 x G under the net split) are capped at half the device's CUs; a device
    too small for even one actor / critic pair falls back to the single-workgroup LDS kernel.
    Host-only planning (runs on CPU)."""
    from imitation_amd import _native

    C = _native.load()
    # MI355X (256 CUs): the 16-chunk minibatch spreads over 16 row groups x 2 nets
    assert C.engine_ppo_path(_plan_dict(1024, 4096, 256)) == "rc:g16x1x64:kt2:ns"
    # a 16-CU device: at most 8 working blocks -> 4 row groups of 4 chunks each
    assert C.engine_ppo_path(_plan_dict(1024, 4096, 16)) == "rc:g4x4x64:kt2:ns"
    assert C.engine_ppo_path(_plan_dict(1024, 4096, 8)) == "rc:g2x8x64:kt2:ns"
    # 2 CUs: the actor / critic pair would be the whole device -> non-cooperative kernel
    assert C.engine_ppo_path(_plan_dict(64, 4096, 2)) == "lds"
    # [64, 64] nets: the spill-free family builds; a non-uniform 64-wide net would need the
    # generic build (scratch) and takes the LDS kernel instead
    assert C.engine_ppo_path(_plan_dict(64, 4096, 256, width=64, act=2)) == "rc:g1x1x64:kt4:ns"
    assert C.engine_ppo_path(_plan_dict(64, 4096, 256, width=64, act=1)) == "rc:g1x1x64:kt4:ns"
    d = _plan_dict(64, 4096, 256, width=64)
    d["pi_dims"] = [17, 64, 48, 6]
    assert C.engine_ppo_path(d) == "lds"
    # 32-row minibatches of a generic <= 32-wide net: both nets per 4-wave workgroup
    d = _plan_dict(32, 4096, 256)
    d["D"], d["pi_dims"], d["vf_dims"] = 3, [3, 32, 32, 1], [3, 32, 32, 1]
    assert C.engine_ppo_path(d) == "rc:g1x1x32:kt2"
    # the device query is the default (CPU host: no device -> the MI355X count)
    d = _plan_dict(64, 4096, 0)
    assert C.engine_ppo_path(d).startswith("rc:g1x1x64")


@gpu
@pytest.mark.parametrize("batch,path", [(64, "rc:g1x1x64:kt2:ns"), (256, "rc:g4x1x64:kt2:ns")])
def test_ppo_kernel_timeout_raises(batch, path):
    """Fail-fast: a cooperating workgroup that never publishes (debug_stall knob)
    makes its partners' bounded spins give up; the persistent error word turns the partial
    update into a RuntimeError at the engine's check instead of a silent update."""
    tr, venv, gen, rn = _setup(n_envs=8, n_steps=64, batch=batch, n_epochs=1)
    assert tr._C.engine_ppo_path(tr._ppo_static) == path
    tr._rollout()
    tr._ppo_update()
    th.cuda.synchronize()
    tr.check_errors(blocking=True)  # a healthy update: no error
    tr._ppo_static["debug_stall"] = 1
    tr._ppo_static["spin_limit"] = 4096
    tr._rollout()
    tr._ppo_update()
    th.cuda.synchronize()
    with pytest.raises(RuntimeError, match="timed out"):
        tr.check_errors(blocking=True)
    # the word was cleared: a healthy update afterwards passes again
    tr._ppo_static["debug_stall"] = 0
    tr._ppo_static["spin_limit"] = 0
    tr._rollout()
    tr._ppo_update()
    th.cuda.synchronize()
    tr.check_errors(blocking=True)


@gpu
def test_airl_pipelined_rounds_are_bitwise_the_serial_order(monkeypatch):
    """AIRL rounds pipelined on the main stream (engine/gail.py ``_overlapped_round`` with
    ``_disc_on_main``: PPO statistics copied asynchronously, the discriminator updates and the next
    rollout enqueued before the host reads anything) give bit-identical parameters, Adam moments
    and normalisers to the serial loop (IMITATION_AMD_DISC_OVERLAP=0) -- also as split rounds
    (the updates' gathers + norm merges staged on the main stream, their fwd/bwd + Adam applied
    on the side stream concurrently with the next rollout's step chain) -- also with the staging
    on the side stream during PPO and the policy-norm merges deferred to one launch after it."""
    runs = []
    for mode, split, early in (("0", "0", "0"), ("1", "0", "0"), ("1", "1", "0"), ("1", "1", "1")):
        monkeypatch.setenv("IMITATION_AMD_DISC_OVERLAP", mode)
        monkeypatch.setenv("IMITATION_AMD_AIRL_SPLIT", split)
        monkeypatch.setenv("IMITATION_AMD_AIRL_EARLY_STAGE", early)
        tr, venv, gen, rn = _setup_airl(n_envs=4, n_steps=64, batch=64, seed=3)
        assert tr._fused_disc, tr._fused_disc_why
        assert tr._overlap_disc == (mode == "1")
        assert tr._disc_split == (split == "1")
        tr.n_disc_updates_per_round = 3
        tr.train(3 * tr.gen_train_timesteps)
        th.cuda.synchronize()
        vals = [p.detach().cpu().clone() for p in list(gen.policy.parameters()) + list(rn.parameters())]
        vals += [t.detach().cpu().clone() for t in (tr._r_m, tr._r_v, tr.exp_avg, tr.exp_avg_sq)]
        vals += [n.running_mean.cpu().clone() for n in _airl_state(tr, rn)]
        runs.append(vals)
        assert tr._disc_step == 9
        assert (getattr(tr, "_early_staged_rounds", 0) > 0) == (early == "1" and split == "1")
    for other in runs[1:]:
        bad = [i for i, (a, b) in enumerate(zip(runs[0], other)) if not th.equal(a, b)]
        assert not bad, bad


@gpu
@pytest.mark.parametrize("T,N,count0,int_count", [(1024, 8, 0, False), (1024, 8, 0, True), (300, 3, 5000, True),
                                                   (64, 4, 17, False)])
def test_reward_outnorm_scan_matches_serial_reference(T, N, count0, int_count):
    """reward_outnorm_kernel's wave-level scan of Chan merges (several steps per lane for
    T > 64) against the per-step serial update in float64: the running (mean, var) each step
    is normalised with, the final state, and the int32 count path."""
    from imitation_amd import _native

    C = _native.load()
    dev = th.device("cuda", 0)
    rng = np.random.default_rng(T + N)
    raw = (rng.normal(size=(T, N)) * 3.0 + 1.5).astype(np.float32)
    boot = (rng.random((T, N)) < 0.05).astype(np.float32) * 0.7
    m0, v0 = (0.4, 2.0) if count0 else (0.0, 1.0)
    mean = th.tensor([m0], dtype=th.float32, device=dev)
    var = th.tensor([v0], dtype=th.float32, device=dev)
    cnt_f = th.tensor([float(count0)], dtype=th.float32, device=dev)
    cnt_i = th.tensor(count0, dtype=th.int32, device=dev)
    rewards = th.empty(T, N, dtype=th.float32, device=dev)
    C.engine_reward_outnorm(dict(T=T, N=N, rew_raw=th.from_numpy(raw).to(dev), boot=th.from_numpy(boot).to(dev),
                                 rewards=rewards, mean=mean, var=var, count=cnt_f,
                                 count_i=cnt_i if int_count else None, eps=1e-8, step_stats=None))
    th.cuda.synchronize()
    # serial float64 reference (RunningNorm.update_stats per step, then normalise)
    m, v, c = float(m0), float(v0), float(count0)
    expect = np.empty((T, N))
    for t in range(T):
        expect[t] = (raw[t] - m) / np.sqrt(v + 1e-8) + boot[t]
        bm, bv, bn = raw[t].astype(np.float64).mean(), raw[t].astype(np.float64).var(), float(N)
        d, tot = bm - m, c + bn
        m, v, c = m + d * bn / tot, (v * c + bv * bn + d * d * c * bn / tot) / tot, tot
    np.testing.assert_allclose(rewards.cpu().numpy(), expect, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(mean.item(), m, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(var.item(), v, rtol=1e-4)
    got_c = cnt_i.item() if int_count else cnt_f.item()
    assert got_c == count0 + T * N


@gpu
@pytest.mark.parametrize("T,N", [(1024, 8), (512, 3), (100, 5), (2048, 2)])
def test_gae_scan_register_and_loop_paths_match_reference(T, N):
    """GAE kernel: the register path (chunks of <= 16 steps, T <= 1024) and the loop path
    (T = 2048) against the plain PyTorch recurrence, with episode starts and a final done."""
    from imitation_amd.ops import rl as rl_ops

    g = th.Generator().manual_seed(T * 7 + N)
    rew = th.randn(T, N, generator=g)
    val = th.randn(T, N, generator=g)
    starts = (th.rand(T, N, generator=g) < 0.02).float()
    last_val = th.randn(N, generator=g)
    dones = (th.rand(N, generator=g) < 0.5).float()
    ref_a, ref_r = rl_ops.gae_reference(rew.double(), val.double(), starts.double(), last_val.double(), dones.double(),
                                        0.99, 0.95)
    adv, ret = rl_ops.gae(*(x.cuda() for x in (rew, val, starts, last_val, dones)), 0.99, 0.95)
    np.testing.assert_allclose(adv.cpu().numpy(), ref_a.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(ret.cpu().numpy(), ref_r.numpy(), rtol=1e-4, atol=1e-4)
    # the same pass's [N][4] return / advantage moments (train/explained_variance)
    mom = th.zeros(N, 4, device="cuda")
    adv2, ret2 = rl_ops.gae(*(x.cuda() for x in (rew, val, starts, last_val, dones)), 0.99, 0.95, moments=mom)
    assert th.equal(adv2, adv) and th.equal(ret2, ret)
    want = th.stack([ref_r.sum(0), ref_r.square().sum(0), ref_a.sum(0), ref_a.square().sum(0)], 1)
    np.testing.assert_allclose(mom.cpu().double().numpy(), want.numpy(), rtol=1e-3, atol=1e-2)


@gpu
@pytest.mark.parametrize("env_id,n_episodes,n_envs", [("Pendulum-v1", 10, 4), ("seals/CartPole-v0", 7, 3)])
def test_device_evaluate_matches_host_evaluate_policy(env_id, n_episodes, n_envs):
    """``device_evaluate`` (deterministic rollout chain on a separate env block) counts episodes
    as SB3 evaluate_policy does, is reproducible, leaves the training state alone, and its mean
    return agrees with the host evaluate_policy of the same policy on the same env seeds."""
    from imitation_amd.envs.vec_env import NativeVecEnv
    from imitation_amd.rl.evaluation import evaluate_policy

    tr, venv, gen, rn = _setup(env_id=env_id, n_envs=4, n_steps=32, batch=64,
                               net_arch=[64, 64] if env_id.startswith("seals") else None)
    st0 = tr.state.clone()
    r1, l1 = tr.device_evaluate(n_episodes, n_envs=n_envs, seed=5)
    r2, l2 = tr.device_evaluate(n_episodes, n_envs=n_envs, seed=5)
    assert len(r1) == n_episodes and r1 == r2 and l1 == l2
    assert th.equal(tr.state, st0)
    horizon = 200 if env_id == "Pendulum-v1" else 500
    assert all(n == horizon for n in l1)  # neither env terminates early
    host_env = NativeVecEnv(env_id, n_envs, seed=5, max_episode_steps=horizon)
    hr, hl = evaluate_policy(gen.policy, host_env, n_eval_episodes=n_episodes, deterministic=True,
                             return_episode_rewards=True)
    assert sorted(hl) == sorted(l1)
    # same completion order ((step, env) row-major) on both sides; the device transcendentals
    # differ in the last ulp (ia/envs.h), which an unstable (spinning) pendulum amplifies over a
    # 200-step episode: most -- not all -- episodes agree to rounding
    close = [abs(a - b) <= 0.01 * abs(b) + 1.0 for a, b in zip(r1, hr)]
    assert sum(close) >= 0.6 * len(close), list(zip(r1, hr))


def _engine_snapshot(tr):
    """Everything a resumed run must reproduce bitwise: weights, Adam moments, normalisers,
    the replay ring, env state and counters."""
    ts = [p.detach().clone() for p in tr.gen_algo.policy.parameters()]
    ts += [p.detach().clone() for p in tr._reward_net.parameters()]
    ts += [b.detach().clone() for b in tr.gen_algo.policy.buffers()] + [b.detach().clone() for b in tr._reward_net.buffers()]
    ts += [tr.exp_avg.clone(), tr.exp_avg_sq.clone(), tr.state.clone(), tr.cur_obs.clone()]
    ts += [v.clone() for v in tr._gen_dev._arrays.values()]
    return ts, (tr._global_step, tr._disc_step, tr.gen_algo.num_timesteps, tr._perm_round, tr._step0)


@gpu
@pytest.mark.parametrize("kind", ["gail", "airl"])
def test_device_engine_checkpoint_resume_is_bitwise(kind, tmp_path):
    """k rounds, save_checkpoint, a FRESH trainer built with a different seed,
    load_checkpoint, k more rounds == 2k uninterrupted rounds, bitwise (device Adam state, env
    state / RNG, Feistel round counter, replay ring, fused-discriminator state)."""
    from imitation_amd.utils import checkpoint

    make = (lambda s=None: _setup(n_envs=8, n_steps=64, batch=64, init_seed=s)[0]) if kind == "gail" else \
        (lambda s=None: _setup_airl(n_envs=8, n_steps=64, batch=256, init_seed=s)[0])
    k = 2
    a = make()
    a.train(2 * k * a.gen_train_timesteps)
    th.cuda.synchronize()
    want, want_ctr = _engine_snapshot(a)
    del a
    b = make()
    b.train(k * b.gen_train_timesteps)
    checkpoint.save_checkpoint(b, str(tmp_path / "ck"))
    del b
    c = make(1234)
    checkpoint.load_checkpoint(c, str(tmp_path / "ck"))
    c.train(k * c.gen_train_timesteps)
    th.cuda.synchronize()
    got, got_ctr = _engine_snapshot(c)
    assert got_ctr == want_ctr
    assert len(got) == len(want)
    for i, (x, y) in enumerate(zip(got, want)):
        assert th.equal(x, y), f"tensor {i} differs after resume"


@gpu
@pytest.mark.parametrize("kind", ["gail", "airl"])
def test_device_engine_nan_reward_weight_fails_fast(kind):
    """a poisoned reward-net weight stops training within one round with
    NonFiniteError naming the round (the checks read the statistics already on the host)."""
    from imitation_amd.utils.watchdog import NonFiniteError

    tr = _setup(n_envs=8, n_steps=64, batch=64)[0] if kind == "gail" else _setup_airl(n_envs=8, n_steps=64, batch=256)[0]
    tr.train(tr.gen_train_timesteps)
    with th.no_grad():  # the output bias: a poisoned hidden weight is masked by ReLU (fmax(NaN, 0) = 0)
        list(tr._reward_net.parameters())[-1].view(-1)[0] = float("nan")
    with pytest.raises(NonFiniteError, match="round"):
        tr.train(tr.gen_train_timesteps)


@gpu
def test_device_rollout_stats_match_host_rollout_stats():
    """The CLI's final imit_stats on the GPU (``device_rollout_stats``): the host
    ``rollout_stats(generate_trajectories(...))`` key set, unbiased stopping (>= n episodes, every
    env finishes its episode in flight), learned-reward returns that agree with the host reward
    wrapper's in distribution (stochastic policy, independent streams: means within a few %)."""
    from imitation_amd.data import rollout as rollout_mod

    tr, venv, gen, rn = _setup(env_id="Pendulum-v1", n_envs=4, n_steps=32, batch=64)
    tr.train(2 * tr.gen_train_timesteps)
    dev = tr.device_rollout_stats(40)
    tr.sync_env_to_host()
    trajs = rollout_mod.generate_trajectories(gen.policy, tr.venv_train, rollout_mod.make_min_episodes(40),
                                              rng=np.random.default_rng(0))
    host = rollout_mod.rollout_stats(trajs)
    assert set(dev) == set(host), set(dev) ^ set(host)
    assert dev["n_traj"] >= 40 and dev["n_traj"] % 4 == 0  # fixed horizon: every env stops together
    assert dev["len_min"] == dev["len_max"] == 200
    for k in ("return_mean", "monitor_return_mean"):
        assert abs(dev[k] - host[k]) <= 0.15 * abs(host[k]) + 1.0, (k, dev[k], host[k])

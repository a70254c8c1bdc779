"""FusedAdam / FusedAdamW (ops/optim.py, csrc/kernels/optim.hip) vs torch.optim.Adam / AdamW."""

import pytest
import torch as th

from imitation_amd.ops import optim as optim_ops


def _nets(device, seed=0):
    th.manual_seed(seed)
    a = th.nn.Sequential(th.nn.Linear(7, 13), th.nn.Tanh(), th.nn.Linear(13, 3)).to(device)
    b = th.nn.Sequential(th.nn.Linear(7, 13), th.nn.Tanh(), th.nn.Linear(13, 3)).to(device)
    b.load_state_dict(a.state_dict())
    return a, b


def _run(device, fused_cls, torch_cls, steps=6, **kw):
    a, b = _nets(device)
    oa = fused_cls(a.parameters(), **kw)
    ob = torch_cls(b.parameters(), **kw)
    g = th.Generator().manual_seed(1)
    for _ in range(steps):
        x = th.randn(16, 7, generator=g).to(device)
        for net, opt in ((a, oa), (b, ob)):
            opt.zero_grad()
            net(x).square().mean().backward()
            opt.step()
    return a, b, oa, ob


@pytest.mark.parametrize("kw", [dict(lr=1e-2), dict(lr=3e-3, weight_decay=0.1), dict(lr=1e-2, betas=(0.8, 0.99), eps=1e-6),
                                dict(lr=1e-2, maximize=True)])
def test_fused_adam_matches_torch_cpu(kw):
    a, b, oa, ob = _run("cpu", optim_ops.FusedAdam, th.optim.Adam, **kw)
    for p, q in zip(a.parameters(), b.parameters()):
        th.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_fused_adamw_matches_torch_cpu():
    a, b, oa, ob = _run("cpu", optim_ops.FusedAdamW, th.optim.AdamW, lr=1e-2, weight_decay=0.05)
    for p, q in zip(a.parameters(), b.parameters()):
        th.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_fused_adam_state_dict_roundtrip_with_torch_adam():
    a, b, oa, ob = _run("cpu", optim_ops.FusedAdam, th.optim.Adam, lr=1e-2)
    c, _ = _nets("cpu")
    c.load_state_dict(b.state_dict())
    oc = optim_ops.FusedAdam(c.parameters(), lr=1e-2)
    oc.load_state_dict(ob.state_dict())  # torch Adam state -> flat buffers
    x = th.randn(4, 7)
    for net, opt in ((b, ob), (c, oc)):
        opt.zero_grad()
        net(x).sum().backward()
        opt.step()
    for p, q in zip(b.parameters(), c.parameters()):
        th.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    assert float(oc.state[next(iter(c.parameters()))]["step"]) == 7.0


def test_fused_adam_state_dict_leaves_the_live_state_bound():
    """Each state_dict is a snapshot of the CURRENT flat step counter and moments: taking one must
    not detach the optimizer's live state (a second checkpoint after more steps once saved the
    first checkpoint's step and moments -- a device DRLHP run resumed from it diverged)."""
    p = th.nn.Parameter(th.randn(4, 3))
    opt = optim_ops.FusedAdamW([p], lr=1e-3)
    f = opt._flat[0]
    for n in (1, 2, 3):
        p.grad = th.randn_like(p)
        opt.step()
        st = opt.state_dict()["state"][0]
        assert float(st["step"]) == n
        assert th.equal(st["exp_avg"].reshape(-1), f["m"][:12]) and th.equal(st["exp_avg_sq"].reshape(-1), f["v"][:12])
        assert opt.state[p]["step"] is f["step"]  # still the live counter
    st["exp_avg"].add_(1.0)  # the snapshot is a copy
    assert not th.equal(st["exp_avg"].reshape(-1), f["m"][:12])


def test_fused_adam_checkpoint_loads_into_torch_adam():
    """fused -> torch direction: per-parameter steps, capturable=False; the torch optimizer then
    continues exactly like the fused one (wrong bias correction if the step were shared)."""
    a, b, oa, ob = _run("cpu", optim_ops.FusedAdam, th.optim.Adam, lr=1e-2)
    c, _ = _nets("cpu")
    c.load_state_dict(a.state_dict())
    sd = oa.state_dict()
    assert all(not g["capturable"] for g in sd["param_groups"])
    steps = [st["step"] for st in sd["state"].values()]
    assert len({id(s) for s in steps}) == len(steps)
    oc = th.optim.Adam(c.parameters(), lr=1e-2)
    oc.load_state_dict(sd)
    g = th.Generator().manual_seed(5)
    for _ in range(3):
        x = th.randn(4, 7, generator=g)
        for net, opt in ((a, oa), (c, oc)):
            opt.zero_grad()
            net(x).sum().backward()
            opt.step()
    for p, q in zip(a.parameters(), c.parameters()):
        th.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    assert [float(oc.state[p]["step"]) for p in c.parameters()] == [9.0] * 4
    assert float(oa.state[next(iter(a.parameters()))]["step"]) == 9.0  # the fused counter untouched by state_dict


def test_grads_stay_bound_after_module_zero_grad():
    a, _ = _nets("cpu")
    opt = optim_ops.FusedAdam(a.parameters(), lr=1e-2)
    a.zero_grad()  # nn.Module sets .grad = None
    a(th.randn(3, 7)).sum().backward()
    opt.step()  # re-binds and consumes the fresh grads
    assert all(p.grad is not None and float(p.grad.abs().sum()) == 0.0 for p in a.parameters())


@pytest.mark.gpu
@pytest.mark.parametrize("cls,tcls,kw", [(optim_ops.FusedAdam, th.optim.Adam, dict(lr=1e-2, weight_decay=0.01)),
                                         (optim_ops.FusedAdamW, th.optim.AdamW, dict(lr=1e-2, weight_decay=0.05))])
def test_fused_adam_kernel_matches_torch(cls, tcls, kw):
    a, b, oa, ob = _run("cuda", cls, tcls, steps=8, **kw)
    for p, q in zip(a.parameters(), b.parameters()):
        th.testing.assert_close(p, q, rtol=2e-5, atol=2e-6)


@pytest.mark.gpu
def test_fused_adam_graph_captured_bc_step_matches_eager():
    """BC on the GPU picks FusedAdam; the graphed minibatch step equals the eager one."""
    import os

    import numpy as np

    from imitation_amd.algorithms import bc
    from imitation_amd.envs import spaces
    from imitation_amd.util import logger

    obs_space = spaces.Box(-1, 1, (5,))
    act_space = spaces.Discrete(3)
    rng = np.random.default_rng(0)
    obs = rng.standard_normal((256, 5)).astype(np.float32)
    acts = rng.integers(0, 3, 256)
    from imitation_amd.data import types

    demos = types.TransitionsMinimal(obs=obs, acts=acts, infos=np.array([{}] * 256))
    res = []
    for graph in ("1", "0"):
        os.environ["IMITATION_AMD_BC_GRAPH"] = graph
        th.manual_seed(0)
        t = bc.BC(observation_space=obs_space, action_space=act_space, rng=np.random.default_rng(0), demonstrations=demos,
                  batch_size=32, device="cuda", custom_logger=logger.configure("/tmp/ia_fa", format_strs=[]))
        t._demo_data_loader._rng = np.random.default_rng(5)
        assert isinstance(t.optimizer, optim_ops.FusedAdam)
        t.train(n_batches=20, progress_bar=False, log_interval=10**9)
        res.append([p.detach().cpu().clone() for p in t.policy.parameters()])
    os.environ.pop("IMITATION_AMD_BC_GRAPH", None)
    for p, q in zip(*res):
        th.testing.assert_close(p, q, rtol=1e-4, atol=1e-5)
    # the fused loss (one HIP op over the logits + flat-bucket l2) == the generic loss
    # computed with torch ops everywhere (IMITATION_AMD_FUSED=0): metrics and gradients
    x = th.tensor(obs[:32], device="cuda")
    a = th.tensor(acts[:32], device="cuda")
    out = []
    for fused in ("1", "0"):
        os.environ["IMITATION_AMD_FUSED"] = fused
        m = t.loss_calculator(t.policy, x, a)
        gr = th.autograd.grad(m.loss, [p for p in t.policy.parameters() if p.requires_grad], allow_unused=True)
        out.append(([float(getattr(m, k)) for k in ("neglogp", "entropy", "ent_loss", "prob_true_act", "l2_norm", "loss")],
                    [g for g in gr]))
    os.environ.pop("IMITATION_AMD_FUSED", None)
    np.testing.assert_allclose(out[0][0], out[1][0], rtol=1e-5, atol=1e-6)
    for g0, g1 in zip(out[0][1], out[1][1]):
        if g0 is None or g1 is None:
            assert (g0 is None or float(g0.abs().sum()) == 0) and (g1 is None or float(g1.abs().sum()) == 0)
        else:
            # FUSED=0 also runs the MLP trunk in torch fp32 (the tmlp kernel takes bf16 MFMA
            # operands), so the parameter gradients agree to bf16 precision; the loss op
            # itself is pinned exactly by test_bc_categorical_loss_kernel_matches_reference
            assert float((g0 - g1).norm()) <= 2e-2 * float(g1.norm()) + 1e-7


def test_backward_into_buckets_equals_backward():
    """Gradients written straight into the zeroed buckets == loss.backward() accumulation,
    including a parameter the loss does not use (its slice stays zero)."""
    from imitation_amd.ops.optim import FusedAdam

    th.manual_seed(0)
    net = th.nn.Sequential(th.nn.Linear(5, 7), th.nn.ReLU(), th.nn.Linear(7, 3))
    unused = th.nn.Linear(3, 2)
    mods = th.nn.ModuleList([net, unused])
    x = th.randn(11, 5)
    ref = [th.zeros_like(p) for p in mods.parameters()]
    net.zero_grad(set_to_none=True)
    net(x).square().sum().backward()
    for r, p in zip(ref, net.parameters()):
        r.copy_(p.grad)
    opt = FusedAdam(mods.parameters(), lr=1e-3)
    opt.zero_grad()
    opt.backward_into_buckets(net(x).square().sum())
    for r, p in zip(ref, mods.parameters()):
        th.testing.assert_close(p.grad, r)
    assert float(opt.flat_grads[0][sum(p.numel() for p in net.parameters()):].abs().sum()) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("zero_grad", [True, False])
def test_adam_flat_with_folded_conv_reductions_is_bitwise_the_two_launches(zero_grad):
    """adam_flat(reduce=...) (csrc/kernels/optim.hip: the conv layers' slab columns summed and
    updated by blocks of the Adam launch; the other quads by the elementwise blocks) == the
    conv_reduce_multi launch then adam_flat: parameters, moments and gradient slots bitwise."""
    from imitation_amd import ops

    C = ops.native()
    g = th.Generator().manual_seed(3)
    # NatureCNN conv2 / conv3 at batch 8, their slots inside a flat buffer with other parameters
    layers = [(8, 32, 64, 4, 2, 20), (8, 64, 64, 3, 1, 9)]
    args = {k: [] for k in ("x", "dy", "kh", "kw", "s", "p", "slab")}
    sizes = []
    for B, Cin, N, KH, S, H in layers:
        OH = (H - KH) // S + 1
        x = th.relu(th.randn(B, H, H, Cin, generator=g)).to(th.bfloat16).cuda()
        y = th.randn(B, OH, OH, N, generator=g).to(th.bfloat16).cuda()
        dy = th.randn(B, OH, OH, N, generator=g).to(th.bfloat16).cuda()
        slab = C.conv_wgrad_partials(x, dy, y, KH, KH, S, 1.0, True, 0)
        for k, v in zip(args, (x, dy, KH, KH, S, 0, slab)):
            args[k].append(v)
        sizes += [N * Cin * KH * KH, N]
    offs, o = [], 64  # a leading block of other parameters
    for n in sizes:
        offs.append(o)
        o += n
    n_all = o + 1000
    p0 = th.randn(n_all, generator=g).cuda()
    g0 = th.randn(n_all, generator=g).cuda()
    m0 = th.randn(n_all, generator=g).cuda() * 0.1
    v0 = th.rand(n_all, generator=g).cuda() * 0.1
    step = th.full((1,), 3.0, device="cuda")
    runs = []
    for fold in (False, True):
        p, gr, m, v = p0.clone(), g0.clone(), m0.clone(), v0.clone()
        dws = [gr[offs[2 * i]:offs[2 * i] + sizes[2 * i]] for i in range(len(layers))]
        dbs = [gr[offs[2 * i + 1]:offs[2 * i + 1] + sizes[2 * i + 1]] for i in range(len(layers))]
        red = tuple(args.values()) + (dws, dbs)
        if not fold:
            C.conv_reduce_multi(*red)
        C.adam_flat(p, gr, m, v, step, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, False, zero_grad, None, None, None, None,
                    red if fold else None)
        th.cuda.synchronize()
        runs.append((p, gr, m, v))
    for a, b in zip(*runs):
        assert th.equal(a, b)
    assert not th.equal(runs[0][0], p0)

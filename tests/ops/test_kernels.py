"""HIP kernel numerics vs plain PyTorch fp32 references (run on the MI355X box: -m gpu)."""

import numpy as np
import pytest
import torch as th

from imitation_amd import ops
from imitation_amd.ops import mlp as mlp_ops
from imitation_amd.ops import rl as rl_ops

gpu = pytest.mark.gpu


def _mk_mlp(dims, dev, seed=0):
    g = th.Generator().manual_seed(seed)
    ws, bs = [], []
    for i in range(len(dims) - 1):
        w = (th.randn(dims[i + 1], dims[i], generator=g) / np.sqrt(dims[i])).to(dev).requires_grad_(True)
        b = (0.1 * th.randn(dims[i + 1], generator=g)).to(dev).requires_grad_(True)
        ws.append(w)
        bs.append(b)
    return ws, bs


def test_tmlp_reference_cpu_matches_sequential():
    ws, bs = _mk_mlp([23, 32, 32, 1], "cpu")
    x = th.randn(50, 23)
    y = mlp_ops.tmlp(x, ws, bs, hidden_act=1, out_act=0)
    h = th.relu(x @ ws[0].T + bs[0])
    h = th.relu(h @ ws[1].T + bs[1])
    ref = h @ ws[2].T + bs[2]
    th.testing.assert_close(y, ref)


@gpu
@pytest.mark.parametrize("dims,act,B", [
    ([23, 32, 32, 1], 1, 16384),
    ([17, 32, 32, 6], 2, 64),
    ([17, 64, 64, 1], 2, 1000),
    ([4, 64, 64, 2], 2, 7),
    ([11, 32, 1], 1, 4096),
    ([40, 128, 100, 128, 3], 3, 333),
])
@pytest.mark.parametrize("norm", [False, True])
def test_tmlp_forward_backward_matches_fp32(dims, act, B, norm):
    dev = th.device("cuda")
    ws, bs = _mk_mlp(dims, dev)
    x = th.randn(B, dims[0], device=dev).mul_(2.0).add_(0.5).requires_grad_(True)
    mean = var = None
    if norm:
        mean = th.randn(dims[0], device=dev) * 0.3
        var = th.rand(dims[0], device=dev) + 0.5
    y = mlp_ops.tmlp(x, ws, bs, act, 0, mean, var)
    wr = [w.detach().clone().requires_grad_(True) for w in ws]
    br = [b.detach().clone().requires_grad_(True) for b in bs]
    xr = x.detach().clone().requires_grad_(True)
    yr = mlp_ops.tmlp_reference(xr, wr, br, act, 0, mean, var, emulate_bf16_operands=True)
    scale = yr.abs().max().item() + 1e-3
    # bf16 operands, fp32 accumulation: relative error ~ 2^-8 per layer
    assert (y - yr).abs().max().item() <= 3e-2 * scale
    gy = th.randn_like(y)
    (y * gy).sum().backward()
    (yr * gy).sum().backward()
    # per layer, errors are measured against the layer's largest gradient entry (a bias
    # gradient is a sum over the batch and may cancel to ~0 while its terms do not)
    for l in range(len(ws)):
        ref = max(wr[l].grad.abs().max().item(), br[l].grad.abs().max().item()) + 1e-3
        for a, b in ((ws[l], wr[l]), (bs[l], br[l])):
            err = (a.grad - b.grad).abs().max().item()
            assert err <= 3e-2 * ref, (l, err, ref)
    err = (x.grad - xr.grad).abs().max().item()
    assert err <= 3e-2 * (xr.grad.abs().max().item() + 1e-3)


@gpu
def test_tmlp_is_deterministic():
    dev = th.device("cuda")
    ws, bs = _mk_mlp([23, 32, 32, 1], dev)
    x = th.randn(16384, 23, device=dev)
    grads = []
    for _ in range(2):
        for p in ws + bs:
            p.grad = None
        mlp_ops.tmlp(x, ws, bs, 1, 0).sum().backward()
        grads.append([p.grad.clone() for p in ws + bs])
    for a, b in zip(*grads):
        assert th.equal(a, b)


def _gae_inputs(T, N, dev, seed=0):
    g = th.Generator().manual_seed(seed)
    rew = th.randn(T, N, generator=g)
    val = th.randn(T, N, generator=g)
    starts = (th.rand(T, N, generator=g) < 0.05).float()
    last = th.randn(N, generator=g)
    dones = (th.rand(N, generator=g) < 0.3).float()
    return [t.to(dev) for t in (rew, val, starts, last, dones)]


@gpu
@pytest.mark.parametrize("T,N", [(512, 8), (1, 1), (100, 70), (2048, 129), (65, 64)])
def test_gae_kernel_matches_reference(T, N):
    dev = th.device("cuda")
    args = _gae_inputs(T, N, dev)
    adv, ret = rl_ops.gae(*args, 0.95, 0.9)
    cpu = [a.cpu() for a in args]
    adv_r, ret_r = rl_ops.gae_reference(*cpu, 0.95, 0.9)
    th.testing.assert_close(adv.cpu(), adv_r, rtol=1e-5, atol=1e-5)
    th.testing.assert_close(ret.cpu(), ret_r, rtol=1e-5, atol=1e-5)


@gpu
@pytest.mark.parametrize("E,n", [(5, 4096), (3, 1), (2, 3), (4, 1000), (5, 32768), (1, 70001)])
def test_perm_feistel_kernel_matches_host_twin(E, n):
    got = rl_ops.random_permutations(E, n, 0xDEADBEEF12345, "cuda").cpu().numpy()
    want = rl_ops.random_permutations_reference(E, n, 0xDEADBEEF12345)
    np.testing.assert_array_equal(got, want)
    for row in got:
        assert np.array_equal(np.sort(row), np.arange(n))


@gpu
def test_native_extension_is_loaded_on_gpu():
    from imitation_amd import _native

    C = _native.load()
    assert C.arch == "gfx950"
    assert ops.use_kernel(th.zeros(1, device="cuda"))


@gpu
@pytest.mark.parametrize("P,L,discount,noise,thr", [(32, 50, 1.0, 0.0, 50.0), (7, 3, 0.9, 0.1, 2.0), (200, 130, 0.99, 0.0, 50.0)])
def test_preference_kernel_matches_reference(P, L, discount, noise, thr):
    from imitation_amd.ops import preference as pref_ops

    g = th.Generator().manual_seed(P + L)
    # scale so |diff| stays O(1): torch's BCE backward is ill-conditioned once p saturates
    # (see test_preference_kernel_saturated_grad for that regime).
    r1 = th.randn(P, L, generator=g) * (1.5 / L**0.5)
    r2 = th.randn(P, L, generator=g) * (1.5 / L**0.5)
    prefs = (th.rand(P, generator=g) > 0.5).float()
    prefs[::5] = 0.5
    a1, a2 = r1.clone().requires_grad_(), r2.clone().requires_grad_()
    loss_r, probs_r = pref_ops.bradley_terry_reference(a1, a2, prefs, discount, thr, noise)
    loss_r.backward()
    b1, b2 = r1.cuda().requires_grad_(), r2.cuda().requires_grad_()
    loss, probs = pref_ops.bradley_terry(b1, b2, prefs.cuda(), discount, thr, noise)
    (3.0 * loss).backward()
    th.testing.assert_close(loss.cpu(), loss_r.detach(), rtol=1e-5, atol=1e-6)
    th.testing.assert_close(probs.cpu(), probs_r.detach(), rtol=1e-5, atol=1e-6)
    th.testing.assert_close(b1.grad.cpu(), 3.0 * a1.grad, rtol=1e-4, atol=1e-7)
    th.testing.assert_close(b2.grad.cpu(), 3.0 * a2.grad, rtol=1e-4, atol=1e-7)


@gpu
def test_preference_kernel_saturated_grad():
    """Past |diff| ~ 17 fp32 autograd of BCE(sigmoid) degenerates; the kernel returns the exact
    derivative dloss/ddiff = y - p (float64 oracle) for noise == 0."""
    from imitation_amd.ops import preference as pref_ops

    g = th.Generator().manual_seed(3)
    P, L, thr = 64, 50, 50.0
    r1 = th.randn(P, L, generator=g) * 4.0
    r2 = th.randn(P, L, generator=g) * 4.0
    prefs = (th.rand(P, generator=g) > 0.5).float()
    b1, b2 = r1.cuda().requires_grad_(), r2.cuda().requires_grad_()
    loss, probs = pref_ops.bradley_terry(b1, b2, prefs.cuda(), 1.0, thr, 0.0)
    loss.backward()
    d = (r2.double() - r1.double()).sum(-1)
    inside = (d.abs() <= thr).double()
    pm = 1.0 / (1.0 + d.clamp(-thr, thr).exp())
    expect = ((prefs.double() - pm) * inside / P)[:, None].expand(P, L)
    assert th.isfinite(b2.grad).all()
    th.testing.assert_close(b2.grad.cpu().double(), expect, rtol=1e-4, atol=1e-6)
    th.testing.assert_close(b1.grad.cpu().double(), -expect, rtol=1e-4, atol=1e-6)
    th.testing.assert_close(probs.cpu().double(), pm, rtol=1e-4, atol=1e-6)


@gpu
@pytest.mark.parametrize("dims,act,B,shared", [([23, 32, 32, 1], 1, 3000, True), ([23, 32, 32, 1], 1, 700, False),
                                                ([17, 64, 64, 3], 2, 97, False), ([11, 32, 1], 1, 16, True)])
def test_tmlp_grouped_matches_per_member_reference(dims, act, B, shared):
    """Grouped launch (grid.y = member; ensembles) == each member's fp32 bf16-emulated reference,
    forward and backward (parameter grads, per-member input grads)."""
    dev = th.device("cuda")
    G = 5
    members = [_mk_mlp(dims, dev) for _ in range(G)]
    Ws = [th.stack([m[0][l] for m in members]).detach().requires_grad_(True) for l in range(len(dims) - 1)]
    bs = [th.stack([m[1][l] for m in members]).detach().requires_grad_(True) for l in range(len(dims) - 1)]
    mean = th.randn(G, dims[0], device=dev) * 0.3
    var = th.rand(G, dims[0], device=dev) + 0.5
    x = th.randn(B, dims[0], device=dev) if shared else th.randn(G, B, dims[0], device=dev)
    x.requires_grad_(not shared)
    y = mlp_ops.tmlp_grouped(x, Ws, bs, act, 0, mean, var)
    assert y.shape == (G, B, dims[-1])
    gy = th.randn_like(y)
    (y * gy).sum().backward()
    for g in range(G):
        wr = [W[g].detach().clone().requires_grad_(True) for W in Ws]
        br = [b[g].detach().clone().requires_grad_(True) for b in bs]
        xr = (x if shared else x[g]).detach().clone().requires_grad_(True)
        yr = mlp_ops.tmlp_reference(xr, wr, br, act, 0, mean[g], var[g], emulate_bf16_operands=True)
        scale = yr.abs().max().item() + 1e-3
        assert (y[g] - yr).abs().max().item() <= 3e-2 * scale, g
        (yr * gy[g]).sum().backward()
        for l in range(len(wr)):
            ref = max(wr[l].grad.abs().max().item(), br[l].grad.abs().max().item()) + 1e-3
            assert (Ws[l].grad[g] - wr[l].grad).abs().max().item() <= 3e-2 * ref, (g, l)
            assert (bs[l].grad[g] - br[l].grad).abs().max().item() <= 3e-2 * ref, (g, l)
        if not shared:
            refx = xr.grad.abs().max().item() + 1e-3
            assert (x.grad[g] - xr.grad).abs().max().item() <= 3e-2 * refx, g


@gpu
def test_reward_cnn_fused_forward_matches_modules():
    """CnnRewardNet / BasicPotentialCNN (build_cnn's CNN module) on the HIP conv path ==
    the same modules run layer by layer, forward and parameter gradients."""
    from imitation_amd.envs import spaces
    from imitation_amd.rewards.reward_nets import BasicPotentialCNN, CnnRewardNet

    th.manual_seed(0)
    obs_space = spaces.Box(0, 255, (84, 84, 4), np.uint8)
    act_space = spaces.Discrete(6)
    net = CnnRewardNet(obs_space, act_space).cuda()
    pot = BasicPotentialCNN(obs_space, hid_sizes=(32, 32)).cuda()
    assert net.cnn._fused_plan() is not None and pot._potential_net._fused_plan() is not None
    B = 8
    s = th.rand(B, 84, 84, 4, device="cuda")
    a = th.nn.functional.one_hot(th.randint(0, 6, (B,), device="cuda"), 6).float()
    d = th.zeros(B, device="cuda")
    for mod, fn in ((net, lambda: net(s, a, s, d)), (pot, lambda: pot(s))):
        out = fn()
        g_fused = th.autograd.grad(out.sum(), list(mod.parameters()))
        seq = net.cnn if mod is net else pot._potential_net
        seq._fused_plan = lambda: None  # the module-by-module path
        try:
            ref = fn()
            g_ref = th.autograd.grad(ref.sum(), list(mod.parameters()))
        finally:
            del seq._fused_plan
        assert th.allclose(out, ref, atol=2e-2, rtol=2e-2), (out - ref).abs().max()
        for x1, x2 in zip(g_fused, g_ref):
            assert (x1 - x2).norm() <= 3e-2 * x2.norm() + 1e-6


@gpu
@pytest.mark.parametrize("B,A", [(32, 6), (1, 2), (1000, 18), (257, 64)])
def test_categorical_eval_kernel_matches_autograd(B, A):
    g = th.Generator().manual_seed(B * 100 + A)
    z = (3 * th.randn(B, A, generator=g)).double()
    a = th.randint(0, A, (B,), generator=g)
    w_lp, w_ent = th.randn(B, generator=g).double(), th.randn(B, generator=g).double()
    zr = z.clone().requires_grad_(True)
    lp_r, ent_r = rl_ops.categorical_eval_reference(zr.double(), a)
    ((lp_r * w_lp).sum() + (ent_r * w_ent).sum()).backward()
    zg = z.float().cuda().requires_grad_(True)
    lp, ent = rl_ops.categorical_eval(zg, a.cuda())
    ((lp * w_lp.float().cuda()).sum() + (ent * w_ent.float().cuda()).sum()).backward()
    th.testing.assert_close(lp.double().cpu(), lp_r.detach(), rtol=1e-5, atol=1e-5)
    th.testing.assert_close(ent.double().cpu(), ent_r.detach(), rtol=1e-5, atol=1e-5)
    th.testing.assert_close(zg.grad.double().cpu(), zr.grad, rtol=1e-4, atol=1e-5)


@gpu
@pytest.mark.parametrize("B,A,n", [(32, 6, 1_700_001), (1, 3, 5), (600, 18, 4096)])
def test_bc_categorical_loss_kernel_matches_reference(B, A, n):
    g = th.Generator().manual_seed(B + A)
    z = 2 * th.randn(B, A, generator=g)
    a = th.randint(0, A, (B,), generator=g)
    flat = th.randn(n, generator=g) * 0.01
    params = [flat[: n // 3], flat[n // 3:]]
    zr = z.double().requires_grad_(True)
    ref = rl_ops.bc_categorical_loss_reference(zr, a, [p.double() for p in params], 1e-3, 0.0)
    wg = th.randn(7, generator=g).double()
    (ref * wg).sum().backward()
    zg = z.cuda().requires_grad_(True)
    fc = flat.cuda()
    got, loss = rl_ops.bc_categorical_loss(zg, a.cuda(), [fc[: n // 3], fc[n // 3:]], 1e-3, 0.0, flat=fc)
    assert got.grad_fn is not None and "BCCategorical" in type(got.grad_fn).__name__
    (got * wg.float().cuda()).sum().backward(retain_graph=True)
    th.testing.assert_close(got.double().cpu(), ref.detach(), rtol=2e-5, atol=1e-5)
    th.testing.assert_close(zg.grad.double().cpu(), zr.grad, rtol=1e-4, atol=1e-6)
    # the separate loss output alone (what BC backpropagates)
    th.testing.assert_close(float(loss), float(got[6]))
    zg.grad = None
    loss.backward()
    zr2 = z.double().requires_grad_(True)
    rl_ops.bc_categorical_loss_reference(zr2, a, [p.double() for p in params], 1e-3, 0.0)[6].backward()
    th.testing.assert_close(zg.grad.double().cpu(), zr2.grad, rtol=1e-4, atol=1e-7)


@gpu
@pytest.mark.parametrize("n_envs", [1, 3])
def test_gather_rows_kernel_matches_indexing(n_envs):
    """One-launch multi-field gather (csrc/kernels/gather.hip): 16-B, 4-B and byte rows,
    (step, env) addressing, out-of-range rows as zeros."""
    g = th.Generator().manual_seed(n_envs)
    R = 50 * n_envs
    srcs = [th.randint(0, 255, (R, 84, 84, 4), generator=g, dtype=th.uint8), th.randn(R, 17, generator=g),
            th.randint(0, 6, (R,), generator=g), th.randint(0, 255, (R, 3), generator=g, dtype=th.uint8), th.randn(R)]
    b = th.randint(0, R // n_envs, (77,), generator=g)
    e = th.randint(0, n_envs, (77,), generator=g) if n_envs > 1 else None
    got = rl_ops.gather_rows([s.cuda() for s in srcs], b.cuda(), None if e is None else e.cuda(), n_envs)
    flat = b if e is None else b * n_envs + e
    for s, o in zip(srcs, got):
        assert th.equal(o.cpu(), s[flat])
    bad = th.tensor([0, R // n_envs + 5, -1], device="cuda")
    o = rl_ops.gather_rows([srcs[1].cuda()], bad, None, 1)[0].cpu() if n_envs == 1 else None
    if o is not None:
        assert th.equal(o[0], srcs[1][0]) and float(o[1:].abs().sum()) == 0.0


@gpu
@pytest.mark.parametrize("dims,act,B", [
    ([20, 256, 256, 128], 2, 96),      # HomogenousFeedForward32Policy trunk, agents folded into B
    ([17, 256, 256, 6], 1, 1000),
    ([23, 512, 512, 1], 2, 333),
    ([17, 1024, 1024, 6], 1, 256),    # SAC1024Policy
    ([33, 200, 129, 7], 3, 45),       # ragged widths: every tail path
])
@pytest.mark.parametrize("norm", [False, True])
def test_wide_mlp_matches_fp32_linear(dims, act, B, norm):
    """csrc/kernels/wlin.hip (wide path of ops.tmlp): forward and every gradient vs the fp32
    F.linear reference with bf16-rounded operands (the kernel's operand precision), and the
    forward vs plain fp32 within bf16 tolerance."""
    from imitation_amd import ops

    assert not mlp_ops.kernel_supports(dims) and mlp_ops.wide_supports(dims)
    dev = th.device("cuda")
    ws, bs = _mk_mlp(dims, dev)
    x = th.randn(B, dims[0], device=dev).mul_(2.0).add_(0.5).requires_grad_(True)
    mean = var = None
    if norm:
        mean = th.randn(dims[0], device=dev) * 0.3
        var = th.rand(dims[0], device=dev) + 0.5
    y = mlp_ops.tmlp(x, ws, bs, act, 0, mean, var, wide=True)
    wr = [w.detach().clone().requires_grad_(True) for w in ws]
    br = [b.detach().clone().requires_grad_(True) for b in bs]
    xr = x.detach().clone().requires_grad_(True)
    yr = mlp_ops.tmlp_reference(xr, wr, br, act, 0, mean, var, emulate_bf16_operands=True)
    y32 = mlp_ops.tmlp_reference(x.detach(), [w.detach() for w in ws], [b.detach() for b in bs], act, 0, mean, var)
    scale = yr.abs().max().item() + 1e-3
    assert (y - yr).abs().max().item() <= 2e-2 * scale
    assert (y - y32).abs().max().item() <= 6e-2 * scale
    gy = th.randn_like(y)
    (y * gy).sum().backward()
    (yr * gy).sum().backward()
    for l in range(len(ws)):
        ref = max(wr[l].grad.abs().max().item(), br[l].grad.abs().max().item()) + 1e-3
        for a, b in ((ws[l], wr[l]), (bs[l], br[l])):
            err = (a.grad - b.grad).abs().max().item()
            assert err <= 3e-2 * ref, (l, err, ref)
    err = (x.grad - xr.grad).abs().max().item()
    assert err <= 3e-2 * (xr.grad.abs().max().item() + 1e-3)
    # deterministic: fixed-order reductions
    y2 = mlp_ops.tmlp(x.detach(), ws, bs, act, 0, mean, var, wide=True)
    assert th.equal(y.detach(), y2)


@gpu
@pytest.mark.parametrize("M,N,K", [(4096, 256, 128), (1000, 256, 12), (300, 7, 33), (64, 1024, 1024)])
def test_wide_dw_split_reduction_deterministic(M, N, K):
    """wlin_backward_w splits M over blocks (csrc/kernels/wlin.hip wlin_dw_kernel): the last
    split of every tile sums the partials in split order, so repeated launches (which reuse
    the self-resetting tile counters) give bit-identical dW / db, equal to the fp32 product
    of the bf16-rounded operands."""
    from imitation_amd import _native

    C = _native.load()
    g = th.Generator(device="cuda").manual_seed(M + N + K)
    dz = th.randn(M, N, device="cuda", generator=g)
    x = th.randn(M, K, device="cuda", generator=g)
    outs = [C.wlin_backward_w(dz, x, True) for _ in range(3)]
    ref = dz.bfloat16().float().t() @ x.bfloat16().float()
    scale = ref.abs().max().item()
    assert (outs[0][0] - ref).abs().max().item() <= 1e-4 * scale * max(1.0, M / 256)
    th.testing.assert_close(outs[0][1], dz.sum(0), rtol=1e-5, atol=1e-3)
    for dw, db in outs[1:]:
        assert th.equal(dw, outs[0][0]) and th.equal(db, outs[0][1])

"""NHWC conv-stack kernels (csrc/kernels/conv.hip) vs the fp32 PyTorch reference."""

import numpy as np
import pytest
import torch as th

from imitation_amd.ops import conv as conv_ops

NATURE = [((32, 4, 8, 8), 4), ((64, 32, 4, 4), 2), ((64, 64, 3, 3), 1)]


def _params(seed, layers=NATURE, device="cpu"):
    g = th.Generator().manual_seed(seed)
    ws, bs, ss = [], [], []
    for shape, s in layers:
        fan_in = shape[1] * shape[2] * shape[3]
        ws.append((th.randn(shape, generator=g) * (2.0 / fan_in) ** 0.5).to(device).requires_grad_(True))
        bs.append((0.05 * th.randn(shape[0], generator=g)).to(device).requires_grad_(True))
        ss.append(s)
    return ws, bs, ss


def test_supported_shapes():
    ws, _, ss = _params(0)
    assert conv_ops.supported((2, 84, 84, 4), ws, ss)
    # K = 27: the tap-checked path (input channels zero-padded to 8) needs stride 1
    assert conv_ops.supported((2, 84, 84, 3), [th.zeros(32, 3, 3, 3)], [1])
    assert not conv_ops.supported((2, 84, 84, 3), [th.zeros(32, 3, 3, 3)], [2])
    # reward CNN: 3x3 'same' padding, stride 1 only
    assert conv_ops.supported((2, 84, 84, 4), [th.zeros(32, 4, 3, 3), th.zeros(32, 32, 3, 3)], [1, 1], [1, 1])
    assert not conv_ops.supported((2, 84, 84, 4), [th.zeros(32, 4, 3, 3)], [2], [1])
    assert not conv_ops.supported((2, 84, 84, 3), ws, ss)  # channel mismatch
    assert not conv_ops.supported((2, 84, 84, 4), [th.zeros(24, 4, 8, 8)], [4])  # N % 16


def test_cpu_path_is_reference():
    ws, bs, ss = _params(1)
    x = th.rand(2, 84, 84, 4)
    y = conv_ops.conv_stack(x, ws, bs, ss)
    assert y.shape == (2, 7, 7, 64)
    th.testing.assert_close(y, conv_ops.conv_stack_reference(x, ws, bs, ss))


def test_nature_cnn_matches_sequential_on_cpu():
    from imitation_amd.envs import spaces
    from imitation_amd.rl.torch_layers import NatureCNN

    space = spaces.Box(0, 255, (84, 84, 4), np.uint8)
    th.manual_seed(0)
    net = NatureCNN(space)
    x = th.rand(3, 84, 84, 4)
    ref = net.linear(net.cnn(x.permute(0, 3, 1, 2)))
    th.testing.assert_close(net(x), ref, rtol=1e-5, atol=1e-5)


def _bf(t):
    return t.to(th.bfloat16).float()


def _bf16_emulated(x, ws, bs, ss, gy, pads=None):
    """fp32 PyTorch with the kernels' bf16 rounding points (operands, stored activations, dZ):
    isolates kernel errors from the bf16 precision choice itself."""
    import torch.nn.functional as F
    from torch.nn import grad as nng

    pads = list(pads) if pads is not None else [0] * len(ws)
    h, inputs, acts = _bf(x.permute(0, 3, 1, 2)), [], []
    for w, b, s, p in zip(ws, bs, ss, pads):
        inputs.append(h)
        h = _bf(F.relu(F.conv2d(h, _bf(w), b, stride=s, padding=p)))
        acts.append(h)
    dz = _bf(gy.permute(0, 3, 1, 2)) * (acts[-1] > 0)
    gws, gbs = [None] * len(ws), [None] * len(ws)
    for i in range(len(ws) - 1, -1, -1):
        dzb = _bf(dz)
        gws[i] = nng.conv2d_weight(inputs[i], ws[i].shape, dzb, stride=ss[i], padding=pads[i])
        gbs[i] = dzb.sum((0, 2, 3))
        if i > 0:
            dz = _bf(nng.conv2d_input(inputs[i].shape, _bf(ws[i]), dzb, stride=ss[i], padding=pads[i]) * (acts[i - 1] > 0))
    return acts[-1].permute(0, 2, 3, 1), gws + gbs


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 3, 16, 64])
def test_conv_stack_forward_backward_matches_reference(B):
    ws, bs, ss = _params(2, device="cuda")
    x = th.rand(B, 84, 84, 4, device="cuda")
    y = conv_ops.conv_stack(x, ws, bs, ss)
    ref = conv_ops.conv_stack_reference(x, ws, bs, ss).detach()
    assert y.shape == ref.shape == (B, 7, 7, 64)
    gy = th.randn_like(ref)
    grads = th.autograd.grad((y * gy).sum(), ws + bs)
    ref_grads = th.autograd.grad((conv_ops.conv_stack_reference(x, ws, bs, ss) * gy).sum(), ws + bs)
    with th.no_grad():
        ye, emu = _bf16_emulated(x, [w.detach() for w in ws], [b.detach() for b in bs], ss, gy)
    # exact w.r.t. the bf16 rounding points
    assert float((y - ye).norm() / ye.norm()) < 2e-3
    for g, e in zip(grads, emu):
        assert g.shape == e.shape
        assert float((g - e).norm() / (e.norm() + 1e-12)) < 1e-2
    # and close to fp32: the forward to bf16 precision; gradients of a random-sign loss are
    # dominated by the few ReLU masks that flip under bf16 (cancelling sums), so cosine
    assert float((y - ref).norm() / ref.norm()) < 1e-2
    for g, r in zip(grads, ref_grads):
        cos = float((g * r).sum() / (g.norm() * r.norm() + 1e-12))
        assert cos > 0.99, cos


@pytest.mark.gpu
def test_conv_kernels_loaded_and_deterministic():
    from imitation_amd import ops

    C = ops.native()
    assert hasattr(C, "conv_fwd") and hasattr(C, "conv_wgrad") and hasattr(C, "conv_dgrad")
    ws, bs, ss = _params(3, device="cuda")
    x = th.rand(8, 84, 84, 4, device="cuda")
    out = []
    for _ in range(2):
        y = conv_ops.conv_stack(x, ws, bs, ss)
        out.append(th.autograd.grad(y.square().sum(), ws))
    for a, b in zip(*out):
        assert th.equal(a, b)


@pytest.mark.gpu
def test_nature_cnn_policy_bc_step_on_gpu():
    """ActorCriticCnnPolicy (NatureCNN on the HIP kernels) evaluate_actions + backward on Pong frames."""
    from imitation_amd.envs import spaces
    from imitation_amd.rl.policies import ActorCriticCnnPolicy

    obs_space = spaces.Box(0, 255, (84, 84, 4), np.uint8)
    act_space = spaces.Discrete(6)
    pol = ActorCriticCnnPolicy(obs_space, act_space, lambda _: 1e-3).cuda()
    obs = th.randint(0, 256, (32, 84, 84, 4), device="cuda", dtype=th.uint8)
    acts = th.randint(0, 6, (32,), device="cuda")
    _, logp, ent = pol.evaluate_actions(obs, acts)
    loss = -logp.mean() - 1e-3 * ent.mean()
    loss.backward()
    g = [p.grad for p in pol.features_extractor.cnn.parameters()]
    assert all(x is not None and th.isfinite(x).all() and float(x.abs().sum()) > 0 for x in g)
    # raw uint8 frames (1/255 folded into the first conv's operand load) == the float
    # preprocessed path, forward and gradients
    fe = pol.features_extractor
    assert fe.raw_frames_ok(obs)
    ws = list(fe.parameters())
    y_raw = fe(obs, 1.0 / 255.0)
    g_raw = th.autograd.grad(y_raw.square().sum(), ws)
    y_f = fe(obs.float() / 255.0)
    g_f = th.autograd.grad(y_f.square().sum(), ws)
    th.testing.assert_close(y_raw, y_f, rtol=1e-3, atol=1e-3)
    for a, b in zip(g_raw, g_f):
        th.testing.assert_close(a, b, rtol=2e-2, atol=1e-3 * float(b.abs().max()))


REWARD_CNN = [((32, 4, 3, 3), 1), ((32, 32, 3, 3), 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("cin,B,H,W", [(4, 6, 20, 17), (8, 2, 84, 84), (3, 5, 9, 11)])
def test_same_padding_stack_matches_reference(cin, B, H, W):
    """Reward-CNN stacks (3x3 stride-1 'same' conv + ReLU x2, reward_nets.py CnnRewardNet /
    BasicPotentialCNN) on the padded kernels: exact w.r.t. the bf16 rounding points, and
    close to fp32 F.conv2d (cosine for the gradients, as above)."""
    layers = [((32, cin, 3, 3), 1), ((32, 32, 3, 3), 1)]
    ws, bs, ss = _params(5, layers, device="cuda")
    pads = [1, 1]
    x = th.rand(B, H, W, cin, device="cuda")
    assert conv_ops.supported(tuple(x.shape), ws, ss, pads)
    y = conv_ops.conv_stack(x, ws, bs, ss, 1.0, pads)
    ref = conv_ops.conv_stack_reference(x, ws, bs, ss, 1.0, pads).detach()
    assert y.shape == ref.shape == (B, H, W, 32)
    gy = th.randn_like(ref)
    grads = th.autograd.grad((y * gy).sum(), ws + bs)
    ref_grads = th.autograd.grad((conv_ops.conv_stack_reference(x, ws, bs, ss, 1.0, pads) * gy).sum(), ws + bs)
    with th.no_grad():
        ye, emu = _bf16_emulated(x, [w.detach() for w in ws], [b.detach() for b in bs], ss, gy, pads)
    assert float((y - ye).norm() / ye.norm()) < 2e-3
    for g, e in zip(grads, emu):
        assert g.shape == e.shape
        assert float((g - e).norm() / (e.norm() + 1e-12)) < 1e-2
    assert float((y - ref).norm() / ref.norm()) < 1e-2
    for g, r in zip(grads, ref_grads):
        cos = float((g * r).sum() / (g.norm() * r.norm() + 1e-12))
        assert cos > 0.99, cos


@pytest.mark.gpu
@pytest.mark.parametrize("B", [32, 1, 70])
def test_conv_stack_fc_matches_reference(B):
    """NatureCNN extractor as one node (convs + NHWC FC on cnn_fc / fc_backward) vs the fp32
    torch modules: output and every parameter gradient to bf16-operand accuracy, uint8 input
    with the 1/255 folded in."""
    from imitation_amd.ops import conv as conv_ops

    g = th.Generator().manual_seed(B)
    convs = [th.nn.Conv2d(4, 32, 8, 4), th.nn.Conv2d(32, 64, 4, 2), th.nn.Conv2d(64, 64, 3, 1)]
    fc = th.nn.Linear(3136, 512)
    mods = th.nn.ModuleList(convs + [fc]).cuda()
    x = th.randint(0, 256, (B, 84, 84, 4), generator=g, dtype=th.uint8).cuda()
    ws, bs, st = [c.weight for c in convs], [c.bias for c in convs], [4, 2, 1]
    assert conv_ops.fc_supported(tuple(x.shape), ws, st, 512)
    wg = th.randn(B, 512, generator=g).cuda()
    y = conv_ops.conv_stack_fc(x, ws, bs, st, fc.weight, fc.bias, 1.0 / 255.0)
    gk = th.autograd.grad((y * wg).sum(), list(mods.parameters()))
    yr = x.float().permute(0, 3, 1, 2) / 255.0
    for c in convs:
        yr = th.relu(c(yr))
    yr = th.relu(fc(yr.reshape(B, -1)))
    gr = th.autograd.grad((yr * wg).sum(), list(mods.parameters()))
    assert float((y - yr).norm() / yr.norm()) < 1e-2
    for a, b in zip(gk, gr):  # cosine: ReLU masks flipped by bf16 dominate the difference (see above)
        assert a.shape == b.shape
        cos = float((a * b).sum() / (a.norm() * b.norm() + 1e-12))
        assert cos > 0.98, cos


@pytest.mark.gpu
@pytest.mark.parametrize("M", [32, 1, 70])
def test_fc_backward_kernel_exact_wrt_bf16_operands(M):
    """fc_backward (csrc/kernels/cnn_fc.hip) against fp64 math on the same bf16 operands:
    dW in torch's (c, h, w) column order, db, dX in NHWC order."""
    from imitation_amd import ops

    C = ops.native()
    g = th.Generator().manual_seed(M)
    C3, H3, W3, NH = 64, 7, 7, 512
    K = C3 * H3 * W3
    x = th.randn(M, H3, W3, C3, generator=g).to(th.bfloat16)
    w = th.randn(NH, C3, H3, W3, generator=g) * 0.02
    h = th.relu(th.randn(M, NH, generator=g))
    dh = th.randn(M, NH, generator=g)
    _, wts = C.conv_pack_weights([w.cuda()], [True], [True])
    dW, db, dx = C.fc_backward(x.cuda().reshape(M, -1), dh.cuda(), h.cuda(), wts[0], C3, True)
    dz = (dh * (h > 0)).to(th.bfloat16).double()
    xd = x.double()
    dW_ref = dz.T @ xd.reshape(M, -1)                                     # NHWC columns
    dW_ref = dW_ref.view(NH, H3, W3, C3).permute(0, 3, 1, 2).reshape(NH, K)  # -> torch (c, h, w)
    th.testing.assert_close(dW.cpu().double(), dW_ref, rtol=1e-4, atol=1e-4)
    th.testing.assert_close(db.cpu().double(), (dh * (h > 0)).double().sum(0), rtol=1e-5, atol=1e-5)
    wb = w.to(th.bfloat16).double().permute(0, 2, 3, 1).reshape(NH, K)     # (h, w, c) columns
    dx_ref = dz @ wb
    assert float((dx.cpu().double() - dx_ref).norm() / dx_ref.norm()) < 5e-3


@pytest.mark.gpu
@pytest.mark.parametrize("M", [32, 70])
def test_fc_wgrad_channel_blocks_bitwise_the_column_blocks(M):
    """The channel-aligned fc_wgrad blocks (16-B NHWC operand loads) give bitwise the dW / db /
    dZ of the 64-consecutive-column blocks (same MFMA operands per element)."""
    from imitation_amd import ops

    C = ops.native()
    g = th.Generator().manual_seed(7 + M)
    C3, H3, W3, NH = 64, 7, 7, 512
    x = th.randn(M, H3, W3, C3, generator=g).to(th.bfloat16).cuda().reshape(M, -1)
    w = (th.randn(NH, C3, H3, W3, generator=g) * 0.02).cuda()
    h = th.relu(th.randn(M, NH, generator=g)).cuda()
    dh = th.randn(M, NH, generator=g).cuda()
    _, wts = C.conv_pack_weights([w], [True], [True])
    # an X that is not 16-B aligned takes the 64-column blocks
    xu = th.empty(x.numel() + 1, dtype=x.dtype, device=x.device)[1:].view_as(x)
    xu.copy_(x)
    assert xu.data_ptr() % 16 != 0
    out = [[t.clone() for t in C.fc_backward(xx, dh, h, wts[0], C3, True)] for xx in (xu, x)]
    for a, b in zip(*out):
        assert th.equal(a, b)


def _layer_case(B, C, N, KH, S, H, seed):
    g = th.Generator().manual_seed(seed)
    OH = (H - KH) // S + 1
    x = th.relu(th.randn(B, H, H, C, generator=g)).to(th.bfloat16).cuda()
    y = th.randn(B, OH, OH, N, generator=g).to(th.bfloat16).cuda()  # signs drive the relu_out mask
    dy = th.randn(B, OH, OH, N, generator=g).to(th.bfloat16).cuda()
    w = (th.randn(N, C, KH, KH, generator=g) * 0.05).cuda()
    return x, y, dy, w


# (B, C, N, KH, S, H): NatureCNN conv3 / conv2 at the BC / collector batch sizes
_BC_LAYERS = [(32, 64, 64, 3, 1, 9), (64, 64, 64, 3, 1, 9), (32, 32, 64, 4, 2, 20), (64, 32, 64, 4, 2, 20),
              (7, 64, 64, 3, 1, 9)]


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,N,KH,S,H", _BC_LAYERS)
def test_conv_dgrad_small_batch_forms_match_fp32_and_pf_is_bitwise_the_plain_loop(monkeypatch, B, C, N, KH, S, H):
    """the prefetching small-batch data gradient (conv_dgrad_pf_kernel) is bitwise the
    plain loop (same tap order and MFMA sequence per accumulator); the split-tap form (taps and
    channel halves over waves, LDS sum) sums in another order and matches the fp32 reference."""
    from imitation_amd import ops

    Cn = ops.native()
    x, y, dy, w = _layer_case(B, C, N, KH, S, H, 11 + B + C)
    _, wts = Cn.conv_pack_weights([w], [True])
    out = {}
    for name, form in (("plain", 0), ("pf", 1), ("split", 2)):
        out[name] = Cn.conv_dgrad(dy, y, wts[0], x, S, True, True, 0, form).clone()
    assert th.equal(out["plain"], out["pf"])
    # fp32 reference: dZ = [x > 0] * conv_transpose(dy * [y > 0]) with the bf16 operands
    dz = (dy.float() * (y.float() > 0)).permute(0, 3, 1, 2)
    wb = w.to(th.bfloat16).float()
    ref = th.nn.functional.conv_transpose2d(dz, wb, stride=S).permute(0, 2, 3, 1)
    ref = ref * (x.float() > 0)
    err = float((out["split"].float() - ref).norm() / ref.norm())
    assert err < 1e-2, err


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,N,KH,S,H", _BC_LAYERS)
def test_conv_backward_pair_is_bitwise_the_two_launches(monkeypatch, B, C, N, KH, S, H):
    """conv_backward_pair (weight-gradient partials + split-tap data gradient in ONE launch) gives
    bitwise the slab of conv_wgrad_partials and the dZ of conv_dgrad (split form)."""
    from imitation_amd import ops

    Cn = ops.native()
    x, y, dy, w = _layer_case(B, C, N, KH, S, H, 3 + B + C)
    _, wts = Cn.conv_pack_weights([w], [True])
    assert Cn.conv_backward_pair_ok(x, N, KH, KH, S)
    slab, dz = Cn.conv_backward_pair(x, dy, y, wts[0], S, True)
    slab_ref = Cn.conv_wgrad_partials(x, dy, y, KH, KH, S, 1.0, True, 0)
    dz_ref = Cn.conv_dgrad(dy, y, wts[0], x, S, True, True, 0, 2)
    assert th.equal(slab, slab_ref)
    assert th.equal(dz, dz_ref)


@pytest.mark.gpu
def test_conv_pack_weights_layouts_in_one_launch():
    """conv_pack_weights (forward images and transposes in ONE launch) == the torch permutes of the
    bf16-rounded weights, for the NatureCNN layers and its FC weight (t_hwc) packed together (row
    form: one block per output channel / per (channel, 64 n)), and for layers too wide for the row
    form's LDS image (C x KH*KW > 4224: the 32 x 32 tiles) and an N that is not a multiple of 64."""
    from imitation_amd import ops

    C = ops.native()
    g = th.Generator().manual_seed(5)
    shapes = [(32, 4, 8, 8), (64, 32, 4, 4), (64, 64, 3, 3), (512, 64, 7, 7), (48, 256, 5, 5), (80, 160, 5, 5),
              (96, 3, 9, 9)]
    ws = [th.randn(*s, generator=g).cuda() for s in shapes]
    want_t, t_hwc = [False, True, True, True, True, True, True], [False, False, False, True, False, True, True]
    wbs, wts = C.conv_pack_weights(ws, want_t, t_hwc)
    for w, wb, wt, t, hwc in zip(ws, wbs, wts, want_t, t_hwc):
        wr = w.to(th.bfloat16)
        assert th.equal(wb, wr.permute(0, 2, 3, 1).contiguous())
        if t:
            src = wr.permute(0, 2, 3, 1) if hwc else wr
            assert th.equal(wt.reshape(-1, w.shape[0]), src.reshape(w.shape[0], -1).t().contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,N,KH,S,H,dtype", [(32, 4, 32, 8, 4, 84, th.uint8), (32, 32, 64, 4, 2, 20, th.bfloat16),
                                              (32, 64, 64, 3, 1, 9, th.bfloat16), (7, 64, 64, 3, 1, 9, th.bfloat16),
                                              (5, 32, 64, 4, 2, 20, th.float32)])
def test_conv_fwd_splitk_matches_fp32_and_the_default_form(B, C, N, KH, S, H, dtype):
    """conv_forward_sk (split-K: 16 x 16 tiles over 2-4 waves, LDS sum in wave order) against the fp32
    conv of the same bf16 operands, and close to the default form (other summation order only)."""
    import torch.nn.functional as F

    from imitation_amd import ops

    Cn = ops.native()
    g = th.Generator().manual_seed(B + C + KH)
    scale = 1.0 / 255.0 if dtype == th.uint8 else 1.0
    if dtype == th.uint8:
        x = th.randint(0, 256, (B, H, H, C), generator=g).to(th.uint8)
    else:
        x = th.randn(B, H, H, C, generator=g).to(dtype)
    w = th.randn(N, C, KH, KH, generator=g) * 0.05
    b = th.randn(N, generator=g) * 0.1
    wbs, _ = Cn.conv_pack_weights([w.cuda()], [False])
    y_sk = Cn.conv_fwd(x.cuda(), wbs[0], b.cuda(), S, scale, True, 0, True).float().cpu()
    y_df = Cn.conv_fwd(x.cuda(), wbs[0], b.cuda(), S, scale, True, 0, False).float().cpu()
    xr = (x.float() * scale).to(th.bfloat16).float().permute(0, 3, 1, 2)
    ref = F.relu(F.conv2d(xr, w.to(th.bfloat16).float(), b, stride=S)).permute(0, 2, 3, 1)
    th.testing.assert_close(y_sk, ref, rtol=1e-2, atol=1e-2)
    th.testing.assert_close(y_sk, y_df, rtol=1e-2, atol=1e-2)

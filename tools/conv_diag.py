"""Per-parameter gradient error of the HIP conv stack vs an fp32 reference and a bf16-emulating reference."""
import sys

import torch as th
import torch.nn.functional as F
from torch.nn import grad as nng

import os  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "ops"))
from imitation_amd.ops import conv as conv_ops  # noqa: E402
from test_conv import _params  # noqa: E402


def bf(t):
    return t.to(th.bfloat16).float()


def emulate(x, ws, bs, ss, gy):
    acts = []
    h = bf(x.permute(0, 3, 1, 2))
    inputs = []
    for w, b, s in zip(ws, bs, ss):
        inputs.append(h)
        h = bf(F.relu(F.conv2d(h, bf(w), b, stride=s)))
        acts.append(h)
    dz = bf(gy.permute(0, 3, 1, 2)) * (acts[-1] > 0)
    gws, gbs = [None] * 3, [None] * 3
    for i in range(2, -1, -1):
        dzb = bf(dz)
        gws[i] = nng.conv2d_weight(inputs[i], ws[i].shape, dzb, stride=ss[i])
        gbs[i] = dzb.sum((0, 2, 3))
        if i > 0:
            dx = nng.conv2d_input(inputs[i].shape, bf(ws[i]), dzb, stride=ss[i])
            dz = bf(dx * (acts[i - 1] > 0))
    return acts[-1].permute(0, 2, 3, 1), gws + gbs


for B in (1, 3, 16):
    ws, bs, ss = _params(2, device="cuda")
    x = th.rand(B, 84, 84, 4, device="cuda")
    y = conv_ops.conv_stack(x, ws, bs, ss)
    ref = conv_ops.conv_stack_reference(x, ws, bs, ss)
    gy = th.randn_like(ref)
    grads = th.autograd.grad((y * gy).sum(), ws + bs)
    ref_grads = th.autograd.grad((ref * gy).sum(), ws + bs)
    with th.no_grad():
        ye, eg = emulate(x, [w.detach() for w in ws], [b.detach() for b in bs], ss, gy)
    print(f"B={B} fwd rel vs fp32 {float((y - ref).norm() / ref.norm()):.2e} vs emu {float((y - ye).norm() / ye.norm()):.2e}")
    names = ["w1", "w2", "w3", "b1", "b2", "b3"]
    for nm, g, r, e in zip(names, grads, ref_grads, eg):
        print(f"  {nm}: rel vs fp32 {float((g - r).norm() / r.norm()):.2e}  vs emu {float((g - e).norm() / e.norm()):.2e}  emu-vs-fp32 {float((e - r).norm() / r.norm()):.2e}")

"""Conv+ReLU stacks on the NHWC implicit-GEMM HIP kernels (``csrc/kernels/conv.hip``).

The NatureCNN trunk of the Atari policies (SB3 ``NatureCNN``, selected by the
reference's ``cnn_policy`` named config, ``src/imitation/scripts/ingredients/policy.py:48-50``;
DAgger-Pong in BASELINE.json) is three valid-padding conv+ReLU layers; the reward CNNs
(``CnnRewardNet`` / ``BasicPotentialCNN``, reference ``reward_nets.py:535-600`` via
``networks.py:286-357`` ``build_cnn``) are 3x3 stride-1 ``same``-padded conv+ReLU layers
(``paddings``; inputs whose channel count is not a multiple of 8 are zero-padded to one).
``conv_stack`` runs either as one autograd node:

* forward: one MFMA kernel per layer (bias + ReLU fused), activations kept NHWC bf16;
* backward: per layer one weight-gradient kernel (+ a deterministic block reduction)
  and, below the top layer, one data-gradient kernel whose epilogue applies the
  previous layer's ReLU mask -- no separate mask / transpose / im2col launches.

Numerics: bf16 operands, fp32 accumulation (weights are fp32 module parameters,
rounded to bf16 per call). ``conv_stack_reference`` is the fp32 PyTorch oracle.
"""

from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.nn.functional as F

from imitation_amd import ops


def conv_stack_reference(x_nhwc: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor],
                         strides: Sequence[int], in_scale: float = 1.0,
                         paddings: Optional[Sequence[int]] = None) -> torch.Tensor:
    """fp32 reference: NHWC in, NHWC out (ReLU after every layer)."""
    x = x_nhwc.float().permute(0, 3, 1, 2) * in_scale
    pads = list(paddings) if paddings is not None else [0] * len(weights)
    for w, b, s, p in zip(weights, biases, strides, pads):
        x = F.relu(F.conv2d(x, w, b, stride=s, padding=p))
    return x.permute(0, 2, 3, 1)


def supported(x_shape, weights: Sequence[torch.Tensor], strides: Sequence[int],
              paddings: Optional[Sequence[int]] = None) -> bool:
    """Whether the kernel path covers this stack: valid layers need KW*C % 8 == 0 (K % 32 for
    the MFMA k-steps, else the tap-checked path); padded layers stride 1 and C % 8 == 0 (the
    first layer's channels are zero-padded to a multiple of 8 by :func:`conv_stack`)."""
    if len(x_shape) != 4:
        return False
    _, H, W, C = x_shape
    pads = list(paddings) if paddings is not None else [0] * len(weights)
    for i, (w, s, p) in enumerate(zip(weights, strides, pads)):
        N, Cw, KH, KW = w.shape
        if Cw != C or N % 16 != 0 or N > 64:
            return False
        tap_checked = p > 0 or (KH * KW * C) % 32 != 0
        Ce = C + (-C) % 8 if (i == 0 and tap_checked) else C
        if tap_checked and (s != 1 or Ce % 8 != 0):
            return False
        if not tap_checked and (KW * C) % 8 != 0:
            return False
        if i > 0 and (C % 16 != 0 or C > 64):
            return False
        if i + 1 < len(weights) and N % 32 != 0:  # dgrad of the next layer walks taps in 32-wide k-steps
            return False
        OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
        if OH <= 0 or OW <= 0:
            return False
        H, W, C = OH, OW, N
    return True


class _ConvStack(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, in_scale, strides, pads, out_bf16, *params):
        C = ops.native()
        ws, bs = params[0::2], params[1::2]
        acts: List[torch.Tensor] = []
        h = x
        # every layer's bf16 GEMM weights (and the data-gradient layouts of layers 1..n-1) in ONE launch
        wbs, wts = C.conv_pack_weights([w.detach().contiguous() for w in ws], [i > 0 for i in range(len(ws))])
        for i, (wb, b, s, p) in enumerate(zip(wbs, bs, strides, pads)):
            h = C.conv_fwd(h, wb, b.detach().float().contiguous(), int(s), float(in_scale) if i == 0 else 1.0, True, int(p))
            acts.append(h)
        ctx.wts = wts
        ctx.save_for_backward(x, *ws, *acts)
        ctx.in_scale = float(in_scale)
        ctx.strides = tuple(int(s) for s in strides)
        ctx.pads = tuple(int(p) for p in pads)
        ctx.n = len(ws)
        return h if out_bf16 else h.float()

    @staticmethod
    def backward(ctx, gy):
        n = ctx.n
        saved = ctx.saved_tensors
        grads = _stack_backward(ctx, saved[0], saved[1 : 1 + n], saved[1 + n :], gy.contiguous().to(torch.bfloat16))
        return (None, None, None, None, None, *grads)


def _stack_backward(ctx, x, ws, acts, dz) -> List[Optional[torch.Tensor]]:
    """Conv-stack backward from the top layer's (pre-ReLU-mask) upstream gradient ``dz``
    (bf16 NHWC): per layer one weight-gradient kernel and, below the top, one data-gradient
    kernel that applies the next-lower layer's ReLU mask."""
    C = ops.native()
    n = len(ws)
    grads: List[Optional[torch.Tensor]] = [None] * (2 * n)
    for i in range(n - 1, -1, -1):
        w, s, p = ws[i], ctx.strides[i], ctx.pads[i]
        N, Cin, KH, KW = w.shape
        inp = x if i == 0 else acts[i - 1]
        top = i == n - 1  # only the top layer's ReLU mask is still pending on dz
        scale = ctx.in_scale if i == 0 else 1.0
        dW, db = C.conv_wgrad(inp, dz, acts[i], int(KH), int(KW), int(s), scale, top, p)  # [N, C, KH, KW]
        grads[2 * i] = dW if dW.dtype == w.dtype else dW.to(w.dtype)
        grads[2 * i + 1] = db
        if i > 0:
            dz = C.conv_dgrad(dz, acts[i], ctx.wts[i], acts[i - 1], int(s), top, True, p)
    return grads


class _ConvStackFC(torch.autograd.Function):
    """Conv stack + flatten + Linear + ReLU (SB3 NatureCNN's whole feature extractor) as one
    autograd node: all weights packed in ONE launch (the FC weight to (h, w, c) columns and
    its transposed data-gradient layout), the FC forward on the conv output's NHWC bf16
    (``cnn_fc``), its backward as 2 launches (``fc_backward``: dW in torch's column order +
    db, and dX in NHWC = the trunk's upstream gradient) -- no flatten permutes, no fp32
    hipBLASLt GEMMs over the 6.4 MB weight."""

    @staticmethod
    def forward(ctx, x, in_scale, strides, *params):
        C = ops.native()
        ws, bs = params[0:-2:2], params[1:-2:2]
        fc_w, fc_b = params[-2], params[-1]
        n = len(ws)
        acts: List[torch.Tensor] = []
        # trunk shape -> the FC weight viewed as a [NH, C3, H3, W3] "conv" for the packer
        h = x
        B = x.shape[0]
        wsrc = [w.detach().contiguous() for w in ws]
        Hh, Ww, Cc = x.shape[1], x.shape[2], x.shape[3]
        for w, s in zip(ws, strides):
            Hh, Ww, Cc = (Hh - w.shape[2]) // int(s) + 1, (Ww - w.shape[3]) // int(s) + 1, w.shape[0]
        NH = fc_w.shape[0]
        wsrc.append(fc_w.detach().contiguous().view(NH, Cc, Hh, Ww))
        wbs, wts = C.conv_pack_weights(wsrc, [i > 0 for i in range(n)] + [True], [False] * n + [True])
        for i, (wb, b, s) in enumerate(zip(wbs[:n], bs, strides)):
            h = C.conv_fwd(h, wb, b.detach().float().contiguous(), int(s), float(in_scale) if i == 0 else 1.0, True, 0)
            acts.append(h)
        xf = h.reshape(B, -1)
        out = C.cnn_fc(xf, wbs[n].view(NH, -1), fc_b.detach().float().contiguous())
        ctx.wts = wts[:n]
        ctx.wt_fc = wts[n]
        ctx.c3 = int(Cc)
        ctx.save_for_backward(x, *ws, *acts, out)
        ctx.in_scale = float(in_scale)
        ctx.strides = tuple(int(s) for s in strides)
        ctx.pads = (0,) * n
        ctx.n = n
        return out

    @staticmethod
    def backward(ctx, dh):
        C = ops.native()
        n = ctx.n
        saved = ctx.saved_tensors
        x, ws, acts, out = saved[0], saved[1 : 1 + n], saved[1 + n : 1 + 2 * n], saved[1 + 2 * n]
        top = acts[-1]
        dW, db, dx = C.fc_backward(top.reshape(top.shape[0], -1), dh, out, ctx.wt_fc, ctx.c3, True)
        grads = _stack_backward(ctx, x, ws, acts, dx.view(top.shape))
        return (None, None, None, *grads, dW, db)


def fc_supported(x_shape, weights: Sequence[torch.Tensor], strides: Sequence[int], fc_out: int) -> bool:
    """Whether :func:`conv_stack_fc` covers this trunk: a valid-padding conv stack the kernels
    take without channel padding, and an FC with K = C3*H3*W3 % 64 == 0, NH % 64 == 0."""
    if not supported(x_shape, weights, strides):
        return False
    _, H, W, C = x_shape
    w0 = weights[0]
    if (w0.shape[1] * w0.shape[2] * w0.shape[3]) % 32 != 0:
        return False  # first layer would take the tap-checked, channel-padded path
    for w, s in zip(weights, strides):
        H, W, C = (H - w.shape[2]) // int(s) + 1, (W - w.shape[3]) // int(s) + 1, w.shape[0]
    return (C * H * W) % 64 == 0 and fc_out % 64 == 0


def conv_stack_fc(x_nhwc: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor],
                  strides: Sequence[int], fc_weight: torch.Tensor, fc_bias: torch.Tensor,
                  in_scale: float = 1.0) -> torch.Tensor:
    """``relu(linear(flatten_chw(conv_stack(x))))`` -- NatureCNN's feature extractor -- as one
    autograd node on the HIP kernels (:class:`_ConvStackFC`); the fp32 reference elsewhere.
    Flatten order is torch's (C, H, W), as ``nn.Flatten`` after NCHW convs."""
    if not ops.use_kernel(x_nhwc) or not fc_supported(tuple(x_nhwc.shape), weights, strides, fc_weight.shape[0]):
        y = conv_stack_reference(x_nhwc, weights, biases, strides, in_scale)
        y = y.permute(0, 3, 1, 2).reshape(y.shape[0], -1)
        return F.relu(F.linear(y, fc_weight, fc_bias))
    params = []
    for w, b in zip(weights, biases):
        params += [w, b]
    return _ConvStackFC.apply(x_nhwc.contiguous(), float(in_scale), tuple(int(s) for s in strides), *params, fc_weight,
                              fc_bias)


def conv_stack(x_nhwc: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor],
               strides: Sequence[int], in_scale: float = 1.0, paddings: Optional[Sequence[int]] = None,
               out_dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """ReLU(conv) x len(weights) over an NHWC input (zero ``paddings`` per layer); returns
    NHWC in ``out_dtype`` (fp32, or the kernels' bf16 activations without a conversion pass).

    GPU tensors run the HIP kernels (raising if the extension is missing); CPU tensors
    and ``IMITATION_AMD_FUSED=0`` use :func:`conv_stack_reference`. The input gets no
    gradient (it is observation data).
    """
    pads = tuple(int(p) for p in paddings) if paddings is not None else (0,) * len(weights)
    if not ops.use_kernel(x_nhwc) or not supported(tuple(x_nhwc.shape), weights, strides, pads):
        return conv_stack_reference(x_nhwc, weights, biases, strides, in_scale, pads).to(out_dtype)
    weights = list(weights)
    w0 = weights[0]
    cpad = (-x_nhwc.shape[-1]) % 8
    if cpad and (pads[0] > 0 or (w0.shape[1] * w0.shape[2] * w0.shape[3]) % 32 != 0):
        # tap-checked first layer: channels zero-padded to a multiple of 8 (input and weights;
        # the weights' padding is differentiable, so their gradient is sliced back by autograd)
        x_nhwc = F.pad(x_nhwc, (0, cpad))
        weights[0] = F.pad(w0, (0, 0, 0, 0, 0, cpad))
    params = []
    for w, b in zip(weights, biases):
        params += [w, b]
    out_bf16 = out_dtype == torch.bfloat16
    y = _ConvStack.apply(x_nhwc.contiguous(), float(in_scale), tuple(int(s) for s in strides), pads, out_bf16, *params)
    return y if out_bf16 or out_dtype == torch.float32 else y.to(out_dtype)

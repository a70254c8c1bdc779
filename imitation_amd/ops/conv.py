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
        C = ops.native()
        n = ctx.n
        saved = ctx.saved_tensors
        x, ws, acts = saved[0], saved[1 : 1 + n], saved[1 + n :]
        grads = [None] * (2 * n)
        dz = gy.contiguous().to(torch.bfloat16)
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
        return (None, None, None, None, None, *grads)


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

"""Fused tiny-MLP op (``csrc/kernels/tmlp.hip``) with autograd.

One launch evaluates a whole ``[norm] -> Linear -> act -> ... -> Linear -> out_act``
stack for every row of the batch on MFMA (bf16 operands, fp32 accumulation);
the backward launch recomputes the forward tile in LDS and emits dW/db (and
dX when needed) with a deterministic block-order reduction.

Replaces the per-layer PyTorch launches of ``build_mlp`` stacks used by the
reference's reward nets and SB3 policy heads
(``src/imitation/util/networks.py:204-283``, ``src/imitation/rewards/reward_nets.py:441-457``).
"""

from __future__ import annotations

import os
from typing import List, Optional, Sequence

import torch
import torch.nn.functional as F

ACT_CODES = {"identity": 0, "relu": 1, "tanh": 2, "leaky_relu": 3, "sigmoid": 4}


def act_code(module_or_name) -> Optional[int]:
    """Activation code for a module / name, or None if the kernel cannot fuse it."""
    import torch.nn as nn

    if module_or_name is None:
        return 0
    if isinstance(module_or_name, str):
        return ACT_CODES.get(module_or_name)
    m = module_or_name
    if isinstance(m, type):
        try:
            m = m()
        except TypeError:
            return None
    if isinstance(m, nn.Identity):
        return 0
    if isinstance(m, nn.ReLU):
        return 1
    if isinstance(m, nn.Tanh):
        return 2
    if isinstance(m, nn.LeakyReLU) and abs(m.negative_slope - 0.01) < 1e-12:
        return 3
    if isinstance(m, nn.Sigmoid):
        return 4
    return None


def _act(code: int, x: torch.Tensor) -> torch.Tensor:
    if code == 1:
        return F.relu(x)
    if code == 2:
        return torch.tanh(x)
    if code == 3:
        return F.leaky_relu(x, 0.01)
    if code == 4:
        return torch.sigmoid(x)
    return x


class _RoundBF16(torch.autograd.Function):
    """Round values to bf16 in the forward pass, identity gradient (straight-through)."""

    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g


def tmlp_reference(
    x: torch.Tensor,
    weights: Sequence[torch.Tensor],
    biases: Sequence[torch.Tensor],
    hidden_act: int,
    out_act: int = 0,
    norm_mean: Optional[torch.Tensor] = None,
    norm_var: Optional[torch.Tensor] = None,
    norm_eps: float = 1e-5,
    emulate_bf16_operands: bool = False,
) -> torch.Tensor:
    """Plain PyTorch fp32 reference of the fused MLP (the kernel's numerics oracle).

    ``emulate_bf16_operands`` rounds every MFMA operand (normalised input, weights,
    hidden activations) to bf16 while keeping fp32 accumulation -- exactly the
    kernel's operand precision -- so that piecewise activations (ReLU) take the same
    branch as the kernel and gradients can be compared tightly.
    """
    rnd = _RoundBF16.apply if emulate_bf16_operands else (lambda t: t)
    h = x
    if norm_mean is not None:
        h = (h - norm_mean) / torch.sqrt(norm_var + norm_eps)
    n = len(weights)
    for i, (w, b) in enumerate(zip(weights, biases)):
        h = F.linear(rnd(h), rnd(w), b)
        h = _act(out_act if i == n - 1 else hidden_act, h)
    return h


class _TMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, hidden_act, out_act, mean, var, eps, *params):
        from imitation_amd.ops import native

        C = native()
        ws: List[torch.Tensor] = [p.contiguous() for p in params[0::2]]
        bs: List[torch.Tensor] = [p.contiguous() for p in params[1::2]]
        xc = x.contiguous()
        y = C.tmlp_forward(xc, ws, bs, int(hidden_act), int(out_act), mean, var, float(eps), 0.0)
        ctx.hidden_act, ctx.out_act, ctx.eps = int(hidden_act), int(out_act), float(eps)
        ctx.has_norm = mean is not None
        ctx.n_layers = len(ws)
        saved = [xc] + ws + bs
        if mean is not None:
            # snapshot: a train-mode RunningNorm updates these buffers in place on its next
            # call (e.g. the potential net of a shaped reward on s and then on s')
            mv = torch.stack([mean, var])
            saved += [mv[0], mv[1]]
        ctx.save_for_backward(*saved)
        return y

    @staticmethod
    def backward(ctx, dy):
        from imitation_amd.ops import native

        C = native()
        saved = ctx.saved_tensors
        L = ctx.n_layers
        x = saved[0]
        ws = list(saved[1 : 1 + L])
        bs = list(saved[1 + L : 1 + 2 * L])
        mean = var = None
        if ctx.has_norm:
            mean, var = saved[1 + 2 * L], saved[2 + 2 * L]
        need_dx = bool(ctx.needs_input_grad[0])
        dx, dws, dbs = C.tmlp_backward(
            x, dy.contiguous(), ws, bs, ctx.hidden_act, ctx.out_act, mean, var, ctx.eps, 0.0, need_dx
        )
        grads = []
        for dw, db in zip(dws, dbs):
            grads += [dw, db]
        return (dx, None, None, None, None, None, *grads)


def kernel_supports(dims: Sequence[int]) -> bool:
    """The whole-network-in-LDS tiny-MLP kernel (tmlp.hip)."""
    return 1 <= len(dims) - 1 <= 4 and max(dims) <= 128


WIDE_MAX = 1024


def wide_supports(dims: Sequence[int]) -> bool:
    """The per-layer wide kernels (wlin.hip): widths up to 1024, any depth."""
    return 1 <= len(dims) - 1 <= 16 and max(dims) <= WIDE_MAX


def wide_default() -> bool:
    """Process default of the bf16-operand wide path (``IMITATION_AMD_WIDE_MLP=1``; off).

    The wide kernels multiply bf16 operands (fp32 accumulation) while the reference runs these
    networks in fp32, so a generic wide MLP stays on the fp32 path unless the caller opts in --
    per module (``policy.wide_bf16 = True``, see :func:`set_wide_bf16`) or per process."""
    return os.environ.get("IMITATION_AMD_WIDE_MLP", "0") == "1"


def set_wide_bf16(module: torch.nn.Module, enabled: bool = True) -> torch.nn.Module:
    """Opt ``module`` (a policy / network using :func:`tmlp`) in or out of the bf16-operand
    wide-MLP kernels; clears a cached fusion plan."""
    for m in module.modules():
        object.__setattr__(m, "wide_bf16", bool(enabled))
        for cache in ("_ia_fusion", "_ia_plan"):
            if hasattr(m, cache):
                object.__setattr__(m, cache, None)
    return module


def fusable(dims: Sequence[int], wide: Optional[bool] = None) -> bool:
    """Whether :func:`tmlp` runs this MLP on a HIP kernel: the tiny kernel (fp32 MFMA) always,
    the bf16-operand wide path when ``wide`` (default: :func:`wide_default`)."""
    if kernel_supports(dims):
        return True
    return (wide_default() if wide is None else wide) and wide_supports(dims)


def _act_grad_from_out(code: int, y: torch.Tensor) -> torch.Tensor:
    if code == 1:
        return (y > 0).to(y.dtype)
    if code == 2:
        return 1.0 - y * y
    if code == 3:
        return torch.where(y > 0, torch.ones_like(y), torch.full_like(y, 0.01))
    if code == 4:
        return y * (1.0 - y)
    return torch.ones_like(y)


class _WideMLPFn(torch.autograd.Function):
    """MLPs wider than the tiny-MLP kernel (the fork's [256, 256, 128] multi-agent policy,
    SAC1024Policy [1024, 1024]): one ``wlin_forward`` launch per layer (GEMM + bias +
    activation), and per layer in the backward one ``wlin_backward_w`` (dW and db) and one
    ``wlin_backward_x`` (dX times the previous activation's derivative) -- bf16 MFMA
    operands, fp32 accumulation (csrc/kernels/wlin.hip)."""

    @staticmethod
    def forward(ctx, x, hidden_act, out_act, mean, var, eps, *params):
        from imitation_amd.ops import native

        C = native()
        ws = [p.contiguous() for p in params[0::2]]
        bs = [p.contiguous() for p in params[1::2]]
        h = x.contiguous()
        rstd = None
        if mean is not None:
            rstd = torch.rsqrt(var + eps)
            h = ((h - mean) * rstd).contiguous()
        hs = [h]
        L = len(ws)
        for l in range(L):
            h = C.wlin_forward(h, ws[l], bs[l], int(out_act if l == L - 1 else hidden_act))
            hs.append(h)
        ctx.cfg = (int(hidden_act), int(out_act), L, rstd is not None)
        ctx.save_for_backward(*hs, *ws, *([rstd] if rstd is not None else []))
        return h

    @staticmethod
    def backward(ctx, dy):
        from imitation_amd.ops import native

        C = native()
        hidden_act, out_act, L, has_norm = ctx.cfg
        saved = ctx.saved_tensors
        hs, ws = saved[: L + 1], saved[L + 1 : 2 * L + 1]
        rstd = saved[2 * L + 1] if has_norm else None
        dz = dy.contiguous()
        if out_act != 0:
            dz = (dz * _act_grad_from_out(out_act, hs[L])).contiguous()
        grads = [None] * (2 * L)
        dx = None
        for l in range(L - 1, -1, -1):
            dW, db = C.wlin_backward_w(dz, hs[l], True)
            grads[2 * l], grads[2 * l + 1] = dW, db
            if l > 0:
                dz = C.wlin_backward_x(dz, ws[l], hs[l], hidden_act, None)
            elif ctx.needs_input_grad[0]:
                if ws[0].shape[1] <= 64:
                    # a narrow input (e.g. SAC's critic input obs + action, 17 -> 1024): the
                    # output has too few 32-column tiles to fill the device, and with no
                    # activation derivative to fuse this is a plain GEMM (hipBLASLt / rocBLAS)
                    dx = dz @ ws[0]
                    if rstd is not None:
                        dx = dx * rstd
                else:
                    dx = C.wlin_backward_x(dz, ws[0], None, 0, rstd)
        return (dx, None, None, None, None, None, *grads)


def tmlp(
    x: torch.Tensor,
    weights: Sequence[torch.Tensor],
    biases: Sequence[torch.Tensor],
    hidden_act: int,
    out_act: int = 0,
    norm_mean: Optional[torch.Tensor] = None,
    norm_var: Optional[torch.Tensor] = None,
    norm_eps: float = 1e-5,
    wide: Optional[bool] = None,
) -> torch.Tensor:
    """Fused MLP forward (differentiable w.r.t. ``x`` and every weight / bias).

    GPU fp32 tensors go through a HIP kernel -- the whole-network tiny-MLP kernel for widths
    <= 128, the per-layer bf16-operand wide kernels up to 1024 when ``wide`` (opt-in, see
    :func:`wide_default`) -- everything else through :func:`tmlp_reference`.
    """
    from imitation_amd.ops import use_kernel

    dims = [weights[0].shape[1]] + [w.shape[0] for w in weights]
    if (
        use_kernel(x)
        and x.dtype == torch.float32
        and x.dim() == 2
        and fusable(dims, wide)
        and all(w.dtype == torch.float32 for w in weights)
    ):
        if norm_mean is not None:
            norm_mean = norm_mean.detach().float().contiguous()
            norm_var = norm_var.detach().float().contiguous()
        params = []
        for w, b in zip(weights, biases):
            params += [w, b]
        fn = _TMLPFn if kernel_supports(dims) else _WideMLPFn
        return fn.apply(x, hidden_act, out_act, norm_mean, norm_var, norm_eps, *params)
    return tmlp_reference(x, weights, biases, hidden_act, out_act, norm_mean, norm_var, norm_eps)


# ----------------------------------------------------------------------------- grouped (ensembles)
def tmlp_grouped_reference(x: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor],
                           hidden_act: int, out_act: int = 0, norm_mean: Optional[torch.Tensor] = None,
                           norm_var: Optional[torch.Tensor] = None, norm_eps: float = 1e-5) -> torch.Tensor:
    """fp32 reference of :func:`tmlp_grouped`: ``x`` [B, din] (shared) or [G, B, din];
    ``weights[l]`` [G, out, in], ``biases[l]`` [G, out], norm stats [G, din] -> [G, B, out]."""
    G = weights[0].shape[0]
    h = x.unsqueeze(0).expand(G, -1, -1) if x.dim() == 2 else x
    if norm_mean is not None:
        h = (h - norm_mean[:, None, :]) / torch.sqrt(norm_var[:, None, :] + norm_eps)
    n = len(weights)
    for i, (w, b) in enumerate(zip(weights, biases)):
        h = torch.baddbmm(b[:, None, :], h, w.transpose(1, 2))
        h = _act(out_act if i == n - 1 else hidden_act, h)
    return h


class _TMLPGroupedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, hidden_act, out_act, mean, var, eps, *params):
        from imitation_amd.ops import native

        C = native()
        ws = [p.contiguous() for p in params[0::2]]
        bs = [p.contiguous() for p in params[1::2]]
        xc = x.contiguous()
        y = C.tmlp_forward_grouped(xc, ws, bs, int(hidden_act), int(out_act), mean, var, float(eps))
        ctx.cfg = (int(hidden_act), int(out_act), float(eps), mean is not None, len(ws))
        saved = [xc] + ws + bs
        if mean is not None:
            mv = torch.stack([mean, var])  # snapshot (a train-mode norm updates in place later)
            saved += [mv[0], mv[1]]
        ctx.save_for_backward(*saved)
        return y

    @staticmethod
    def backward(ctx, dy):
        from imitation_amd.ops import native

        hidden_act, out_act, eps, has_norm, L = ctx.cfg
        saved = ctx.saved_tensors
        x, ws, bs = saved[0], list(saved[1 : 1 + L]), list(saved[1 + L : 1 + 2 * L])
        mean = var = None
        if has_norm:
            mean, var = saved[1 + 2 * L], saved[2 + 2 * L]
        need_dx = bool(ctx.needs_input_grad[0]) and x.dim() == 3
        dx, dws, dbs = native().tmlp_backward_grouped(x, dy.contiguous(), ws, bs, hidden_act, out_act, mean, var, eps,
                                                      need_dx)
        grads = []
        for dw, db in zip(dws, dbs):
            grads += [dw, db]
        return (dx, None, None, None, None, None, *grads)


def tmlp_grouped(x: torch.Tensor, weights: Sequence[torch.Tensor], biases: Sequence[torch.Tensor], hidden_act: int,
                 out_act: int = 0, norm_mean: Optional[torch.Tensor] = None, norm_var: Optional[torch.Tensor] = None,
                 norm_eps: float = 1e-5) -> torch.Tensor:
    """G structurally identical MLPs (an ensemble) in ONE launch: ``grid.y`` = member, each
    with its own stacked weights / biases / input-norm statistics; ``x`` is shared
    ([B, din]) or per member ([G, B, din]). Differentiable w.r.t. the stacked parameters
    (and a per-member ``x``). GPU fp32 -> HIP kernel (csrc/kernels/tmlp.hip), else the
    batched-matmul reference."""
    from imitation_amd.ops import use_kernel

    dims = [weights[0].shape[2]] + [w.shape[1] for w in weights]
    if use_kernel(x) and x.dtype == torch.float32 and kernel_supports(dims) and all(w.dtype == torch.float32 for w in weights):
        if norm_mean is not None:
            norm_mean = norm_mean.detach().float().contiguous()
            norm_var = norm_var.detach().float().contiguous()
        params = []
        for w, b in zip(weights, biases):
            params += [w, b]
        return _TMLPGroupedFn.apply(x, hidden_act, out_act, norm_mean, norm_var, norm_eps, *params)
    return tmlp_grouped_reference(x, weights, biases, hidden_act, out_act, norm_mean, norm_var, norm_eps)

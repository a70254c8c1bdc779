"""Bradley-Terry preference loss over fragment pairs (HIP kernel ``csrc/kernels/pref.hip``).

``bradley_terry(r1, r2, prefs, discount, threshold, noise)`` with ``r1, r2`` of shape
``[P, L]`` (per-transition rewards of the two fragments of each pair) returns
``(mean BCE loss, probs [P])`` where ``probs`` is the modelled probability that
fragment 1 is preferred (reference ``PreferenceModel.probability`` +
``CrossEntropyRewardLoss``). GPU tensors run the fused kernel; CPU tensors run the
PyTorch reference below, which is also the kernel's numerics oracle.
"""

from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F

from imitation_amd.ops import native, use_kernel


def bradley_terry_probs_reference(r1: torch.Tensor, r2: torch.Tensor, discount: float, threshold: float,
                                  noise: float) -> torch.Tensor:
    if discount == 1:
        diff = (r2 - r1).sum(-1)
    else:
        disc = discount ** torch.arange(r1.shape[-1], device=r1.device, dtype=r1.dtype)
        diff = (disc * (r2 - r1)).sum(-1)
    diff = torch.clip(diff, -threshold, threshold)
    return noise * 0.5 + (1 - noise) * (1 / (1 + diff.exp()))


def _finite_probs(probs: torch.Tensor) -> torch.Tensor:
    """``F.binary_cross_entropy`` rejects NaN inputs with a RuntimeError on the CPU and a
    device-side assert on the GPU; a NaN reward model raises ``NonFiniteError`` here instead."""
    if not bool(torch.isfinite(probs).all()):
        from imitation_amd.utils.watchdog import NonFiniteError

        raise NonFiniteError("non-finite preference probabilities: the reward model's output is NaN/Inf")
    return probs


def bradley_terry_reference(r1, r2, prefs, discount: float = 1.0, threshold: float = 50.0, noise: float = 0.0):
    probs = _finite_probs(bradley_terry_probs_reference(r1, r2, discount, threshold, noise))
    return F.binary_cross_entropy(probs, prefs), probs


class _BTFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, r1, r2, prefs, discount, threshold, noise):
        C = native()
        probs, losses, coef = C.pref_loss_fwd(r1.contiguous(), r2.contiguous(), prefs.contiguous(), discount, threshold,
                                              noise)
        ctx.save_for_backward(coef)
        ctx.L = r1.shape[1]
        ctx.discount = discount
        ctx.mark_non_differentiable(probs)
        return losses.mean(), probs

    @staticmethod
    def backward(ctx, gloss, gprobs):
        (coef,) = ctx.saved_tensors
        d1, d2 = native().pref_loss_bwd(coef, gloss.reshape(1).float().contiguous(), ctx.L, ctx.discount)
        return d1, d2, None, None, None, None


def bradley_terry(r1: torch.Tensor, r2: torch.Tensor, prefs: torch.Tensor, discount: float = 1.0,
                  threshold: float = 50.0, noise: float = 0.0) -> Tuple[torch.Tensor, torch.Tensor]:
    prefs = prefs.to(device=r1.device, dtype=torch.float32)
    if use_kernel(r1, r2):
        return _BTFn.apply(r1.float(), r2.float(), prefs, float(discount), float(threshold), float(noise))
    return bradley_terry_reference(r1, r2, prefs, discount, threshold, noise)

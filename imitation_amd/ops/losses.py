"""Loss ops: BCE-with-logits (discriminator, K4), ``-log σ(-x)`` (GAIL reward, K7).

Numerically stable forms in fp32: ``bce(x, y) = max(x,0) - x·y + log1p(exp(-|x|))``
and ``-log σ(-x) = softplus(x)``. These are single elementwise passes; on the
GPU they are fused into the discriminator kernels of the device engine
(``csrc/kernels/engine.hip``); standalone they run as PyTorch elementwise ops.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F


def bce_with_logits(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Mean binary cross-entropy of ``labels`` under Bernoulli(σ(logits))."""
    return F.binary_cross_entropy_with_logits(logits, labels)


def neg_logsigmoid_neg(logits: torch.Tensor) -> torch.Tensor:
    """``-log σ(-logits)`` == ``softplus(logits)`` (GAIL generator reward)."""
    return F.softplus(logits)

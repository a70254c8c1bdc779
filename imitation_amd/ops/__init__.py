"""Device ops: Python entry points of the hand-written HIP/CDNA4 kernels.

Dispatch rule (one rule for every op in this package):

* GPU tensor  -> the HIP kernel from ``imitation_amd._C`` (built in-tree for
  gfx950). If the extension cannot be loaded on a GPU machine the call raises;
  there is no silent eager fallback.
* CPU tensor  -> the plain PyTorch fp32 reference implementation that lives next
  to the kernel wrapper. Those references double as the numerics oracles of the
  kernel tests (``tests/ops``).

``IMITATION_AMD_FUSED=0`` disables the kernels for A/B measurements (every op
then runs its PyTorch reference on the GPU as well).
"""

from __future__ import annotations

import os

import torch


def fused_enabled() -> bool:
    return os.environ.get("IMITATION_AMD_FUSED", "1") != "0"


def use_kernel(*tensors: torch.Tensor) -> bool:
    """True iff the HIP kernel path must be used for these tensors."""
    if not fused_enabled():
        return False
    return all(t is None or t.is_cuda for t in tensors) and any(t is not None and t.is_cuda for t in tensors)


def native():
    """The loaded ``_C`` extension (raises loudly if it is missing)."""
    from imitation_amd import _native

    return _native.load()


from imitation_amd.ops.mlp import ACT_CODES, act_code, tmlp, tmlp_reference  # noqa: E402

__all__ = ["fused_enabled", "use_kernel", "native", "tmlp", "tmlp_reference", "ACT_CODES", "act_code"]

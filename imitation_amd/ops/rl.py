"""RL update ops: GAE scan and the fused PPO clipped-surrogate loss.

``gae`` replaces SB3's host-side reversed Python loop over ``n_steps``
(``RolloutBuffer.compute_returns_and_advantage``): the HIP
kernel runs one lane per env and scans time backwards in registers.
"""

from __future__ import annotations

from typing import Tuple

import torch


def gae_reference(rewards, values, episode_starts, last_values, dones, gamma: float, lam: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Plain PyTorch GAE(γ, λ) over ``[T, N]`` arrays (SB3 semantics)."""
    T = rewards.shape[0]
    adv = torch.zeros_like(rewards)
    last = torch.zeros_like(last_values)
    for t in reversed(range(T)):
        if t == T - 1:
            nnt = 1.0 - dones
            nv = last_values
        else:
            nnt = 1.0 - episode_starts[t + 1]
            nv = values[t + 1]
        delta = rewards[t] + gamma * nv * nnt - values[t]
        last = delta + gamma * lam * nnt * last
        adv[t] = last
    return adv, adv + values


def gae(rewards, values, episode_starts, last_values, dones, gamma: float, lam: float) -> Tuple[torch.Tensor, torch.Tensor]:
    from imitation_amd.ops import native, use_kernel

    if use_kernel(rewards) and rewards.dtype == torch.float32:
        C = native()
        return C.gae(
            rewards.contiguous(),
            values.contiguous().float(),
            episode_starts.contiguous().float(),
            last_values.contiguous().float(),
            dones.contiguous().float(),
            float(gamma),
            float(lam),
        )
    return gae_reference(rewards, values, episode_starts, last_values, dones, gamma, lam)

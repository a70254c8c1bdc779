"""RL update ops: GAE scan and the fused PPO clipped-surrogate loss.

``gae`` replaces SB3's host-side reversed Python loop over ``n_steps``
(``RolloutBuffer.compute_returns_and_advantage``): the HIP
kernel gives each env one wave and runs the backward recurrence as a parallel affine
scan over 64 time chunks. ``random_permutations`` produces the PPO epochs' minibatch
orders without a sort (keyed Feistel bijections).
"""

from __future__ import annotations

from typing import Optional, Tuple

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


def gae(rewards, values, episode_starts, last_values, dones, gamma: float, lam: float,
        moments: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """GAE(γ, λ) advantages and returns. ``moments`` (optional ``[N, 4]`` fp32): per-env sums
    (ΣR, ΣR², ΣA, ΣA²) of the returns R and advantages A = R - V, for
    :func:`explained_variance_from_moments` (written by the same kernel pass)."""
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
            moments,
        )
    adv, ret = gae_reference(rewards, values, episode_starts, last_values, dones, gamma, lam)
    if moments is not None:
        moments.view(-1, 4).copy_(torch.stack([ret.sum(0), ret.square().sum(0), adv.sum(0), adv.square().sum(0)], 1))
    return adv, ret


def explained_variance_from_moments(moments, rows: int) -> float:
    """SB3 ``explained_variance(values, returns)`` = 1 - Var(R - V) / Var(R) (population
    variances) from the per-env moment sums of :func:`gae`; NaN when Var(R) == 0."""
    import numpy as np

    m = np.asarray(moments, dtype=np.float64).reshape(-1, 4).sum(0)
    var_r = m[1] / rows - (m[0] / rows) ** 2
    var_a = m[3] / rows - (m[2] / rows) ** 2
    return float("nan") if var_r == 0 else float(1.0 - var_a / var_r)


_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def _mix32(x):
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    return x ^ (x >> 16)


def random_permutations_reference(E: int, n: int, seed: int):
    """Host (numpy) twin of the ``perm_feistel`` kernel (csrc/kernels/rl.hip): row ``e`` of
    the ``[E, n]`` int32 result is the keyed 4-round Feistel permutation of ``0..n-1``
    with cycle walking. Bit-identical to the GPU kernel for the same ``seed``."""
    import numpy as np

    seed &= _M64
    bits = 2
    while (1 << bits) < n:
        bits += 2
    h = bits // 2
    mask = np.uint64((1 << h) - 1)
    out = np.empty((E, n), dtype=np.int32)
    for e in range(E):
        k01 = _splitmix64(seed ^ ((0xA24BAED4963EE407 * (e + 1)) & _M64))
        k23 = _splitmix64(k01)
        keys = [k01 & 0xFFFFFFFF, k01 >> 32, k23 & 0xFFFFFFFF, k23 >> 32]
        x = np.arange(n, dtype=np.uint64)
        todo = np.ones(n, dtype=bool)
        res = np.empty(n, dtype=np.uint64)
        while todo.any():
            lh, rh = x >> np.uint64(h), x & mask
            for k in keys:
                f = _mix32(rh ^ np.uint64(k)) & mask
                lh, rh = rh, lh ^ f
            x = (lh << np.uint64(h)) | rh
            done = todo & (x < np.uint64(n))
            res[done] = x[done]
            todo &= ~done
        out[e] = res.astype(np.int32)
    return out


def random_permutations(E: int, n: int, seed: int, device) -> torch.Tensor:
    """``[E, n]`` int32 minibatch orders (one permutation of the rows per epoch), keyed by
    ``seed``; replaces ``torch.randperm`` per epoch (a device radix sort) with one
    ``perm_feistel`` launch. Same values on the GPU kernel and the numpy fallback."""
    from imitation_amd.ops import native

    device = torch.device(device)
    seed = int(seed) & _M64
    if device.type == "cuda":
        s = seed - (1 << 64) if seed >= (1 << 63) else seed  # int64 two's complement for the binding
        return native().random_permutations(int(E), int(n), s, device)
    return torch.from_numpy(random_permutations_reference(E, n, seed))


def categorical_eval_reference(logits: torch.Tensor, actions: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(log π(a), entropy) of a categorical head from raw logits ``[B, A]`` (fp32 oracle)."""
    z = logits if logits.is_floating_point() else logits.float()
    lp = z - z.logsumexp(-1, keepdim=True)
    return lp.gather(-1, actions.long().reshape(-1, 1)).squeeze(-1), -(lp.exp() * lp).sum(-1)


class _CategoricalEval(torch.autograd.Function):
    """One-pass categorical ``evaluate_actions`` (rl.hip ``cat_eval_*``): logsumexp, gather,
    softmax and entropy fused forward, and the logit gradient
    ``dz = g_lp (onehot(a) - p) - g_ent p (log p + H)`` in one backward launch -- the ~10
    elementwise / reduce kernels of the unfused form become 2 (BC / PPO on Atari heads)."""

    @staticmethod
    def forward(ctx, logits, actions):
        from imitation_amd.ops import native

        z = logits.contiguous()
        a = actions.reshape(-1).long().contiguous()
        logp, ent = native().cat_eval_fwd(z, a)
        ctx.save_for_backward(z, a)
        return logp, ent

    @staticmethod
    def backward(ctx, g_lp, g_ent):
        from imitation_amd.ops import native

        z, a = ctx.saved_tensors
        return native().cat_eval_bwd(z, a, g_lp, g_ent), None


def categorical_eval(logits: torch.Tensor, actions: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(log π(a), entropy) per row from raw logits; HIP kernel on GPU fp32 with ≤64 actions."""
    from imitation_amd.ops import use_kernel

    if (use_kernel(logits) and logits.dtype == torch.float32 and logits.dim() == 2 and logits.shape[1] <= 64
            and actions.numel() == logits.shape[0]):
        return _CategoricalEval.apply(logits, actions)
    return categorical_eval_reference(logits, actions)


BC_METRICS = ("neglogp", "entropy", "ent_loss", "prob_true_act", "l2_norm", "l2_loss", "loss")


def bc_categorical_loss_reference(logits, actions, params, ent_weight: float, l2_weight: float) -> torch.Tensor:
    """The BC loss metrics of a categorical head as one ``[7]`` vector (order ``BC_METRICS``)."""
    lp, ent = categorical_eval_reference(logits, actions)
    l2 = torch.stack([p.square().sum() for p in params]).sum() / 2 if params else logits.new_zeros(())
    neglogp, entropy = -lp.mean(), ent.mean()
    ent_loss, l2_loss = -ent_weight * entropy, l2_weight * l2
    return torch.stack([neglogp, entropy, ent_loss, lp.exp().mean(), l2, l2_loss, neglogp + ent_loss + l2_loss])


class _BCCategoricalLoss(torch.autograd.Function):
    """rl.hip ``bc_cat_loss_*``: the whole BC loss of a categorical head (log-prob, entropy,
    means, prob_true_act, ||θ||²/2 over the flat parameter bucket, totals) as 2 forward
    launches and a 1-launch logit gradient. ``||θ||²`` is a logged metric only (the fused
    path is taken for ``l2_weight == 0``), so no parameter gradient flows from it."""

    @staticmethod
    def forward(ctx, logits, actions, flat, ent_weight, l2_weight):
        from imitation_amd.ops import native

        z = logits.contiguous()
        a = actions.reshape(-1).long().contiguous()
        out, loss = native().bc_cat_loss_fwd(z, a, flat, float(ent_weight), float(l2_weight))
        ctx.save_for_backward(z, a)
        ctx.ent_weight = float(ent_weight)
        ctx.set_materialize_grads(False)
        return out, loss

    @staticmethod
    def backward(ctx, g, g_loss):
        from imitation_amd.ops import native

        z, a = ctx.saved_tensors
        return native().bc_cat_loss_bwd(z, a, g, g_loss, ctx.ent_weight), None, None, None, None


def flat_param_view(params) -> "torch.Tensor | None":
    """A 1-D view over ``params`` when they are adjacent contiguous slices of one buffer in
    this order (FusedAdam's bucket layout), 16-B aligned; else None."""
    if not params:
        return None
    p0 = params[0]
    st = p0.untyped_storage()
    off = base = p0.storage_offset()
    for p in params:
        if (p.dtype != torch.float32 or not p.is_contiguous() or p.device != p0.device
                or p.untyped_storage().data_ptr() != st.data_ptr() or p.storage_offset() != off):
            return None
        off += p.numel()
    view = p0.new_empty(0).set_(st, base, (off - base,), (1,))
    return view if view.data_ptr() % 16 == 0 else None


def bc_categorical_loss(logits, actions, params, ent_weight: float, l2_weight: float,
                        flat: "torch.Tensor | None" = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """``(metrics [7], loss)``: the BC metric vector (``BC_METRICS`` order) and the loss as
    its own scalar, both differentiable w.r.t. the logits (backpropagating ``loss`` alone
    needs no zero-filled vector gradient). HIP kernels on the GPU when ``l2_weight == 0`` and
    the parameters form one flat buffer (``flat``), else the reference."""
    from imitation_amd.ops import use_kernel

    if (use_kernel(logits) and logits.dtype == torch.float32 and logits.dim() == 2 and 0 < logits.shape[1] <= 64
            and logits.shape[0] > 0 and actions.numel() == logits.shape[0] and l2_weight == 0.0 and flat is not None):
        return _BCCategoricalLoss.apply(logits, actions, flat.detach(), ent_weight, l2_weight)
    m = bc_categorical_loss_reference(logits, actions, params, ent_weight, l2_weight)
    return m, m[6]


def gather_rows(srcs, b: torch.Tensor, e: "torch.Tensor | None" = None, n_envs: int = 1, dst=None):
    """``[s[b * n_envs + e] for s in srcs]`` (or ``s[b]``) for row-major sources ``[R, ...]``:
    one HIP launch for every field on the GPU (csrc/kernels/gather.hip), torch indexing on
    the CPU. Out-of-range rows come back as zeros on the GPU. ``dst``: caller-owned outputs."""
    from imitation_amd.ops import native, use_kernel

    srcs = list(srcs)
    if use_kernel(b) and 0 < len(srcs) <= 8 and all(s.is_cuda and s.is_contiguous() for s in srcs):
        return native().gather_rows(srcs, b.long().contiguous(), None if e is None else e.long().contiguous(), int(n_envs),
                                    None if dst is None else list(dst))
    flat = b.long() if e is None else b.long() * n_envs + e.long()
    if dst is not None:
        for s, o in zip(srcs, dst):
            torch.index_select(s, 0, flat, out=o)
        return list(dst)
    return [s.index_select(0, flat) for s in srcs]

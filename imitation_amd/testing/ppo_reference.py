"""Plain PyTorch fp32 PPO update (SB3 ``PPO.train`` semantics) with a given permutation.

The numerics reference for the device PPO kernels (tests/engine, the data-parallel
device worker): minibatch advantage normalisation, clipped surrogate, value MSE,
entropy bonus, ``clip_grad_norm_`` and Adam(eps=1e-5), one optimizer step per
minibatch of ``batch`` rows taken in ``perm`` order.
"""

from __future__ import annotations

import torch as th


def torch_ppo_reference(gen, obs, acts, old_logp, adv, ret, perm, clip, lr, batch=None):
    import torch.nn.functional as F

    pol = gen.policy
    pol.set_training_mode(True)
    params = list(pol.parameters())
    opt = th.optim.Adam(params, lr=lr, eps=1e-5)
    B = int(batch or gen.batch_size)
    rows = obs.shape[0]
    for e in range(perm.shape[0]):
        for mb in range(rows // B):
            idx = perm[e, mb * B:(mb + 1) * B].long()
            v, lp, ent = pol.evaluate_actions(obs[idx], acts[idx])
            v = v.flatten()
            a = adv[idx]
            a = (a - a.mean()) / (a.std() + 1e-8)
            ratio = th.exp(lp - old_logp[idx])
            pl = -th.min(a * ratio, a * th.clamp(ratio, 1 - clip, 1 + clip)).mean()
            vl = F.mse_loss(ret[idx], v)
            el = -th.mean(ent)
            loss = pl + gen.ent_coef * el + gen.vf_coef * vl
            opt.zero_grad()
            loss.backward()
            th.nn.utils.clip_grad_norm_(params, gen.max_grad_norm)
            opt.step()

"""Batched reward ensembles: every member in one grouped launch (SURVEY §2.4 "ensemble parallelism").

The reference evaluates and trains the members of a :class:`RewardEnsemble` one after
another (``reward_nets.py:946-953`` ``predict_processed_all``,
``preference_comparisons.py:1415-1424`` ``EnsembleTrainer._train``) -- M x the launches
of one small MLP. Here structurally identical ``BasicRewardNet`` members are viewed as
ONE stacked MLP:

* :class:`EnsembleStack` gathers the members' Linear weights / biases into ``[M, out, in]``
  / ``[M, out]`` tensors and their input ``RunningNorm`` buffers into ``[M, din]``, and
  scatters trained values back; the members stay ordinary modules (checkpoints, state
  dicts and the sequential fallback are untouched);
* :func:`imitation_amd.ops.mlp.tmlp_grouped` runs all members over one input batch (or
  per-member batches, e.g. bootstrap bags) in ONE kernel launch, ``grid.y`` = member,
  forward and backward;
* the input-norm update of all members is one vectorised Chan merge over the stacked
  buffers.
"""

from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch as th

from imitation_amd.util import networks


def _member_plan(member) -> Optional[dict]:
    from imitation_amd.rewards import reward_nets

    if type(member) is not reward_nets.BasicRewardNet or not isinstance(member.mlp, networks.MLP):
        return None
    plan = member.mlp._fusion_plan()
    if not plan or plan["has_dropout"] or plan["flatten"]:
        return None
    norm = plan["norm"]
    if norm is not None and type(norm) is not networks.RunningNorm:
        return None
    return plan


class EnsembleStack:
    """Stacked view of the members of a :class:`~imitation_amd.rewards.reward_nets.RewardEnsemble`."""

    def __init__(self, members: Sequence, plans: Sequence[dict]):
        self.members = list(members)
        self.plans = list(plans)
        p0 = plans[0]
        self.hidden_act, self.out_act = p0["hidden_act"], p0["out_act"]
        self.n_layers = len(p0["linears"])
        self.has_norm = p0["norm"] is not None
        self.eps = p0["norm"].eps if self.has_norm else 1e-5

    @staticmethod
    def build(ensemble) -> Optional["EnsembleStack"]:
        """The stack of ``ensemble``'s members, or None when they are not structurally
        identical fusable ``BasicRewardNet`` MLPs."""
        members = list(ensemble.members)
        plans = [_member_plan(m) for m in members]
        if any(p is None for p in plans):
            return None
        m0, p0 = members[0], plans[0]
        sig = lambda m, p: (m.use_state, m.use_action, m.use_next_state, m.use_done, p["hidden_act"], p["out_act"],  # noqa: E731
                            p["squeeze"], p["norm"] is not None,
                            tuple((l.in_features, l.out_features) for l in p["linears"]),
                            p["norm"].eps if p["norm"] is not None else None)
        if any(sig(m, p) != sig(m0, p0) for m, p in zip(members, plans)):
            return None
        dev = {t.device for m in members for t in m.parameters()}
        if len(dev) != 1:
            return None
        return EnsembleStack(members, plans)

    # ------------------------------------------------------------------ gather / scatter
    def gather_params(self) -> List[th.Tensor]:
        """[W_0 [M,out,in], b_0 [M,out], W_1, b_1, ...] (fresh stacked copies)."""
        out: List[th.Tensor] = []
        for l in range(self.n_layers):
            out.append(th.stack([p["linears"][l].weight.detach() for p in self.plans]))
            out.append(th.stack([p["linears"][l].bias.detach() for p in self.plans]))
        return out

    def gather_norm(self) -> Optional[Tuple[th.Tensor, th.Tensor, th.Tensor]]:
        """(mean [M, din], var [M, din], count [M] float64) or None."""
        if not self.has_norm:
            return None
        norms = [p["norm"] for p in self.plans]
        return (th.stack([n.running_mean for n in norms]), th.stack([n.running_var for n in norms]),
                th.stack([n.count for n in norms]).double())

    @th.no_grad()
    def scatter(self, params: Sequence[th.Tensor], norm: Optional[Tuple[th.Tensor, th.Tensor, th.Tensor]] = None) -> None:
        """Write stacked values back into the member modules."""
        for m, p in enumerate(self.plans):
            for l, lin in enumerate(p["linears"]):
                lin.weight.copy_(params[2 * l][m])
                lin.bias.copy_(params[2 * l + 1][m])
            if norm is not None:
                n = p["norm"]
                n.running_mean.copy_(norm[0][m])
                n.running_var.copy_(norm[1][m])
                n.count.copy_(norm[2][m].to(n.count.dtype))

    # ------------------------------------------------------------------ compute
    def features(self, state: th.Tensor, action: th.Tensor, next_state: th.Tensor, done: th.Tensor) -> th.Tensor:
        """The members' common MLP input (``BasicRewardNet.forward``'s concatenation)."""
        m = self.members[0]
        parts = []
        if m.use_state:
            parts.append(th.flatten(state, 1))
        if m.use_action:
            parts.append(th.flatten(action, 1))
        if m.use_next_state:
            parts.append(th.flatten(next_state, 1))
        if m.use_done:
            parts.append(th.reshape(done, [-1, 1]))
        x = th.cat(parts, dim=1) if len(parts) > 1 else parts[0]
        return x.float()

    def forward(self, x: th.Tensor, params: Sequence[th.Tensor], norm=None) -> th.Tensor:
        """Every member's reward for ``x`` [B, din] (shared) or [M, B, din] -> [M, B]."""
        from imitation_amd.ops import mlp as mlp_ops

        mean = var = None
        if norm is not None:
            mean, var = norm[0], norm[1]
        y = mlp_ops.tmlp_grouped(x, params[0::2], params[1::2], self.hidden_act, self.out_act, mean, var, self.eps)
        return y.squeeze(-1)

    @staticmethod
    @th.no_grad()
    def update_norm(norm: Tuple[th.Tensor, th.Tensor, th.Tensor], x: th.Tensor) -> None:
        """RunningNorm.update_stats of every member at once: ``x`` [M, n, din] (each member's
        batch), Chan merge on the stacked buffers (moments all-reduced under DP)."""
        from imitation_amd.parallel import dist as pdist

        mean, var, count = norm
        n = float(x.shape[1])
        if pdist.norm_sync_active():
            xd = x.double()
            msg = th.cat([xd.sum(1), (xd * xd).sum(1)], dim=1)
            pdist.allreduce_sum_(msg)
            n_tot = n * pdist.world_size()
            d = x.shape[2]
            bmean = (msg[:, :d] / n_tot)
            bvar = (msg[:, d:] / n_tot - bmean * bmean).clamp_min(0.0)
            bmean, bvar, n = bmean.to(mean.dtype), bvar.to(mean.dtype), n_tot
        else:
            bmean = x.mean(1)
            bvar = x.var(1, unbiased=False)
        c = count[:, None].to(mean.dtype)
        tot = c + n
        delta = bmean - mean
        mean += delta * n / tot
        var.mul_(c).add_(bvar * n).add_(delta.square() * c * n / tot).div_(tot)
        count += n

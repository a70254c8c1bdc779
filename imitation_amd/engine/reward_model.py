"""Fused preference reward-model minibatch (csrc/kernels/pref_rm.hip).

One minibatch of ``BasicRewardTrainer`` (reference
``src/imitation/algorithms/preference_comparisons.py:1255-1282``: reward net over the pairs'
fragments, Bradley-Terry probability ``:411-530``, ``CrossEntropyRewardLoss`` ``:1050-1090``
scaled by ``n / batch_size``, backward, AdamW) as four launches -- gather, forward with the
input RunningNorm merge, Bradley-Terry + backward, AdamW with the fixed-order gradient
reduction -- reading the device-resident fragment store of ``_MinibatchGraph`` and updating
the reward net's parameters, normaliser and the optimizer's flat buffers in place.

Applies to a single ``BasicRewardNet`` (MLP of <= 4 layers, widths <= 64, scalar identity
head, optional RunningNorm input layer) trained by a one-group :class:`~imitation_amd.ops.optim.FusedAdam`
over exactly its MLP parameters; ``IMITATION_AMD_PREF_FUSED=0`` keeps the autograd step.
"""

from __future__ import annotations

import os
from typing import Optional, Tuple

import torch as th

from imitation_amd.ops import optim as optim_ops
from imitation_amd.rewards import reward_nets
from imitation_amd.util import networks


def fused_check(trainer) -> Tuple[bool, str]:
    """Whether the reward trainer's minibatch can run on the fused kernels (and why not)."""
    from imitation_amd.engine.gail import _mlp_layers

    if os.environ.get("IMITATION_AMD_PREF_FUSED", "1") == "0":
        return False, "disabled (IMITATION_AMD_PREF_FUSED=0)"
    net = trainer._preference_model.model
    if type(net) is not reward_nets.BasicRewardNet:
        return False, "reward net is not a BasicRewardNet"
    opt = trainer.optim
    if not isinstance(opt, optim_ops.FusedAdam) or len(opt.param_groups) != 1:
        return False, "optimizer is not a one-group FusedAdam"
    g = opt.param_groups[0]
    if g.get("maximize"):
        return False, "maximize"
    try:
        norm, lins, hidden, out_act = _mlp_layers(net.mlp)
    except ValueError as e:
        return False, str(e)
    if norm is not None and type(norm) is not networks.RunningNorm:
        return False, "input normaliser is not RunningNorm"
    if out_act != 0 or lins[-1].out_features != 1 or len(lins) > 4:
        return False, "reward MLP shape"
    if max([l.out_features for l in lins[:-1]] + [lins[0].in_features]) > 64:
        return False, "reward MLP wider than 64 (or more than 64 input columns)"
    order = [p for l in lins for p in (l.weight, l.bias)]
    if [id(p) for p in opt._flat[0]["params"]] != [id(p) for p in order]:
        return False, "optimizer parameters are not exactly the MLP's (W0, b0, W1, b1, ...)"
    if not lins[0].weight.is_cuda:
        return False, "reward net not on the GPU"
    return True, ""


def build_plan(trainer, store, L: int, capacity: int):
    """A ``PrefRmPlan`` over the fragment store ``store`` (a ``_MinibatchGraph``)."""
    from imitation_amd import ops
    from imitation_amd.engine.gail import _mlp_layers

    pm = trainer._preference_model
    net = pm.model
    norm, lins, hidden, _ = _mlp_layers(net.mlp)
    opt = trainer.optim
    f = opt._flat[0]
    g = opt.param_groups[0]
    rows = store.s.shape[0]
    flat2 = lambda t: t.reshape(rows, -1)  # noqa: E731
    s2, a2, ns2 = flat2(store.s), flat2(store.a), flat2(store.ns)
    d = dict(L=L, batch=trainer.batch_size, capacity=capacity,
             ds=s2.shape[1] if net.use_state else 0, da=a2.shape[1] if net.use_action else 0,
             dns=ns2.shape[1] if net.use_next_state else 0, use_done=int(net.use_done),
             s_all=s2 if net.use_state else None, a_all=a2 if net.use_action else None,
             ns_all=ns2 if net.use_next_state else None, d_all=store.d_f if net.use_done else None,
             prefs_all=store.prefs, gt_all=store.gt.reshape(-1) if store.gt is not None else None,
             net=dict(W=[l.weight for l in lins], b=[l.bias for l in lins], hidden_act=int(hidden)),
             rmean=norm.running_mean if norm is not None else None, rvar=norm.running_var if norm is not None else None,
             rcount=norm.count if norm is not None else None, eps=float(norm.eps) if norm is not None else 1e-5,
             discount=float(pm.discount_factor), threshold=float(pm.threshold), noise=float(pm.noise_prob),
             params=f["flat"], exp_avg=f["m"], exp_avg_sq=f["v"], step=f["step"], lr=float(g["lr"]),
             beta1=float(g["betas"][0]), beta2=float(g["betas"][1]), adam_eps=float(g["eps"]),
             weight_decay=float(g["weight_decay"]), decoupled=bool(g["decoupled_weight_decay"]))
    return ops.native().PrefRmPlan(d), norm


class FusedMinibatch:
    """``step(idx) -> metrics`` of one reward-model minibatch on the fused kernels.

    Data parallel (each rank its slice of the global minibatch, as the autograd fast path):
    the RunningNorm block sums are all-reduced between the gather and the forward when
    normaliser statistics are synchronised, and the reduced gradient before AdamW -- two
    collectives. On the one-shot IPC all-reduce (both buffers fit its staging slot) they are
    capturable and the DP step is graph-replayed like the single-rank one; over RCCL / gloo
    the step runs eagerly (``capturable`` False)."""

    def __init__(self, trainer, store, L: int, capacity: int):
        from imitation_amd.parallel import dist as pdist

        self.trainer = trainer
        self.L = L
        self.plan, self.norm = build_plan(trainer, store, L, capacity)
        self.n_metrics = 3 if store.gt is not None else 2
        self.world = pdist.world_size()
        self.capturable = self.world == 1 or self._oneshot_ok()

    def _oneshot_ok(self) -> bool:
        from imitation_amd.parallel import dist as pdist

        if not pdist.oneshot_active():
            return False
        from imitation_amd.parallel import oneshot

        return all(oneshot._COMM.fits(t) for t in (self.plan.sums, self.plan.grads))

    def step(self, idx: th.Tensor) -> th.Tensor:
        from imitation_amd.parallel import dist as pdist

        merge = self.norm is not None and self.norm.training
        plan = self.plan
        if self.world == 1:
            return plan.step(idx, merge)[: self.n_metrics]
        sync = self.norm is not None and pdist.norm_sync_active()
        plan.gather(idx, merge)
        if sync:
            pdist.allreduce_sum_(plan.sums)
        plan.forward(idx, merge, self.world * 2 * self.L * int(idx.shape[0]) if sync else 0)
        plan.backward(idx, merge)
        pdist.allreduce_grads_flat(plan.grads)
        plan.apply(idx)
        return plan.metrics[: self.n_metrics]


def maybe_fused(trainer, store, L: int, capacity: int) -> Optional[FusedMinibatch]:
    ok, _ = fused_check(trainer)
    return FusedMinibatch(trainer, store, L, capacity) if ok else None

"""Fused BC minibatch of a NatureCNN categorical policy (the DAgger-Pong learner).

Reference: ``src/imitation/algorithms/bc.py:443-510`` (``BehaviorCloningLossCalculator``:
``policy.evaluate_actions`` -> ``-log_prob.mean()``, ``-ent_weight * entropy.mean()``, the
``||theta||^2 / 2`` metric; ``loss.backward()``; ``optimizer.step()``), with the SB3
``ActorCriticCnnPolicy`` (``NatureCNN`` features, ``net_arch=[]``, ``action_net`` Linear) of
the reference's ``cnn_policy`` config.

One step without autograd, every gradient written straight into the ``FusedAdam`` bucket:

* one launch packs every bf16 GEMM layout (conv weights, the FC weight in NHWC column order,
  their transposed data-gradient images);
* three conv+ReLU MFMA launches on the uint8 frames (``/255`` folded into the first layer's
  operand load) and the 512-unit FC+ReLU (``cnn_fc``);
* ONE head launch (``bc_head.hip``): logits, log-softmax, entropy, the seven BC metrics,
  ``dL/dlogits``, ``dW`` / ``db`` of ``action_net`` into the bucket, ``dL/dh`` and the
  ``||theta||^2`` reduction over the whole parameter bucket;
* the FC backward (dW, db into the bucket; dX in NHWC) and the conv stack backward (weight
  gradient partials per layer, their fixed-order reductions into the bucket as ONE launch;
  data gradients with the ReLU masks fused);
* the optimizer step is the caller's (one ``adam_flat`` launch).

The value head is not evaluated: BC never uses it, and its bucket slice stays zero, as its
``.grad`` would. Numerics: bf16 MFMA operands with fp32 accumulation in the trunk (as the
autograd path of ``ops/conv.py``), fp32 head.
"""

from __future__ import annotations

from typing import Any, Dict, List, Optional

import torch as th
from torch import nn

METRICS = ("neglogp", "entropy", "ent_loss", "prob_true_act", "l2_norm", "l2_loss", "loss")


def _grad_views(optimizer) -> Optional[Dict[int, th.Tensor]]:
    from imitation_amd.ops import optim as optim_ops

    if not isinstance(optimizer, optim_ops.FusedAdam) or len(optimizer._flat) != 1 or not optimizer._flat[0]["n"]:
        return None
    f = optimizer._flat[0]
    return {id(p): gv for p, (_, _, gv) in zip(f["params"], f["views"])}


class FusedCnnBCStep:
    """``step(obs_u8, acts) -> metrics [8]`` (``METRICS`` order) with the gradients of every
    policy parameter in ``optimizer``'s bucket. Build with :meth:`maybe`."""

    def __init__(self, policy, optimizer, ent_weight: float, l2_weight: float):
        from imitation_amd import ops

        self.C = ops.native()
        self.policy = policy
        self.optimizer = optimizer
        self.ent_weight, self.l2_weight = float(ent_weight), float(l2_weight)
        fe = policy.features_extractor
        self.convs: List[nn.Conv2d] = [m for m in fe.cnn if isinstance(m, nn.Conv2d)]
        self.lin: nn.Linear = fe.linear[0]
        self.head: nn.Linear = policy.action_net
        views = _grad_views(optimizer)
        self.g_conv = [(views[id(c.weight)], views[id(c.bias)]) for c in self.convs]
        self.g_lin = (views[id(self.lin.weight)], views[id(self.lin.bias)])
        self.g_head = (views[id(self.head.weight)], views[id(self.head.bias)])
        self.flat = optimizer._flat[0]["flat"]
        dev = self.flat.device
        self.metrics = th.zeros(8, device=dev)
        self.ws = th.zeros(int(self.C.bc_head_workspace(self.flat.numel())), device=dev)  # word 0: counter

    @staticmethod
    def maybe(policy, optimizer, obs, ent_weight: float, l2_weight: float) -> Optional["FusedCnnBCStep"]:
        """The fused step when it reproduces the loss calculator exactly, else None."""
        import os

        from imitation_amd import ops
        from imitation_amd.ops import conv as conv_ops
        from imitation_amd.rl.distributions import CategoricalDistribution
        from imitation_amd.rl.policies import ActorCriticPolicy
        from imitation_amd.rl.preprocessing import is_image_space
        from imitation_amd.rl.torch_layers import NatureCNN

        if os.environ.get("IMITATION_AMD_BC_CNN_FUSED", "1") == "0" or l2_weight != 0.0:
            return None
        if not (isinstance(policy, ActorCriticPolicy) and isinstance(obs, th.Tensor) and ops.use_kernel(obs)):
            return None
        if not (isinstance(policy.action_dist, CategoricalDistribution) and policy.share_features_extractor
                and isinstance(policy.features_extractor, NatureCNN) and policy.normalize_images
                and is_image_space(policy.observation_space)):
            return None
        fe = policy.features_extractor
        if not fe.raw_frames_ok(obs) or len(fe.linear) != 2 or not isinstance(fe.linear[1], nn.ReLU):
            return None
        if len(policy.mlp_extractor.policy_net) != 0 or not isinstance(policy.action_net, nn.Linear):
            return None
        convs = [m for m in fe.cnn if isinstance(m, nn.Conv2d)]
        lin = fe.linear[0]
        if not conv_ops.fc_supported(tuple(obs.shape), [c.weight for c in convs], [c.stride[0] for c in convs],
                                     lin.out_features):
            return None
        B, NH, A = obs.shape[0], lin.out_features, policy.action_net.out_features
        if not (0 < B <= 64 and NH in (256, 512) and 0 < A <= 8):
            return None
        views = _grad_views(optimizer)
        if views is None or any(id(p) not in views for p in policy.parameters()):
            return None
        flat = optimizer._flat[0]["flat"]
        if any(t.data_ptr() % 16 for t in (flat, policy.action_net.weight)):
            return None
        return FusedCnnBCStep(policy, optimizer, ent_weight, l2_weight)

    # the convs' forward in the split-K form (conv_forward_sk: 16 x 16 tiles over 2-4 waves, all of a
    # wave's loads at once); False: the default form (A/B hook)
    splitk_fwd = True

    def __call__(self, obs: th.Tensor, acts: th.Tensor, after_fc=None, gather=None, defer_reduce: bool = False) -> th.Tensor:
        """``after_fc``: called (no arguments) once the FC layer's gradients are in the bucket and
        before the conv backward -- the data-parallel epoch starts the FC bucket's all-reduce there,
        on a side stream, so it overlaps the conv backward. ``gather``: ``(srcs, perm, cursor, n,
        [obs, acts], step_counter)`` of the minibatch's ``gather_rows_cursor``, run inside the
        weight-packing launch (one dispatch fewer per step); ``obs`` / ``acts`` are its outputs.
        ``defer_reduce``: the conv weight-gradient reductions are not launched; their arguments are
        left in ``self.pending_reduce`` for the optimizer step to run them in its own launch
        (``FusedAdam.step(reduce=...)``) -- only when :attr:`reduce_foldable`."""
        if gather is not None and not (obs.is_contiguous() and acts.is_contiguous()):
            raise ValueError("the fused gather writes obs / acts in place: they must be contiguous")
        C = self.C
        convs, lin, head = self.convs, self.lin, self.head
        n = len(convs)
        x = obs.contiguous()
        B = x.shape[0]
        H, W = x.shape[1], x.shape[2]
        for c in convs:
            H, W = (H - c.kernel_size[0]) // c.stride[0] + 1, (W - c.kernel_size[1]) // c.stride[0] + 1
        C3, NH = convs[-1].out_channels, lin.out_features
        with th.no_grad():
            wsrc = [c.weight.detach() for c in convs] + [lin.weight.detach().view(NH, C3, H, W)]
            wbs, wts = C.conv_pack_weights(wsrc, [i > 0 for i in range(n)] + [True], [False] * n + [True], gather)
            hs: List[th.Tensor] = []
            h = x
            for i, c in enumerate(convs):
                h = C.conv_fwd(h, wbs[i], c.bias.detach(), int(c.stride[0]), 1.0 / 255.0 if i == 0 else 1.0, True, 0,
                               self.splitk_fwd)
                hs.append(h)
            xf = h.reshape(B, -1)
            out = C.cnn_fc(xf, wbs[n].view(NH, -1), lin.bias.detach())
            a = acts.reshape(-1).long().contiguous()
            dh = C.bc_head_train(out, head.weight.detach(), head.bias.detach(), a, self.flat, self.g_head[0], self.g_head[1],
                                 self.metrics, self.ws, self.ent_weight, self.l2_weight)
            _, _, dx = C.fc_backward(xf, dh, out, wts[n], C3, True, self.g_lin[0], self.g_lin[1])
            if after_fc is not None:
                after_fc()
            dz = dx.view(hs[-1].shape)
            # weight-gradient partials per layer; their fixed-order reductions in ONE launch at the end
            red = {k: [] for k in ("x", "dy", "kh", "kw", "s", "p", "slab", "dw", "db")}
            pair = self._pairs(x, hs)
            for i in range(n - 1, -1, -1):
                c = convs[i]
                inp = x if i == 0 else hs[i - 1]
                top = i == n - 1  # relu_out: the top conv's ReLU mask is applied to dZ in the loads
                kh, kw, st = int(c.kernel_size[0]), int(c.kernel_size[1]), int(c.stride[0])
                if i > 0 and pair[i]:
                    # this layer's weight-gradient partials and data gradient in ONE launch (they
                    # read the same dZ and neither feeds the other)
                    slab, dz_next = C.conv_backward_pair(inp, dz, hs[i], wts[i], st, top)
                else:
                    slab = C.conv_wgrad_partials(inp, dz, hs[i], kh, kw, st, 1.0 / 255.0 if i == 0 else 1.0, top, 0)
                    dz_next = C.conv_dgrad(dz, hs[i], wts[i], hs[i - 1], st, top, True, 0) if i > 0 else None
                for k, v in zip(red, (inp, dz, kh, kw, st, 0, slab, self.g_conv[i][0], self.g_conv[i][1])):
                    red[k].append(v)
                dz = dz_next
            if defer_reduce:
                self.pending_reduce = tuple(red.values())
            else:
                C.conv_reduce_multi(*red.values())
        return self.metrics

    @property
    def reduce_foldable(self) -> bool:
        """Whether every conv layer's dW / db slot is a whole number of 16-B quads of the flat
        gradient buffer (the fused Adam launch's column blocks own exactly those quads)."""
        base = self.optimizer._flat[0]["grad"].data_ptr()
        return all((t.data_ptr() - base) % 16 == 0 and t.numel() % 4 == 0 for pair in self.g_conv for t in pair)


    def _pairs(self, x: th.Tensor, hs: List[th.Tensor]) -> List[bool]:
        """Per conv layer: whether its backward runs as one paired launch (bf16 input, BC-size batch;
        0.159 -> 0.145 ms per batch-32 step against the separate wgrad / dgrad launches,
        ``profiles/r6_bc_step.md``)."""
        key = (tuple(x.shape), len(hs))
        cached = getattr(self, "_pair_key", None)
        if cached is not None and cached[0] == key:
            return cached[1]
        out = [False]
        for i in range(1, len(self.convs)):
            c = self.convs[i]
            out.append(bool(self.C.conv_backward_pair_ok(hs[i - 1], c.out_channels, int(c.kernel_size[0]),
                                                                int(c.kernel_size[1]), int(c.stride[0]))))
        self._pair_key = (key, out)
        return out


def metrics_fields(m: th.Tensor) -> Dict[str, Any]:
    """``BCTrainingMetrics`` keyword arguments from the metric vector."""
    return {k: m[i] for i, k in enumerate(METRICS)}

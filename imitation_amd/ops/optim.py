"""Fused flat-buffer Adam / AdamW (SURVEY §2.2 "fused optimizer step", K26).

The reference trains with ``th.optim.Adam`` (BC ``bc.py:284``, discriminator
``common.py:123``) and ``th.optim.AdamW`` (preference reward ``preference_comparisons.py:1192``).
PyTorch's capturable foreach Adam is ~8 multi-tensor launches per step; for the KB-MB
models here those launches ARE the optimizer's cost. :class:`FusedAdam` re-points every
parameter of a group at a view of ONE contiguous fp32 buffer (and every ``.grad`` at a
view of one gradient buffer, which is also the natural DP all-reduce bucket), so a step
is ONE ``adam_flat`` launch (csrc/kernels/optim.hip) that also advances the device step
counter and clears the gradient it consumed. Everything lives on
the device, so the step is HIP-graph capturable.

On the CPU the same update runs as plain torch ops (numerics tests compare both against
``th.optim.Adam`` / ``AdamW``). ``state_dict`` has torch's per-parameter layout
(``step`` / ``exp_avg`` / ``exp_avg_sq``), so checkpoints interchange with torch Adam.
"""

from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional

import torch as th


class FusedAdam(th.optim.Optimizer):
    """Adam (``decoupled_weight_decay=False``) or AdamW over flat per-group buffers."""

    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, amsgrad: bool = False, *, maximize: bool = False,
                 decoupled_weight_decay: bool = False, capturable: bool = True, foreach: Optional[bool] = None,
                 differentiable: bool = False, fused: Optional[bool] = None):
        if amsgrad:
            raise ValueError("FusedAdam does not implement amsgrad")
        if differentiable:
            raise ValueError("FusedAdam is not differentiable")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=maximize,
                        decoupled_weight_decay=decoupled_weight_decay, capturable=True)
        super().__init__(params, defaults)
        self._flat: List[Dict[str, Any]] = []
        self._seeds: Dict[Any, th.Tensor] = {}
        for group in self.param_groups:
            self._flat.append(self._pack_group(group))

    # ------------------------------------------------------------------ layout
    def _pack_group(self, group) -> Dict[str, Any]:
        ps = [p for p in group["params"]]
        if not ps:
            return {"params": [], "n": 0}
        dev = ps[0].device
        if any(p.device != dev or p.dtype != th.float32 for p in ps):
            raise ValueError("FusedAdam needs fp32 parameters on one device")
        n = sum(p.numel() for p in ps)
        pad = (-n) % 4  # float4 kernel access
        flat = th.zeros(n + pad, device=dev)
        grad = th.zeros(n + pad, device=dev)
        m = th.zeros(n + pad, device=dev)
        v = th.zeros(n + pad, device=dev)
        step = th.zeros(1, device=dev)
        views = []
        off = 0
        for p in ps:
            k = p.numel()
            flat[off : off + k].copy_(p.detach().reshape(-1))
            if p.grad is not None:
                grad[off : off + k].copy_(p.grad.detach().reshape(-1))
            p.data = flat[off : off + k].view_as(p)
            gv = grad[off : off + k].view_as(p)
            p.grad = gv
            views.append((off, k, gv))
            self.state[p] = {"step": step, "exp_avg": m[off : off + k].view_as(p), "exp_avg_sq": v[off : off + k].view_as(p)}
            off += k
        # hand-off counter of the kernel's own step increment (stays zero between launches)
        cnt = th.zeros(1, dtype=th.int32, device=dev)
        return {"params": ps, "flat": flat, "grad": grad, "m": m, "v": v, "step": step, "views": views, "n": n, "cnt": cnt}

    @property
    def flat_grads(self) -> List[th.Tensor]:
        """The gradient bucket of every group (what a DP all-reduce should reduce)."""
        return [f["grad"] for f in self._flat if f["n"]]

    def _bind_grads(self, f: Dict[str, Any]) -> None:
        """Re-point ``.grad`` at the bucket views if something replaced them (e.g. a module's
        ``zero_grad()`` set them to None or autograd installed a fresh tensor)."""
        for p, (off, k, gv) in zip(f["params"], f["views"]):
            g = p.grad
            if g is None:
                gv.zero_()
            elif g.data_ptr() != gv.data_ptr():
                gv.copy_(g)
            else:
                continue
            p.grad = gv

    def zero_grad(self, set_to_none: bool = True) -> None:
        """Zero the gradient buckets; ``.grad`` stays bound to them (``set_to_none`` is moot)."""
        for f in self._flat:
            if f["n"]:
                f["grad"].zero_()
                self._bind_grads(f)

    def backward_into_buckets(self, loss: th.Tensor) -> None:
        """``loss.backward()`` for buckets that are zero on entry (after ``zero_grad()`` or a
        ``step()``, which clears what it consumed): the gradients are taken with
        ``autograd.grad`` and written into the bucket with one copy launch per run of
        adjacent parameters that received one, instead of one accumulate-add launch per
        parameter. Parameters without a gradient keep their zero slice."""
        live = [(f, i) for f in self._flat if f["n"] for i in range(len(f["params"]))]
        params = [f["params"][i] for f, i in live]
        # a persistent unit seed: no fill launch per step (and graph-capturable)
        seed = self._seeds.get((loss.device, loss.dtype, tuple(loss.shape)))
        if seed is None:
            seed = self._seeds[(loss.device, loss.dtype, tuple(loss.shape))] = th.ones_like(loss)
        grads = th.autograd.grad(loss, params, grad_outputs=seed, allow_unused=True)
        run: List[th.Tensor] = []
        start = end = 0
        cur = None

        def flush():
            if run:
                dst = cur["grad"][start:end]
                if len(run) == 1:
                    dst.copy_(run[0].reshape(-1))
                else:
                    th.cat([g.reshape(-1) for g in run], out=dst)

        for (f, i), g in zip(live, grads):
            off, k, _ = f["views"][i]
            if g is None or f is not cur or off != end:
                flush()
                run, cur, start, end = [], f, off, off
            if g is not None:
                run.append(g)
                end = off + k
            else:
                start = end = off + k
        flush()
        for f in self._flat:
            if f["n"]:
                self._bind_grads(f)

    # ------------------------------------------------------------------ step
    def graph_epoch_step_ok(self) -> bool:
        """Whether :meth:`step` can take ``step_incremented`` / ``append`` (one flat GPU group on
        the kernel path): the graphed BC epoch then folds the step-counter add into its gather
        launch and its metrics append into the Adam launch."""
        from imitation_amd import ops

        live = [f for f in self._flat if f["n"]]
        return len(live) == 1 and live[0]["flat"].is_cuda and ops.use_kernel(live[0]["flat"])

    def step_counter(self) -> th.Tensor:
        """The device step counter of the (single) flat group."""
        return next(f for f in self._flat if f["n"])["step"]

    @th.no_grad()
    def step(self, closure=None, step_incremented: bool = False, append=None, reduce=None, zero_grad: bool = True):
        """``step_incremented``: the step counter was already advanced for this step (by the
        caller's own launch). ``append``: ``(src, all, cursor)`` -- after the update, block 0 of
        the Adam launch copies ``src`` into row ``*cursor`` of ``all`` and advances the cursor.
        ``reduce``: ``conv_reduce_multi``'s nine argument lists -- those conv weight-gradient
        reductions run inside the Adam launch, their gradient slots summed from the slabs before
        their update (bitwise the two launches). All three need :meth:`graph_epoch_step_ok`.
        ``zero_grad=False``: the kernel leaves the gradient bucket as it is (one 4-B store per
        parameter less) -- for callers whose next backward rewrites every slot it reads."""
        loss = None
        if closure is not None:
            with th.enable_grad():
                loss = closure()
        from imitation_amd import ops

        for group, f in zip(self.param_groups, self._flat):
            if not f["n"]:
                continue
            self._bind_grads(f)
            b1, b2 = group["betas"]
            if f["flat"].is_cuda and ops.use_kernel(f["flat"]):
                # small buckets: the kernel advances the device step counter itself (no separate
                # add launch); large ones keep the add -- the one-counter hand-off costs ~12 ns per
                # arriving block (1,640 blocks for NatureCNN's 1.7M parameters: 11 -> 25 us)
                small = f["flat"].numel() <= 64 * 1024 and not step_incremented
                if not small and not step_incremented:
                    f["step"].add_(1.0)
                app = append if append is not None else (None, None, None)
                ops.native().adam_flat(f["flat"], f["grad"], f["m"], f["v"], f["step"], float(group["lr"]), float(b1),
                                       float(b2), float(group["eps"]), float(group["weight_decay"]),
                                       bool(group["decoupled_weight_decay"]), bool(group["maximize"]), bool(zero_grad),
                                       f["cnt"] if small else None, app[0], app[1], app[2], reduce)
            else:
                if step_incremented or append is not None or reduce is not None:
                    raise ValueError("step_incremented / append / reduce need the kernel path (graph_epoch_step_ok)")
                f["step"].add_(1.0)
                self._step_reference(group, f)
        return loss

    @staticmethod
    def _step_reference(group, f) -> None:
        """Same update as the kernel, in torch ops (CPU / fallback)."""
        p, g, m, v = f["flat"], f["grad"], f["m"], f["v"]
        b1, b2 = group["betas"]
        lr, eps, wd = group["lr"], group["eps"], group["weight_decay"]
        t = f["step"]
        gr = -g if group["maximize"] else g.clone()
        if wd != 0.0:
            if group["decoupled_weight_decay"]:
                p.mul_(1.0 - lr * wd)
            else:
                gr.add_(p, alpha=wd)
        m.lerp_(gr, 1.0 - b1)
        v.mul_(b2).addcmul_(gr, gr, value=1.0 - b2)
        step_size = lr / (1.0 - b1**t)
        denom = v.sqrt() / th.sqrt(1.0 - b2**t) + eps
        p.sub_(step_size * (m / denom))
        g.zero_()

    # ------------------------------------------------------------------ checkpoints
    def state_dict(self) -> Dict[str, Any]:
        """torch Adam layout that loads into ``th.optim.Adam`` / ``AdamW`` as-is: every
        parameter gets its OWN scalar ``step`` (the flat group shares one device counter,
        which torch would otherwise increment once per parameter) and the groups say
        ``capturable=False`` (torch refuses a capturable step on CPU parameters)."""
        sd = super().state_dict()
        # (new per-parameter dicts: torch's state_dict hands out the live ``self.state`` dicts, and
        # writing the snapshots into those would detach them from the flat buffers -- every later
        # state_dict would then return this one's step and moments)
        sd["state"] = {i: {k: (th.tensor(float(v), dtype=th.float32) if k == "step" else
                               v.detach().clone() if k in ("exp_avg", "exp_avg_sq") else v)
                           for k, v in st.items()}
                       for i, st in sd["state"].items()}
        sd["param_groups"] = [dict(g, capturable=False) for g in sd["param_groups"]]
        return sd

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        """Load a torch-Adam-layout state and copy it into the flat buffers (the loaded
        tensors would otherwise replace the views)."""
        super().load_state_dict(state_dict)
        for group, f in zip(self.param_groups, self._flat):
            group["capturable"] = True
            for key in ("lr", "eps", "weight_decay", "maximize"):
                group.setdefault(key, self.defaults[key])
            group["betas"] = tuple(group["betas"])
            group.setdefault("decoupled_weight_decay", self.defaults["decoupled_weight_decay"])
            if not f["n"]:
                continue
            steps = []
            with th.no_grad():
                for p, (off, k, _) in zip(f["params"], f["views"]):
                    st = self.state.get(p, {})
                    if "exp_avg" in st:
                        f["m"][off : off + k].copy_(st["exp_avg"].reshape(-1))
                        f["v"][off : off + k].copy_(st["exp_avg_sq"].reshape(-1))
                        steps.append(float(st["step"]))
                    self.state[p] = {"step": f["step"], "exp_avg": f["m"][off : off + k].view_as(p),
                                     "exp_avg_sq": f["v"][off : off + k].view_as(p)}
                f["step"].fill_(max(steps) if steps else 0.0)


class FusedAdamW(FusedAdam):
    """AdamW (decoupled weight decay, default 1e-2 like ``th.optim.AdamW``)."""

    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, **kwargs):
        kwargs.pop("decoupled_weight_decay", None)
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                         decoupled_weight_decay=True, **kwargs)


def fused_for(optimizer_cls, device) -> Optional[type]:
    """The fused replacement of ``optimizer_cls`` on ``device`` (None = keep the given class).
    Exactly ``th.optim.Adam`` / ``th.optim.AdamW`` on a GPU, unless ``IMITATION_AMD_FUSED_ADAM=0``."""
    import os

    if th.device(device).type != "cuda" or os.environ.get("IMITATION_AMD_FUSED_ADAM", "1") == "0":
        return None
    if optimizer_cls is th.optim.Adam:
        return FusedAdam
    if optimizer_cls is th.optim.AdamW:
        return FusedAdamW
    return None


def to_fused(optimizer: th.optim.Optimizer) -> th.optim.Optimizer:
    """Swap a single-group ``th.optim.Adam`` / ``AdamW`` on a GPU for its fused equivalent over
    the same parameters, hyper-parameters and (torch-layout) state; anything else is
    returned unchanged. Call before any graph or kernel descriptor captured the parameters'
    storage (the fused optimiser re-points them into its flat bucket)."""
    if len(optimizer.param_groups) != 1:
        return optimizer
    g = optimizer.param_groups[0]
    params = list(g["params"])
    if not params or g.get("amsgrad", False) or g.get("differentiable", False):
        return optimizer
    cls = fused_for(type(optimizer), params[0].device)
    if cls is None:
        return optimizer
    new = cls(params, lr=g["lr"], betas=g["betas"], eps=g["eps"], weight_decay=g["weight_decay"],
              maximize=g.get("maximize", False))
    if optimizer.state:
        new.load_state_dict(optimizer.state_dict())
    return new

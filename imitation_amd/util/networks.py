"""Neural-network building blocks (reference: ``src/imitation/util/networks.py``).

* :func:`training_mode` / :func:`training` / :func:`evaluating` (``networks.py:12-34``);
* :class:`SqueezeLayer` (``:37-44``);
* :class:`BaseNorm`, :class:`RunningNorm` (Chan et al. parallel merge, ``:98-134``),
  :class:`EMANorm` (batched EMA/EMV, ``:137-201``);
* :func:`build_mlp` (``:204-283``) and :func:`build_cnn` (``:286-357``).

MI355X specifics:

* :func:`build_mlp` returns an :class:`MLP` (an ``nn.Sequential`` with the
  reference's layer names, so state dicts are interchangeable) whose forward on a
  GPU runs the whole stack -- including the RunningNorm/EMANorm prologue -- as
  ONE fused MFMA launch (``csrc/kernels/tmlp.hip``) instead of 2L+1 PyTorch launches.
* Normalisation statistics are data-parallel aware: under an initialised
  process group (``imitation_amd.parallel``) the batch moments are all-reduced
  before the Chan/EMA merge so every replica holds identical stats
  (SURVEY §7.4 item 4).
"""

from __future__ import annotations

import abc
import collections
import contextlib
import functools
from typing import Dict, Iterable, Optional, Type, Union

import torch as th
from torch import nn

from imitation_amd import ops
from imitation_amd.ops.mlp import act_code, fusable


@contextlib.contextmanager
def training_mode(m: nn.Module, mode: bool = False):
    """Temporarily switch module ``m`` to specified training ``mode``."""
    old_mode = m.training
    m.train(mode)
    try:
        yield m
    finally:
        m.train(old_mode)


training = functools.partial(training_mode, mode=True)
evaluating = functools.partial(training_mode, mode=False)


class SqueezeLayer(nn.Module):
    """Torch module that squeezes a B*1 tensor down into a size-B vector."""

    def forward(self, x):
        assert x.ndim == 2 and x.shape[1] == 1
        new_value = x.squeeze(1)
        assert new_value.ndim == 1
        return new_value


def _global_batch_moments(batch: th.Tensor):
    """(mean, biased var, count) of ``batch`` over dim 0, reduced across DP ranks."""
    from imitation_amd.parallel import dist as pdist

    n = batch.shape[0]
    if pdist.norm_sync_active():
        out = pdist.allreduce_moments_device(batch)  # one-shot path: no host sync, capturable
        return out if out is not None else pdist.allreduce_moments(batch)
    return th.mean(batch, dim=0), th.var(batch, dim=0, unbiased=False), n


class BaseNorm(nn.Module, abc.ABC):
    """Normalise inputs to mean 0 / variance 1 with statistics from all batches seen."""

    running_mean: th.Tensor
    running_var: th.Tensor
    count: th.Tensor

    def __init__(self, num_features: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.num_features = num_features
        self.register_buffer("running_mean", th.empty(num_features))
        self.register_buffer("running_var", th.empty(num_features))
        self.register_buffer("count", th.empty((), dtype=th.int))
        BaseNorm.reset_running_stats(self)

    def reset_running_stats(self) -> None:
        """Identity transform: mean 0, var 1, count 0 (``networks.py:73-77``)."""
        self.running_mean.zero_()
        self.running_var.fill_(1)
        self.count.zero_()

    def forward(self, x: th.Tensor) -> th.Tensor:
        if self.training:
            with th.no_grad():
                self.update_stats(x)
        return (x - self.running_mean) / th.sqrt(self.running_var + self.eps)

    @abc.abstractmethod
    def update_stats(self, batch: th.Tensor) -> None:
        """Update ``running_mean``, ``running_var`` and ``count``."""


class RunningNorm(BaseNorm):
    """Running mean/variance normaliser (Chan et al. 1979 pairwise merge).

    On the GPU (2-D fp32 batches, no DP statistics sync) the update and the normalisation run
    as ONE HIP launch (``csrc/kernels/norm.hip``) instead of ~20 elementwise / reduce kernels;
    inputs that need a gradient keep the differentiable torch normalisation."""

    def _fused_ok(self, x: th.Tensor) -> bool:
        from imitation_amd import ops
        from imitation_amd.parallel import dist as pdist

        return (x.dim() == 2 and x.dtype == th.float32 and ops.use_kernel(x) and self.running_mean.is_cuda
                and self.count.dtype == th.int32 and 0 < x.shape[1] <= 256 and 0 < x.shape[0] * x.shape[1] <= (1 << 20)
                and not pdist.norm_sync_active())

    def forward(self, x: th.Tensor) -> th.Tensor:
        if self._fused_ok(x) and not (x.requires_grad and th.is_grad_enabled()):
            from imitation_amd import ops

            return ops.native().running_norm(x.contiguous(), self.running_mean, self.running_var, self.count,
                                             float(self.eps), bool(self.training), True)
        return super().forward(x)

    def update_stats(self, batch: th.Tensor) -> None:
        if self._fused_ok(batch):
            from imitation_amd import ops

            ops.native().running_norm(batch.detach().contiguous(), self.running_mean, self.running_var, self.count,
                                      float(self.eps), True, False)
            return
        batch_mean, batch_var, batch_count = _global_batch_moments(batch)
        delta = batch_mean - self.running_mean
        tot_count = self.count + batch_count
        self.running_mean += delta * batch_count / tot_count
        self.running_var *= self.count
        self.running_var += batch_var * batch_count
        self.running_var += th.square(delta) * self.count * batch_count / tot_count
        self.running_var /= tot_count
        self.count += batch_count


class EMANorm(BaseNorm):
    """Exponentially-weighted running normaliser (``networks.py:137-201``).

    On the GPU (2-D fp32 batches, no DP statistics sync) the update and the normalisation run
    on the RunningNorm kernels (``csrc/kernels/norm.hip``) in their EMA merge mode: the same
    batch moments, then ``lr = 1 / (inv_lr + decay^num_batches)`` and the moving-average
    update of mean / var, the count, ``inv_learning_rate`` and ``num_batches`` advanced on the
    device -- one launch (three for large batches) instead of ~25 elementwise kernels."""

    inv_learning_rate: th.Tensor
    num_batches: th.IntTensor

    def __init__(self, num_features: int, decay: float = 0.99, eps: float = 1e-5):
        super().__init__(num_features, eps=eps)
        if not 0 < decay < 1:
            raise ValueError("decay must be between 0 and 1")
        self.decay = decay
        self.register_buffer("inv_learning_rate", th.empty(()))
        self.register_buffer("num_batches", th.empty((), dtype=th.int))
        EMANorm.reset_running_stats(self)

    def reset_running_stats(self):
        super().reset_running_stats()
        self.inv_learning_rate.zero_()
        self.num_batches.zero_()

    def _fused_ok(self, x: th.Tensor) -> bool:
        return RunningNorm._fused_ok(self, x) and self.num_batches.dtype == th.int32 and self.inv_learning_rate.dtype == th.float32

    def _native(self, x: th.Tensor, update: bool, want_y: bool):
        from imitation_amd import ops

        return ops.native().running_norm(x.contiguous(), self.running_mean, self.running_var, self.count, float(self.eps),
                                         update, want_y, self.inv_learning_rate, self.num_batches, float(self.decay))

    def forward(self, x: th.Tensor) -> th.Tensor:
        if self._fused_ok(x) and not (x.requires_grad and th.is_grad_enabled()):
            return self._native(x, bool(self.training), True)
        return super().forward(x)

    def update_stats(self, batch: th.Tensor) -> None:
        b_size = batch.shape[0]
        if len(batch.shape) == 1:
            batch = batch.reshape(b_size, 1)
        if self._fused_ok(batch):
            self._native(batch.detach(), True, False)
            return
        self.inv_learning_rate += self.decay**self.num_batches
        learning_rate = 1 / self.inv_learning_rate
        batch_mean, batch_var, b_size = _global_batch_moments(batch)
        delta_mean = batch_mean - self.running_mean
        self.running_mean += learning_rate * delta_mean
        delta_var = batch_var + (1 - learning_rate) * delta_mean**2 - self.running_var
        self.running_var += learning_rate * delta_var
        self.count += b_size
        self.num_batches += 1  # type: ignore[misc]


class MLP(nn.Sequential):
    """``nn.Sequential`` MLP that runs as one fused HIP launch on the GPU.

    The module tree (names, parameters, buffers) is exactly what the reference's
    ``build_mlp`` creates, so checkpoints and ``named_parameters`` are identical.
    On CPU (or when the stack has a layer the kernel cannot fuse -- dropout in
    training mode, an exotic activation, widths > 128) it runs layer by layer.
    """

    def _fusion_plan(self):
        plan = getattr(self, "_ia_plan", None)
        if plan is not None:
            return plan
        mods = list(self._modules.values())
        i = 0
        flatten = squeeze = False
        norm = None
        if i < len(mods) and isinstance(mods[i], nn.Flatten):
            flatten, i = True, i + 1
        if i < len(mods) and isinstance(mods[i], BaseNorm):
            norm, i = mods[i], i + 1
        linears, acts = [], []
        while i < len(mods):
            m = mods[i]
            if isinstance(m, nn.Linear):
                if m.bias is None:
                    plan = False
                    break
                linears.append(m)
                acts.append(0)
                i += 1
            elif isinstance(m, nn.Dropout):
                i += 1  # identity in eval mode; training-mode dropout disables fusion at call time
            elif isinstance(m, SqueezeLayer):
                squeeze, i = True, i + 1
            else:
                c = act_code(m)
                if c is None or not linears:
                    plan = False
                    break
                acts[-1] = c
                i += 1
        if plan is not False:
            hid = set(acts[:-1])
            dims = [linears[0].in_features] + [l.out_features for l in linears] if linears else []
            wide = getattr(self, "wide_bf16", None)  # opt-in bf16 wide path (ops/mlp.py)
            if not linears or len(hid) > 1 or not fusable(dims, wide):
                plan = False
            else:
                plan = dict(
                    flatten=flatten,
                    norm=norm,
                    linears=linears,
                    hidden_act=(acts[0] if len(acts) > 1 else 0),
                    out_act=acts[-1],
                    squeeze=squeeze,
                    wide=wide,
                    has_dropout=any(isinstance(m, nn.Dropout) for m in mods),
                )
        object.__setattr__(self, "_ia_plan", plan)
        return plan

    def forward(self, x):
        if x.is_cuda and ops.fused_enabled() and x.dtype == th.float32:
            plan = self._fusion_plan()
            if plan and not (plan["has_dropout"] and self.training):
                h = x.flatten(1) if plan["flatten"] else x
                mean = var = None
                eps = 1e-5
                norm = plan["norm"]
                if norm is not None:
                    if norm.training:
                        with th.no_grad():
                            norm.update_stats(h)
                    mean, var, eps = norm.running_mean, norm.running_var, norm.eps
                lin = plan["linears"]
                y = ops.tmlp(
                    h,
                    [l.weight for l in lin],
                    [l.bias for l in lin],
                    plan["hidden_act"],
                    plan["out_act"],
                    mean,
                    var,
                    eps,
                    plan["wide"],
                )
                if plan["squeeze"]:
                    y = y.squeeze(1)
                return y
        return super().forward(x)


def build_mlp(
    in_size: int,
    hid_sizes: Iterable[int],
    out_size: int = 1,
    name: Optional[str] = None,
    activation: Type[nn.Module] = nn.ReLU,
    dropout_prob: float = 0.0,
    squeeze_output: bool = False,
    flatten_input: bool = False,
    normalize_input_layer: Optional[Type[nn.Module]] = None,
) -> nn.Module:
    """Construct an MLP with the reference's layer naming (``networks.py:204-283``)."""
    layers: Dict[str, nn.Module] = {}
    prefix = "" if name is None else f"{name}_"
    if flatten_input:
        layers[f"{prefix}flatten"] = nn.Flatten()
    if normalize_input_layer:
        try:
            layer_instance = normalize_input_layer(in_size)  # type: ignore[call-arg]
        except TypeError as exc:
            raise ValueError(
                f"normalize_input_layer={normalize_input_layer} is not a valid "
                "normalization layer type accepting only one argument (in_size).",
            ) from exc
        layers[f"{prefix}normalize_input"] = layer_instance
    prev_size = in_size
    for i, size in enumerate(hid_sizes):
        layers[f"{prefix}dense{i}"] = nn.Linear(prev_size, size)
        prev_size = size
        if activation:
            layers[f"{prefix}act{i}"] = activation()
        if dropout_prob > 0.0:
            layers[f"{prefix}dropout{i}"] = nn.Dropout(dropout_prob)
    layers[f"{prefix}dense_final"] = nn.Linear(prev_size, out_size)
    if squeeze_output:
        if out_size != 1:
            raise ValueError("squeeze_output is only applicable when out_size=1")
        layers[f"{prefix}squeeze"] = SqueezeLayer()
    return MLP(collections.OrderedDict(layers))


def build_cnn(
    in_channels: int,
    hid_channels: Iterable[int],
    out_size: int = 1,
    name: Optional[str] = None,
    activation: Type[nn.Module] = nn.ReLU,
    kernel_size: int = 3,
    stride: int = 1,
    padding: Union[int, str] = "same",
    dropout_prob: float = 0.0,
    squeeze_output: bool = False,
) -> nn.Module:
    """Construct a CNN: conv+act stack, global average pool, linear (``networks.py:286-357``)."""
    layers: Dict[str, nn.Module] = {}
    prefix = "" if name is None else f"{name}_"
    prev_channels = in_channels
    for i, n_channels in enumerate(hid_channels):
        layers[f"{prefix}conv{i}"] = nn.Conv2d(prev_channels, n_channels, kernel_size, stride=stride, padding=padding)
        prev_channels = n_channels
        if activation:
            layers[f"{prefix}act{i}"] = activation()
        if dropout_prob > 0.0:
            layers[f"{prefix}dropout{i}"] = nn.Dropout(dropout_prob)
    layers[f"{prefix}avg_pool"] = nn.AdaptiveAvgPool2d(1)
    layers[f"{prefix}flatten"] = nn.Flatten()
    layers[f"{prefix}dense_final"] = nn.Linear(prev_channels, out_size)
    if squeeze_output:
        if out_size != 1:
            raise ValueError("squeeze_output is only applicable when out_size=1")
        layers[f"{prefix}squeeze"] = SqueezeLayer()
    return CNN(collections.OrderedDict(layers))


class CNN(nn.Sequential):
    """``build_cnn``'s module: the same ``nn.Sequential`` (layer names, state dict), whose
    forward on a GPU runs the conv+ReLU stack on the NHWC HIP kernels (``ops.conv.conv_stack``:
    zero-padded ``same`` convs, bf16 operands, fp32 accumulation) followed by the average
    pool and the final linear layer. Other configurations (non-ReLU activations, active
    dropout, even kernels, strides with padding, CPU tensors) run the modules as given."""

    def _fused_plan(self) -> Optional[dict]:
        convs, pads = [], []
        mods = list(self.children())
        i = 0
        while i < len(mods) and isinstance(mods[i], nn.Conv2d):
            c = mods[i]
            if c.groups != 1 or c.dilation != (1, 1) or c.kernel_size[0] != c.kernel_size[1] or c.stride[0] != c.stride[1]:
                return None
            if c.bias is None:
                return None
            if c.padding == "valid":
                p = 0
            elif c.padding == "same":
                if c.kernel_size[0] % 2 == 0 or c.stride[0] != 1:
                    return None
                p = (c.kernel_size[0] - 1) // 2
            elif isinstance(c.padding, tuple) and c.padding[0] == c.padding[1] and c.padding_mode == "zeros":
                p = int(c.padding[0])
            else:
                return None
            if i + 1 >= len(mods) or type(mods[i + 1]) is not nn.ReLU:
                return None
            convs.append(c)
            pads.append(p)
            i += 2
            while i < len(mods) and isinstance(mods[i], nn.Dropout):
                if mods[i].p > 0 and mods[i].training:
                    return None
                i += 1
        rest = mods[i:]
        if not convs or len(rest) not in (3, 4):
            return None
        if not (isinstance(rest[0], nn.AdaptiveAvgPool2d) and rest[0].output_size in (1, (1, 1))
                and isinstance(rest[1], nn.Flatten) and isinstance(rest[2], nn.Linear)):
            return None
        squeeze = len(rest) == 4
        if squeeze and not isinstance(rest[3], SqueezeLayer):
            return None
        return dict(convs=convs, pads=pads, dense=rest[2], squeeze=squeeze)

    def forward(self, x):
        from imitation_amd.ops import conv as conv_ops

        plan = self._fused_plan() if (x.is_cuda and x.dim() == 4 and ops.use_kernel(x)) else None
        if plan is not None:
            convs = plan["convs"]
            x_nhwc = x.float().permute(0, 2, 3, 1)  # a view when x is channels_last
            ws = [c.weight for c in convs]
            if conv_ops.supported(tuple(x_nhwc.shape), ws, [c.stride[0] for c in convs], plan["pads"]):
                h = conv_ops.conv_stack(x_nhwc, ws, [c.bias for c in convs], [c.stride[0] for c in convs], 1.0,
                                        plan["pads"], out_dtype=th.bfloat16)
                pooled = h.mean(dim=(1, 2), dtype=th.float32)
                out = nn.functional.linear(pooled, plan["dense"].weight, plan["dense"].bias)
                return out.squeeze(1) if plan["squeeze"] else out
        return super().forward(x)

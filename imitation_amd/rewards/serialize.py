"""Load serialized reward functions by type key (reference: src/imitation/rewards/serialize.py).

Reward nets are written by :func:`save_reward_net` (tensor-only; see
``imitation_amd.util.module_spec``) and loaded with ``weights_only=True``. Registry
keys and wrapper semantics match the reference:

* ``RewardNet_shaped``     -- net must be a ShapedRewardNet; ``predict``
* ``RewardNet_unshaped``   -- strips a ShapedRewardNet wrapper; ``predict``
* ``RewardNet_normalized`` -- net must be a NormalizedRewardNet; ``predict_processed(update_stats=False)``
* ``RewardNet_unnormalized`` -- strips NormalizedRewardNet; ``predict``
* ``RewardNet_std_added``  -- AddSTDRewardWrapper (optionally under NormalizedRewardNet); ``predict_processed``
* ``zero``                 -- constant 0
"""

from __future__ import annotations

from typing import Any, Callable, Dict, Iterable, Optional, Sequence, Type, Union, cast

import numpy as np
import torch as th

from imitation_amd.rewards import reward_function, reward_nets
from imitation_amd.util import module_spec, registry

RewardFnLoaderFn = Callable[..., reward_function.RewardFn]
reward_registry: registry.Registry[RewardFnLoaderFn] = registry.Registry()


def save_reward_net(net: reward_nets.RewardNet, path) -> None:
    module_spec.save_module(net, path)


def load_reward_net(path, device: Union[str, th.device, None] = None) -> reward_nets.RewardNet:
    net = module_spec.load_module(path, map_location=device)
    assert isinstance(net, reward_nets.RewardNet)
    return cast(reward_nets.RewardNet, net)


class ValidateRewardFn(reward_function.RewardFn):
    """Checks that the reward vector has one entry per input transition."""

    def __init__(self, reward_fn: reward_function.RewardFn) -> None:
        super().__init__()
        self.reward_fn = reward_fn

    def __call__(self, state, action, next_state, done) -> np.ndarray:
        rew = self.reward_fn(state, action, next_state, done)
        assert rew.shape == (len(state),)
        return rew


def _strip_wrappers(net: reward_nets.RewardNet, wrapper_types: Iterable[Type[reward_nets.RewardNetWrapper]]):
    for wt in wrapper_types:
        assert issubclass(wt, reward_nets.RewardNetWrapper), f"trying to remove non-wrapper type {wt}"
        if isinstance(net, wt):
            net = net.base
        else:
            break
    return net


def _make_functional(net, attr: str = "predict", default_kwargs: Optional[Dict[str, Any]] = None, **kwargs):
    default_kwargs = dict(default_kwargs or {})
    default_kwargs.update(kwargs)
    return lambda *args: getattr(net, attr)(*args, **default_kwargs)


def _prefix_matches(wrappers: Sequence[type], prefix: Sequence[type]) -> bool:
    if len(prefix) == 0:
        return True
    if len(wrappers) == 0:
        return False
    return issubclass(wrappers[0], prefix[0]) and _prefix_matches(wrappers[1:], prefix[1:])


def _validate_wrapper_structure(net, prefixes: Iterable[Sequence[type]]):
    """Return ``net`` if its wrapper chain (outermost first) starts with one of ``prefixes``."""
    chain = []
    w = net
    while hasattr(w, "base"):
        chain.append(type(w))
        w = w.base
    chain.append(type(w))
    prefixes = list(prefixes)
    if any(_prefix_matches(chain, p) for p in prefixes):
        return net
    fmt = " or ".join("[" + ",".join(t.__name__ for t in p) + "]" for p in prefixes)
    raise TypeError(f"Wrapper structure should match {fmt} but found [" + ",".join(t.__name__ for t in chain) + "]")


def load_zero(path: str, venv) -> reward_function.RewardFn:
    del path, venv

    def f(state, action, next_state, done) -> np.ndarray:
        return np.zeros(np.shape(state)[0])

    return f


reward_registry.register(
    key="RewardNet_shaped",
    value=lambda path, _, **kw: ValidateRewardFn(
        _make_functional(_validate_wrapper_structure(load_reward_net(path), {(reward_nets.ShapedRewardNet,)}))),
)
reward_registry.register(
    key="RewardNet_unshaped",
    value=lambda path, _, **kw: ValidateRewardFn(
        _make_functional(_strip_wrappers(load_reward_net(path), (reward_nets.ShapedRewardNet,)))),
)
reward_registry.register(
    key="RewardNet_normalized",
    value=lambda path, _, **kw: ValidateRewardFn(
        _make_functional(_validate_wrapper_structure(load_reward_net(path), {(reward_nets.NormalizedRewardNet,)}),
                         attr="predict_processed", default_kwargs={"update_stats": False}, **kw)),
)
reward_registry.register(
    key="RewardNet_unnormalized",
    value=lambda path, _, **kw: ValidateRewardFn(
        _make_functional(_strip_wrappers(load_reward_net(path), (reward_nets.NormalizedRewardNet,)))),
)
reward_registry.register(
    key="RewardNet_std_added",
    value=lambda path, _, **kw: ValidateRewardFn(
        _make_functional(
            _strip_wrappers(
                _validate_wrapper_structure(
                    load_reward_net(path),
                    {(reward_nets.AddSTDRewardWrapper,), (reward_nets.NormalizedRewardNet, reward_nets.AddSTDRewardWrapper)},
                ),
                (reward_nets.NormalizedRewardNet,),
            ),
            attr="predict_processed", default_kwargs={}, **kw)),
)
reward_registry.register(key="zero", value=load_zero)


def load_reward(reward_type: str, reward_path: str, venv, **kwargs) -> reward_function.RewardFn:
    """Load reward ``reward_type`` stored at ``reward_path``."""
    reward_loader = reward_registry.get(reward_type)
    return reward_loader(reward_path, venv, **kwargs)

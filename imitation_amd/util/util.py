"""Miscellaneous utilities (reference: ``src/imitation/util/util.py``).

``make_vec_env`` (``util.py:80-166``) keeps the reference's contract (per-env
non-sequential seeds from ``make_seeds``, Monitor, optional ``log_dir``
monitor CSVs, ``post_wrappers``, Dummy vs Subproc) but, for every built-in env
id, returns a :class:`~imitation_amd.envs.vec_env.NativeVecEnv`: all of the
rank's envs in one C++ SoA block stepped by a single call, instead of one Python
env object per env behind pipes. ``post_wrappers`` that need a per-env Python
object fall back to the Dummy/Subproc path, except ``RolloutInfoWrapper``,
which maps onto the equivalent vectorised wrapper.
"""

from __future__ import annotations

import datetime
import functools
import itertools
import os
import pathlib
import uuid
import warnings
from typing import Any, Callable, Iterable, Iterator, List, Mapping, Optional, Sequence, Tuple, TypeVar, Union

import numpy as np
import torch as th

from imitation_amd.data.types import AnyPath
from imitation_amd.envs import core as env_core
from imitation_amd.envs.vec_env import DummyVecEnv, Monitor, NativeVecEnv, SubprocVecEnv, VecEnv


def save_policy(policy, policy_path: AnyPath) -> None:
    """Save a policy (``final.th`` in the CLI) as a tensor-only file (see ``BaseModel.save``)."""
    policy.save(parse_path(policy_path))


def oric(x: np.ndarray) -> np.ndarray:
    """Optimal rounding under integer constraints (keeps the sum)."""
    rounded = np.floor(x)
    shortfall = x - rounded
    total_shortfall = np.round(shortfall.sum()).astype(int)
    indices = np.argsort(-shortfall)
    rounded[indices[:total_shortfall]] += 1
    return rounded.astype(int)


def make_unique_timestamp() -> str:
    timestamp = datetime.datetime.now().strftime("%Y%m%d_%H%M%S")
    return f"{timestamp}_{uuid.uuid4().hex[:6]}"


def _native_id(env_name: str) -> Optional[str]:
    try:
        spec = env_core.spec(env_name)
    except Exception:
        return None
    return getattr(spec, "native_id", None) or (spec.kwargs.get("native_id") if getattr(spec, "kwargs", None) else None)


class _ProbeEnv(env_core.Env):
    """Stand-in env used to recognise ``lambda e, i: RolloutInfoWrapper(e)`` post-wrappers."""

    def __init__(self):
        from imitation_amd.envs import spaces

        self.observation_space = spaces.Discrete(1)
        self.action_space = spaces.Discrete(1)

    def reset(self, *, seed=None, options=None):  # pragma: no cover
        return 0, {}

    def step(self, action):  # pragma: no cover
        return 0, 0.0, False, False, {}


def _is_rollout_info_wrapper(w) -> bool:
    """True if post-wrapper ``w`` only adds RolloutInfoWrapper (the native VecEnv then
    gets the batched VecRolloutInfoWrapper instead of per-env Python wrappers)."""
    from imitation_amd.data.wrappers import RolloutInfoWrapper

    if w is RolloutInfoWrapper or getattr(w, "_imitation_amd_rollout_info", False):
        return True
    if isinstance(w, functools.partial) and w.func is RolloutInfoWrapper:
        return True
    try:
        probe = _ProbeEnv()
        out = w(probe, 0)
    except Exception:
        return False
    return type(out) is RolloutInfoWrapper and out.env is probe


def make_vec_env(
    env_name: str,
    *,
    rng: np.random.Generator,
    n_envs: int = 8,
    parallel: bool = False,
    log_dir: Optional[str] = None,
    max_episode_steps: Optional[int] = None,
    post_wrappers: Optional[Sequence[Callable[[env_core.Env, int], env_core.Env]]] = None,
    env_make_kwargs: Optional[Mapping[str, Any]] = None,
) -> VecEnv:
    """Make a VecEnv of ``n_envs`` copies of ``env_name`` with per-env seeds from ``rng``."""
    from imitation_amd.data.wrappers import RolloutInfoWrapper, VecRolloutInfoWrapper

    env_seeds = make_seeds(rng, n_envs)
    env_make_kwargs = dict(env_make_kwargs or {})
    native = _native_id(env_name)
    wrappers = list(post_wrappers or [])
    is_info = [_is_rollout_info_wrapper(w) for w in wrappers]
    rollout_info = any(is_info)
    other_wrappers = [w for w, f in zip(wrappers, is_info) if not f]
    if native is not None and not other_wrappers and not env_make_kwargs:
        mon_dir = os.path.join(log_dir, "monitor") if log_dir is not None else None
        venv: VecEnv = NativeVecEnv(native, n_envs, seed=env_seeds[0], max_episode_steps=max_episode_steps, log_dir=mon_dir)
        venv.seed_envs(env_seeds)
        if rollout_info:
            venv = VecRolloutInfoWrapper(venv)
        return venv

    spec = env_core.spec(env_name)

    def make_env(i: int, this_seed: int) -> env_core.Env:
        env = env_core.make(spec, max_episode_steps=max_episode_steps, **env_make_kwargs)
        env.reset(seed=int(this_seed))
        log_path = None
        if log_dir is not None:
            log_subdir = os.path.join(log_dir, "monitor")
            os.makedirs(log_subdir, exist_ok=True)
            log_path = os.path.join(log_subdir, f"mon{i:03d}")
        env = Monitor(env, log_path)
        for wrapper in wrappers:
            env = wrapper(env, i)
        return env

    env_fns = [functools.partial(make_env, i, s) for i, s in enumerate(env_seeds)]
    if parallel:
        return SubprocVecEnv(env_fns, start_method="forkserver")
    return DummyVecEnv(env_fns)


def make_seeds(rng: np.random.Generator, n: Optional[int] = None) -> Union[Sequence[int], int]:
    """Draw ``n`` (or one) non-sequential seeds from ``rng``."""
    seeds = rng.integers(0, (1 << 31) - 1, (n if n is not None else 1,)).tolist()
    return seeds[0] if n is None else seeds


def docstring_parameter(*args, **kwargs):
    def helper(obj):
        obj.__doc__ = obj.__doc__.format(*args, **kwargs)
        return obj

    return helper


T = TypeVar("T")


def endless_iter(iterable: Iterable[T]) -> Iterator[T]:
    """Cycle a re-iterable forever (raises on a one-shot iterator)."""
    if iter(iterable) == iterable:
        raise ValueError("endless_iter needs a non-iterator Iterable.")
    _, iterable = get_first_iter_element(iterable)
    return itertools.chain.from_iterable(itertools.repeat(iterable))


def safe_to_tensor(array, **kwargs) -> th.Tensor:
    if isinstance(array, th.Tensor):
        return th.as_tensor(array, **kwargs)
    array = np.asarray(array)
    if not array.flags.writeable:
        array = array.copy()
    return th.as_tensor(array, **kwargs)


def safe_to_numpy(obj, warn: bool = False):
    if obj is None:
        return None
    if isinstance(obj, np.ndarray):
        return obj
    if warn:
        warnings.warn("Converted tensor to numpy array, might affect performance. Make sure this is the intended behavior.")
    return obj.detach().cpu().numpy()


def to_numpy(obj) -> np.ndarray:
    if isinstance(obj, th.Tensor):
        return obj.detach().cpu().numpy()
    return np.asarray(obj)


def tensor_iter_norm(tensor_iter: Iterable[th.Tensor], ord: Union[int, float] = 2) -> th.Tensor:  # noqa: A002
    if ord == 0:
        raise ValueError("This function cannot compute p-norms for p=0.")
    norms = [th.norm(t.flatten(), p=ord) for t in tensor_iter]
    return th.norm(th.stack(norms) if norms else th.zeros(0), p=ord)


def get_first_iter_element(iterable: Iterable[T]) -> Tuple[T, Iterable[T]]:
    iterator = iter(iterable)
    try:
        first = next(iterator)
    except StopIteration:
        raise ValueError(f"iterable {iterable} had no elements to iterate over.")
    if iterator == iterable:
        return first, itertools.chain([first], iterator)
    return first, iterable


def parse_path(path: AnyPath, allow_relative: bool = True, base_directory: Optional[pathlib.Path] = None) -> pathlib.Path:
    if base_directory is not None and not allow_relative:
        raise ValueError("If `base_directory` is specified, then `allow_relative` must be True.")
    if isinstance(path, pathlib.Path):
        parsed = path
    elif isinstance(path, str):
        parsed = pathlib.Path(path)
    elif isinstance(path, bytes):
        parsed = pathlib.Path(path.decode())
    else:
        parsed = pathlib.Path(str(path))
    if parsed.is_absolute():
        return parsed
    if allow_relative:
        return (base_directory or pathlib.Path.cwd()) / parsed
    raise ValueError(f"Path {str(parsed)} is not absolute")


def parse_optional_path(path: Optional[AnyPath], allow_relative: bool = True, base_directory: Optional[pathlib.Path] = None):
    return None if path is None else parse_path(path, allow_relative, base_directory)


def split_in_half(x: int) -> Tuple[int, int]:
    half = x // 2
    return half, x - half


def clear_screen() -> None:
    os.system("cls" if os.name == "nt" else "clear")

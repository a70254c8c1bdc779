"""Single-environment API (gymnasium-compatible semantics) and env registry.

The reference uses ``gymnasium`` envs (``reset(seed=...) -> (obs, info)``,
5-tuple ``step``) created through ``gym.make`` with ``TimeLimit``
(``src/imitation/util/util.py:80-166`` ``make_vec_env``;
``scripts/ingredients/environment.py:26-69``). This module provides the same
surface natively: :class:`Env`, :class:`Wrapper` family, :class:`TimeLimit`,
:class:`EnvSpec`, and a registry with :func:`make` / :func:`register` /
:func:`spec`.
"""

from __future__ import annotations

import copy
import dataclasses
import importlib
from typing import Any, Callable, Dict, Optional, SupportsFloat, Tuple, Union

import numpy as np

from imitation_amd.envs import spaces


@dataclasses.dataclass
class EnvSpec:
    id: str
    entry_point: Union[str, Callable[..., "Env"]]
    max_episode_steps: Optional[int] = None
    kwargs: Dict[str, Any] = dataclasses.field(default_factory=dict)
    reward_threshold: Optional[float] = None
    nondeterministic: bool = False
    # Native batched implementation name (csrc/runtime/envs.h) if one exists.
    native_id: Optional[str] = None

    def make(self, **kwargs) -> "Env":
        return make(self.id, **kwargs)


class Env:
    """Base class for environments (gymnasium ``Env`` semantics)."""

    metadata: Dict[str, Any] = {"render_modes": []}
    render_mode: Optional[str] = None
    spec: Optional[EnvSpec] = None
    observation_space: spaces.Space
    action_space: spaces.Space
    reward_range = (-float("inf"), float("inf"))
    _np_random: Optional[np.random.Generator] = None

    @property
    def np_random(self) -> np.random.Generator:
        if self._np_random is None:
            self._np_random = np.random.default_rng()
        return self._np_random

    @np_random.setter
    def np_random(self, value):
        self._np_random = value

    def reset(self, *, seed: Optional[int] = None, options: Optional[dict] = None) -> Tuple[Any, dict]:
        if seed is not None:
            self._np_random = np.random.default_rng(seed)
        return None, {}

    def step(self, action) -> Tuple[Any, SupportsFloat, bool, bool, dict]:  # pragma: no cover
        raise NotImplementedError

    def render(self):
        return None

    def close(self):
        pass

    @property
    def unwrapped(self) -> "Env":
        return self

    def get_wrapper_attr(self, name: str):
        return getattr(self, name)

    def __str__(self):
        return f"<{type(self).__name__}<{self.spec.id if self.spec else ''}>>"

    def __enter__(self):
        return self

    def __exit__(self, *args):
        self.close()
        return False


class Wrapper(Env):
    def __init__(self, env: Env):
        self.env = env
        self._action_space: Optional[spaces.Space] = None
        self._observation_space: Optional[spaces.Space] = None

    @property
    def action_space(self):
        return self._action_space if self._action_space is not None else self.env.action_space

    @action_space.setter
    def action_space(self, space):
        self._action_space = space

    @property
    def observation_space(self):
        return self._observation_space if self._observation_space is not None else self.env.observation_space

    @observation_space.setter
    def observation_space(self, space):
        self._observation_space = space

    @property
    def spec(self):
        return self.env.spec

    @property
    def metadata(self):
        return self.env.metadata

    @property
    def render_mode(self):
        return self.env.render_mode

    @property
    def np_random(self):
        return self.env.np_random

    @np_random.setter
    def np_random(self, value):
        self.env.np_random = value

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def get_wrapper_attr(self, name: str):
        if name in self.__dict__ or hasattr(type(self), name):
            return getattr(self, name)
        return self.env.get_wrapper_attr(name)

    def reset(self, *, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        return self.env.step(action)

    def render(self):
        return self.env.render()

    def close(self):
        return self.env.close()

    @property
    def unwrapped(self):
        return self.env.unwrapped

    def __str__(self):
        return f"<{type(self).__name__}{self.env}>"


class ObservationWrapper(Wrapper):
    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self.observation(obs), info

    def step(self, action):
        obs, rew, term, trunc, info = self.env.step(action)
        return self.observation(obs), rew, term, trunc, info

    def observation(self, obs):  # pragma: no cover
        raise NotImplementedError


class RewardWrapper(Wrapper):
    def step(self, action):
        obs, rew, term, trunc, info = self.env.step(action)
        return obs, self.reward(rew), term, trunc, info

    def reward(self, reward):  # pragma: no cover
        raise NotImplementedError


class ActionWrapper(Wrapper):
    def step(self, action):
        return self.env.step(self.action(action))

    def action(self, action):  # pragma: no cover
        raise NotImplementedError


class TimeLimit(Wrapper):
    """Truncate episodes after ``max_episode_steps`` steps."""

    def __init__(self, env: Env, max_episode_steps: int):
        super().__init__(env)
        self._max_episode_steps = int(max_episode_steps)
        self._elapsed_steps: Optional[int] = None

    def step(self, action):
        obs, rew, term, trunc, info = self.env.step(action)
        self._elapsed_steps += 1
        if self._elapsed_steps >= self._max_episode_steps:
            trunc = True
        return obs, rew, term, trunc, info

    def reset(self, *, seed=None, options=None):
        self._elapsed_steps = 0
        return self.env.reset(seed=seed, options=options)


class ClipAction(ActionWrapper):
    def action(self, action):
        return np.clip(action, self.action_space.low, self.action_space.high)


class FlattenObservation(ObservationWrapper):
    def __init__(self, env):
        super().__init__(env)
        n = spaces.flatdim(env.observation_space)
        self.observation_space = spaces.Box(-np.inf, np.inf, (n,), np.float32)

    def observation(self, obs):
        return spaces.flatten(self.env.observation_space, obs).astype(np.float32)


# --------------------------------------------------------------------------- registry
registry: Dict[str, EnvSpec] = {}


def register(
    id: str,
    entry_point: Union[str, Callable[..., Env]],
    max_episode_steps: Optional[int] = None,
    native_id: Optional[str] = None,
    **kwargs,
) -> None:
    registry[id] = EnvSpec(
        id=id,
        entry_point=entry_point,
        max_episode_steps=max_episode_steps,
        native_id=native_id,
        kwargs=kwargs.pop("kwargs", {}) | kwargs,
    )


def _resolve_entry(entry_point):
    if callable(entry_point):
        return entry_point
    mod, _, attr = entry_point.partition(":")
    return getattr(importlib.import_module(mod), attr)


def spec(env_id: str) -> EnvSpec:
    _ensure_builtin()
    if env_id not in registry:
        # allow "module:EnvId" style like gymnasium, importing the module first
        if ":" in env_id:
            mod, _, name = env_id.partition(":")
            importlib.import_module(mod)
            env_id = name
        if env_id not in registry:
            raise KeyError(f"No registered env with id: {env_id}")
    return registry[env_id]


def make(env_id: Union[str, EnvSpec], max_episode_steps: Optional[int] = None, **kwargs) -> Env:
    """Create an environment from the registry, wrapped in :class:`TimeLimit`."""
    env_spec = env_id if isinstance(env_id, EnvSpec) else spec(env_id)
    ctor = _resolve_entry(env_spec.entry_point)
    all_kwargs = dict(env_spec.kwargs)
    all_kwargs.update(kwargs)
    env = ctor(**all_kwargs)
    sp = copy.copy(env_spec)
    sp.kwargs = all_kwargs
    steps = max_episode_steps if max_episode_steps is not None else env_spec.max_episode_steps
    sp.max_episode_steps = steps
    env.unwrapped.spec = sp
    if steps is not None:
        env = TimeLimit(env, steps)
    return env


_BUILTIN_DONE = False


def _ensure_builtin():
    global _BUILTIN_DONE
    if not _BUILTIN_DONE:
        _BUILTIN_DONE = True
        from imitation_amd.envs import registration  # noqa: F401  (registers built-in envs)

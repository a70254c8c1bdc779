"""Vectorized environment ingredient (reference: scripts/ingredients/environment.py).

Built-in env ids map to the native batched C++ runtime (``NativeVecEnv``); ``parallel``
then has no effect (the runtime is already batched and multi-threaded).
"""

import contextlib
from typing import Any, Generator, Mapping

import numpy as np

from imitation_amd.data import wrappers
from imitation_amd.scripts.config_engine import Ingredient
from imitation_amd.util import util

environment_ingredient = Ingredient("environment")


@environment_ingredient.config
def config():
    num_vec = 8  # number of environments in VecEnv
    parallel = True  # Use SubprocVecEnv rather than DummyVecEnv (Python envs only)
    max_episode_steps = None  # Set to positive int to limit episode horizons
    env_make_kwargs = {}  # The kwargs passed to `spec.make`.
    gym_id = "seals/CartPole-v0"  # The environment to train on
    locals()


@contextlib.contextmanager
@environment_ingredient.capture
def make_venv(gym_id: str, num_vec: int, parallel: bool, max_episode_steps: int, env_make_kwargs: Mapping[str, Any],
              _run, _rnd: np.random.Generator, **kwargs) -> Generator:
    log_dir = _run.config["logging"]["log_dir"] if "logging" in _run.config else None
    venv = util.make_vec_env(gym_id, rng=_rnd, n_envs=num_vec, parallel=parallel, max_episode_steps=max_episode_steps,
                             log_dir=str(log_dir) if log_dir is not None else None, env_make_kwargs=env_make_kwargs,
                             **kwargs)
    try:
        yield venv
    finally:
        venv.close()


@contextlib.contextmanager
@environment_ingredient.capture
def make_rollout_venv(gym_id: str, num_vec: int, parallel: bool, max_episode_steps: int,
                      env_make_kwargs: Mapping[str, Any], _rnd: np.random.Generator) -> Generator:
    """No logging; RolloutInfoWrapper applied (for expert rollouts)."""
    venv = util.make_vec_env(gym_id, rng=_rnd, n_envs=num_vec, parallel=parallel, max_episode_steps=max_episode_steps,
                             log_dir=None, env_make_kwargs=env_make_kwargs,
                             post_wrappers=[lambda env, i: wrappers.RolloutInfoWrapper(env)])
    try:
        yield venv
    finally:
        venv.close()


@environment_ingredient.named_config
def fast():
    num_vec = 2
    parallel = False
    max_episode_steps = 5
    locals()

"""Built-in environment registrations.

Mirrors the env ids the reference's configs name (``scripts/ingredients/environment.py``,
``scripts/config/*`` named configs: cartpole, seals_cartpole, pendulum,
mountain_car, seals_half_cheetah, seals_hopper, seals_walker, seals_swimmer,
seals_ant, Pong). Every built-in id is backed by the native batched
implementation (``csrc/include/ia/envs.h``); see that header for which are
exact (classic control) and which are synthetic stand-ins (MuJoCo, Atari).
"""

from __future__ import annotations

import functools

from imitation_amd.envs import core, tabular, toy_text  # noqa: F401  (toy_text registers FrozenLake)

_NATIVE_IDS = {
    "CartPole-v0": 200,
    "CartPole-v1": 500,
    "seals/CartPole-v0": 500,
    "Pendulum-v1": 200,
    "MountainCar-v0": 200,
    "seals/MountainCar-v0": 200,
    "Acrobot-v1": 500,
    "seals/HalfCheetah-v0": 1000,
    "seals/HalfCheetah-v1": 1000,
    "HalfCheetah-v4": 1000,
    "seals/Hopper-v0": 1000,
    "seals/Hopper-v1": 1000,
    "Hopper-v4": 1000,
    "seals/Walker2d-v0": 1000,
    "seals/Walker2d-v1": 1000,
    "Walker2d-v4": 1000,
    "seals/Swimmer-v0": 1000,
    "seals/Swimmer-v1": 1000,
    "Swimmer-v4": 1000,
    "seals/Ant-v0": 1000,
    "seals/Ant-v1": 1000,
    "Ant-v4": 1000,
    "PongNoFrameskip-v4": 27000,
    "ALE/Pong-v5": 27000,
    "Pong-synthetic-v0": 27000,
}

# Environments with a fixed horizon (seals): episodes never terminate early.
FIXED_HORIZON_IDS = {k for k in _NATIVE_IDS if k.startswith("seals/")}


def _make_native(native_id: str):
    from imitation_amd.envs.vec_env import NativeEnv

    return NativeEnv(native_id)


for _id, _steps in _NATIVE_IDS.items():
    core.register(_id, entry_point=functools.partial(_make_native, _id), max_episode_steps=_steps, native_id=_id)

core.register("seals/RandomTransition-v0", entry_point=tabular.RandomTransitionEnv)
core.register(
    "seals/Random-v0",
    entry_point=functools.partial(tabular.RandomTransitionEnv, n_states=16, n_actions=3, branch_factor=2, horizon=20,
                                  random_obs=True, obs_dim=5, generator_seed=42),
)
core.register("seals/CliffWorld-v0", entry_point=tabular.CliffWorld)

"""Environment layer: spaces, single-env API, vectorized envs, native batched envs."""

from imitation_amd.envs import spaces
from imitation_amd.envs.core import (
    ActionWrapper,
    ClipAction,
    Env,
    EnvSpec,
    FlattenObservation,
    ObservationWrapper,
    RewardWrapper,
    TimeLimit,
    Wrapper,
    make,
    register,
    registry,
    spec,
)
from imitation_amd.envs.vec_env import (
    DummyVecEnv,
    Monitor,
    NativeEnv,
    NativeVecEnv,
    SubprocVecEnv,
    VecEnv,
    VecEnvWrapper,
    VecNormalize,
)

__all__ = [
    "spaces",
    "Env",
    "EnvSpec",
    "Wrapper",
    "ObservationWrapper",
    "RewardWrapper",
    "ActionWrapper",
    "TimeLimit",
    "ClipAction",
    "FlattenObservation",
    "make",
    "register",
    "registry",
    "spec",
    "VecEnv",
    "VecEnvWrapper",
    "DummyVecEnv",
    "SubprocVecEnv",
    "NativeVecEnv",
    "NativeEnv",
    "Monitor",
    "VecNormalize",
]
